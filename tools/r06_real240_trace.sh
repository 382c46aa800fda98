#!/bin/bash
# Round 6: kernel trace of bench.py --mode file on the 240-frame reference-encoded clean scene.
set -o pipefail
O=gpurun_out/r06/real240_trace; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python bench.py --mode file --frontend gpu --mpg realdata/clean_1080p_240.mpg --steps 10 --warmup 2 --no-cpu --no-verify > $O/kt.log 2>&1 || { echo STOP kt; tail -5 $O/kt.log; exit 1; }
f=$(find $O/kt -name "kt_kernel_trace.csv" | head -1)
python - "$f" <<'PY' | tee $O/summary.txt
import collections, csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = collections.defaultdict(float); cnt = collections.Counter()
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mj423::", "").replace("(anonymous namespace)::", "")
    tot[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6; cnt[n] += 1
passes = 12
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"{k[:50]:50s} {v / passes:8.4f} ms/pass  {cnt[k] / passes:5.1f} launches/pass")
PY
