#!/bin/bash
# Round 6: kernel trace of the whole-file decode of a reference-encoded file (tools/real_mpg.py) at
# $ITERS_LIST synchronisation iterations: per-kernel time per pass.
set -o pipefail
O=gpurun_out/r06/real_trace; mkdir -p $O && export TMPDIR=/tmp
P=mjpeg423-video-decoder-software_amd/libmj423gpu.so
F=${F:-clean}
for it in ${ITERS_LIST:-10 4}; do
  AB_FILE=realdata/${F}_1080p.mpg timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_${F}_$it -o kt --output-format csv -- \
    python tools/ab_file.py 1 -- $P@MJ423_GPU_FE_ITERS=$it > $O/kt_${F}_$it.log 2>&1 || { echo STOP kt $it; tail -5 $O/kt_${F}_$it.log; exit 1; }
  f=$(find $O/kt_${F}_$it -name "kt_kernel_trace.csv" | head -1)
  python - "$f" "$it" <<'PY' | tee $O/summary_${F}_$it.txt
import collections, csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = collections.defaultdict(float); cnt = collections.Counter()
for r in rows:
    n = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("mj423::", "").replace("(anonymous namespace)::", "")
    tot[n] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6; cnt[n] += 1
passes = 10
print("iters", sys.argv[2])
for k, v in sorted(tot.items(), key=lambda kv: -kv[1]):
    print(f"{k[:50]:50s} {v / passes:8.4f} ms/pass  {cnt[k] / passes:5.1f} launches/pass")
PY
done
