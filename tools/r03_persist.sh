#!/bin/bash
# Round 3: is the stream kernel's gap to the batch kernel the loop itself?  The batch kernel one-shot
# against persistent (each workgroup loops over tiles, grid stride or XCD eighths), with the stream
# kernel beside them, one process; then the whole-file paths at 1080p with fair priority on/off.
mkdir -p gpurun_out/persist && export TMPDIR=/tmp
O=gpurun_out/persist
for m in "420 3840 2160 300 20" "420 1920 1080 300 60"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_PERSIST=1 PROBE_DELTAS=1 PROBE_WARM_S=1.5 timeout -k 10 240 ./tools/probe $m > $O/persist_$1_$2.log 2>&1 || { cat $O/persist_$1_$2.log; exit 1; }
  echo "== $1 $2x$3"; grep -E "decode<|gop<" $O/persist_$1_$2.log
done
for fe in host gpu; do
  for fair in auto 0; do
    e=""; [ $fair != auto ] && e="MJ423_GOP_FAIR=$fair"
    env $e timeout -k 10 300 python bench.py --mode file --config f2 --frontend $fe --sink device > $O/f2_${fe}_fair$fair.json 2>$O/f2_${fe}_fair$fair.err || { tail -3 $O/f2_${fe}_fair$fair.err; exit 1; }
    echo "f2 $fe fair=$fair $(python -c "import json; d=json.loads(open('$O/f2_${fe}_fair$fair.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['parity_verified'], d['config']['chunks'])")"
  done
done
echo "r03_persist done"
