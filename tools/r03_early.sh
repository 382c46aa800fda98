#!/bin/bash
# Round 3: 4:2:0 stream kernel with the next frame's loads issued before the IDCT (kGopEarly, as 4:2:2 /
# 4:4:4 do) against production (after the IDCT), after the prefetch-liveness fix; two processes per size.
mkdir -p gpurun_out/early && export TMPDIR=/tmp
O=gpurun_out/early
for run in 1 2; do
for m in "420 3840 2160 300 50" "420 1920 1080 300 100"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_OPT=1 PROBE_EARLY420=1 PROBE_DELTAS=1 PROBE_WARM_S=1.0 timeout -k 10 240 ./tools/probe $m > $O/early_$2_$run.log 2>&1 || { cat $O/early_$2_$run.log; exit 1; }
  echo "== $2x$3 run $run"; grep -E "gop<|vs production" $O/early_$2_$run.log | grep -E "median|differing [1-9]"
done
done
echo "r03_early done"
