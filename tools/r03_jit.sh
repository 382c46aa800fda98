#!/bin/bash
# Round 3: one-round stream grids (640x480 4:4:4): priority by frames left with and without start jitter.
mkdir -p gpurun_out/jit && export TMPDIR=/tmp
O=gpurun_out/jit
for run in 1 2; do
  PROBE_R03=1 PROBE_GOP=24 PROBE_OPT=1 PROBE_DELTAS=1 PROBE_WARM_S=1.5 timeout -k 10 240 ./tools/probe 444 640 480 300 200 > $O/opt_444_640_$run.log 2>&1 || { cat $O/opt_444_640_$run.log; exit 1; }
  echo "== run $run"; grep -E "gop<" $O/opt_444_640_$run.log | grep -v "vs production"
done
echo "r03_jit done"
