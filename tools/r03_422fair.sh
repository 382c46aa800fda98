#!/bin/bash
# Round 3: 4:2:2 stream kernels (production exact, optimistic, each with priority by frames left), two runs.
mkdir -p gpurun_out/422fair && export TMPDIR=/tmp
O=gpurun_out/422fair
for run in 1 2; do
  for m in "422 7680 4320 15 60" "422 1920 1080 300 60"; do
    set -- $m
    PROBE_R03=1 PROBE_GOP=24 PROBE_OPT=1 PROBE_DELTAS=1 PROBE_WARM_S=1.5 timeout -k 10 240 ./tools/probe $m > $O/opt_$1_$2_$run.log 2>&1 || { cat $O/opt_$1_$2_$run.log; exit 1; }
    echo "== $1 $2x$3 run $run"; grep -E "gop<" $O/opt_$1_$2_$run.log | grep -v "vs production"
  done
done
echo "r03_422fair done"
