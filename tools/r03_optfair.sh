#!/bin/bash
# Round 3: 4:2:0 optimistic kernel (six per CU) with priority by frames left, against production and fair.
mkdir -p gpurun_out/optfair && export TMPDIR=/tmp
O=gpurun_out/optfair
for run in 1 2; do
for m in "420 3840 2160 300 20" "420 1920 1080 300 60"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_OPT=1 PROBE_DELTAS=1 PROBE_WARM_S=1.0 timeout -k 10 240 ./tools/probe $m > $O/opt_$1_$2_$run.log 2>&1 || { cat $O/opt_$1_$2_$run.log; exit 1; }
  echo "== $1 $2x$3 run $run"; grep -E "\(production\)|priority by|optimistic" $O/opt_$1_$2_$run.log | grep -v "vs production"
done
done
echo "r03_optfair done"
