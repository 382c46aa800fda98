#!/bin/bash
# Round 3: one-round stream grids -- a start delay by arrival order on the CU on top of priority by frames left.
# (The start-delay variants this ran are gone from tools/probe.hip; their flag bit went to kGopLockstep, tools/r03_lock.sh.)
mkdir -p gpurun_out/stagger2 && export TMPDIR=/tmp
O=gpurun_out/stagger2
for run in 1 2; do
for m in "444 640 480 300 200" "444 1920 1080 48 200"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_OPT=1 PROBE_DELTAS=1 PROBE_WARM_S=1.0 timeout -k 10 240 ./tools/probe $m > $O/opt_$1_$2_$run.log 2>&1 || { cat $O/opt_$1_$2_$run.log; exit 1; }
  echo "== $1 $2x$3 x$4 run $run"; grep -E "\(production\)|priority" $O/opt_$1_$2_$run.log | grep -v "vs production"
done
done
echo "r03_stagger done"
