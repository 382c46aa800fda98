#!/bin/bash
# Round 3: batch kernel with raised wave priority at load issue / during the CSC, same process, two runs.
mkdir -p gpurun_out/bprio && export TMPDIR=/tmp
O=gpurun_out/bprio
for run in 1 2; do
for m in "420 3840 2160 300 20" "420 1920 1080 300 60" "444 640 480 300 200" "422 7680 4320 15 60"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_BPRIO=1 PROBE_WARM_S=1.0 timeout -k 10 240 ./tools/probe $m > $O/bprio_$1_$2_$run.log 2>&1 || { cat $O/bprio_$1_$2_$run.log; exit 1; }
  echo "== $1 $2x$3 run $run"; grep -E "production|priority|both" $O/bprio_$1_$2_$run.log
done
done
echo "r03_bprio done"
