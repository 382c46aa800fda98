#!/bin/bash
# Round 3: rotating wave priority against production and priority by frames left, grids of many rounds.
mkdir -p gpurun_out/rot && export TMPDIR=/tmp
O=gpurun_out/rot
for m in "420 3840 2160 300 20" "420 1920 1080 300 60" "444 1920 1080 300 40" "444 640 480 300 200"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_OPT=1 PROBE_DELTAS=1 PROBE_WARM_S=1.0 timeout -k 10 240 ./tools/probe $m > $O/opt_$1_$2.log 2>&1 || { cat $O/opt_$1_$2.log; exit 1; }
  echo "== $1 $2x$3"; grep -E "\(production\)|priority" $O/opt_$1_$2.log | grep -v "vs production"
done
echo "r03_rot done"
