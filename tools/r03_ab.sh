#!/bin/bash
# Round 3 A/B (same process, warmed clocks, interleaved rounds): int16-workspace IDCT + 16-bit
# CSC against the round-2 forms, batch and stream kernels.  Usage: r03_ab.sh [tag]
mkdir -p gpurun_out/ab && export TMPDIR=/tmp
O=gpurun_out/ab; T=${1:-run}
for m in "444 640 480 300 200" "420 1920 1080 300 60" "420 3840 2160 300 20" "422 7680 4320 15 60" "444 1920 1080 300 40"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_WARM_S=1.5 timeout -k 10 240 ./tools/probe $m > $O/${T}_$1_$2.log 2>&1 || { cat $O/${T}_$1_$2.log; exit 1; }
  echo "== $1 $2x$3"; grep -E "round|IDCT|CSC" $O/${T}_$1_$2.log
done
