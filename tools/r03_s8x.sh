#!/bin/bash
# Round 3: the int8-state stream kernel with the exact int32 transform + CSC (only an int8 overflow escapes
# to the re-run pass) at five and six workgroups per CU, against production, in one process per geometry.
mkdir -p gpurun_out/s8x && export TMPDIR=/tmp
O=gpurun_out/s8x
for m in "420 3840 2160 300 50" "420 1920 1080 300 100" "422 7680 4320 48 100" "444 640 480 300 200" "444 1920 1080 48 200"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_OPT=1 PROBE_S8X=1 PROBE_DELTAS=1 PROBE_WARM_S=1.0 timeout -k 10 240 ./tools/probe $m > $O/s8x_$1_$2.log 2>&1 || { cat $O/s8x_$1_$2.log; exit 1; }
  echo "== $1 $2x$3 x$4"; grep -E "median|vs production" $O/s8x_$1_$2.log
done
echo "r03_s8x done"
