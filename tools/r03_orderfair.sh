#!/bin/bash
# Round 3: stream-kernel workgroup orders crossed with priority by frames left (kGopFair).
mkdir -p gpurun_out/orderfair && export TMPDIR=/tmp
O=gpurun_out/orderfair
for m in "420 3840 2160 300 20" "420 1920 1080 300 60" "422 7680 4320 15 60" "444 1920 1080 300 40"; do
  set -- $m
  PROBE_GOP=24 PROBE_GOP_ORDERS=1 PROBE_DELTAS=1 PROBE_WARM_S=1.5 timeout -k 10 240 ./tools/probe $m > $O/orders_$1_$2.log 2>&1 || { cat $O/orders_$1_$2.log; exit 1; }
  echo "== $1 $2x$3"; grep -E "order" $O/orders_$1_$2.log
done
echo "r03_orderfair done"
