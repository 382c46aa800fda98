#!/bin/bash
# Round 3 diagnostic: the one-shot batch body under stream-like workgroup orders (PROBE_ORDERS,
# decode_order_kernel in tools/probe_variants.hip) beside the stream kernel, one process per size.
mkdir -p gpurun_out/orders && export TMPDIR=/tmp
O=gpurun_out/orders
for m in "420 3840 2160 300 50" "420 1920 1080 300 100"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_ORDERS=1 PROBE_DELTAS=1 PROBE_WARM_S=1.0 timeout -k 10 240 ./tools/probe $m > $O/orders_$1_$2.log 2>&1 || { cat $O/orders_$1_$2.log; exit 1; }
  echo "== $1 $2x$3 x$4"; grep -E "median|vs production" $O/orders_$1_$2.log
done
echo "r03_orders done"
