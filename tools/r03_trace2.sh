#!/bin/bash
# Round 3: phase traces of the stream kernel and the batch kernel on the same frames (PROBE_TRACE),
# then the stream-kernel workgroup orders and ablations with the current kernel (PROBE_GOP_ORDERS).
mkdir -p gpurun_out/trace2 && export TMPDIR=/tmp
O=gpurun_out/trace2
for m in "444 640 480 300" "420 1920 1080 300" "420 3840 2160 300"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_TRACE=1 PROBE_DELTAS=1 timeout -k 10 120 ./tools/probe $m > $O/trace_$1_$2.log 2>&1 || { cat $O/trace_$1_$2.log; exit 1; }
  echo "== $1 $2x$3"; grep trace $O/trace_$1_$2.log
done
for m in "420 3840 2160 300 20" "420 1920 1080 300 60" "444 640 480 300 200"; do
  set -- $m
  PROBE_GOP=24 PROBE_GOP_ORDERS=1 PROBE_DELTAS=1 PROBE_WARM_S=1.5 timeout -k 10 240 ./tools/probe $m > $O/orders_$1_$2.log 2>&1 || { cat $O/orders_$1_$2.log; exit 1; }
  echo "== $1 $2x$3"; grep -E "gop<" $O/orders_$1_$2.log
done
echo "r03_trace2 done"
