#!/bin/bash
# Round 3: per-frame phase timestamps of the stream kernel (PROBE_TRACE), then the conditional-
# against-unconditional prefetch A/B and the optimistic forms (PROBE_OPT), one process per geometry.
mkdir -p gpurun_out/trace && export TMPDIR=/tmp
O=gpurun_out/trace
for m in "444 640 480 300" "420 1920 1080 300" "420 3840 2160 300" "422 7680 4320 15"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_TRACE=1 PROBE_DELTAS=1 timeout -k 10 120 ./tools/probe $m > $O/trace_$1_$2.log 2>&1 || { cat $O/trace_$1_$2.log; exit 1; }
  echo "== $1 $2x$3"; grep trace $O/trace_$1_$2.log
done
for m in "444 640 480 300 200" "420 1920 1080 300 60" "420 3840 2160 300 20" "422 7680 4320 15 60" "444 1920 1080 300 40"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_OPT=1 PROBE_DELTAS=1 PROBE_WARM_S=1.5 timeout -k 10 240 ./tools/probe $m > $O/opt_$1_$2.log 2>&1 || { cat $O/opt_$1_$2.log; exit 1; }
  echo "== $1 $2x$3"; grep -E "gop<" $O/opt_$1_$2.log
done
echo "r03_trace done"
