#!/bin/bash
# Round 3: stream kernel with wave priority by frames left in the job (kGopFair) against production:
# outputs compared, timed in one process (PROBE_OPT), and traced by frame index (PROBE_TRACE).
mkdir -p gpurun_out/fair && export TMPDIR=/tmp
O=gpurun_out/fair
for m in "444 640 480 300 200" "444 1920 1080 300 40" "420 1920 1080 300 60" "420 3840 2160 300 20" "422 7680 4320 15 60"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_OPT=1 PROBE_DELTAS=1 PROBE_WARM_S=1.5 timeout -k 10 240 ./tools/probe $m > $O/opt_$1_$2.log 2>&1 || { cat $O/opt_$1_$2.log; exit 1; }
  echo "== $1 $2x$3"; grep -E "gop<" $O/opt_$1_$2.log | grep -v "vs production"
done
for m in "444 640 480 300" "420 3840 2160 300"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_TRACE=1 PROBE_DELTAS=1 timeout -k 10 120 ./tools/probe $m > $O/trace_$1_$2.log 2>&1 || { cat $O/trace_$1_$2.log; exit 1; }
  echo "== $1 $2x$3"; grep "trace" $O/trace_$1_$2.log | grep -v "CU span"
done
echo "r03_fair done"
