#!/bin/bash
# Round 3: stream-kernel jobs of one XCD band in loose lock step (kGopLockstep, PROBE_LOCK) against
# production, eighths order and frames-left priority, one process per geometry; then the order diagnostic.
mkdir -p gpurun_out/lock && export TMPDIR=/tmp
O=gpurun_out/lock
for m in "420 3840 2160 300 50" "420 1920 1080 300 100" "444 640 480 300 200" "444 1920 1080 48 200"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_OPT=1 PROBE_LOCK=1 PROBE_DELTAS=1 PROBE_WARM_S=1.0 timeout -k 10 240 ./tools/probe $m > $O/lock_$1_$2.log 2>&1 || { cat $O/lock_$1_$2.log; exit 1; }
  echo "== $1 $2x$3 x$4"; grep -E "gop<|vs production" $O/lock_$1_$2.log
done
echo "r03_lock done"
