#!/bin/bash
# Round 3: the stream kernel's loop-header wait -- production (the previous frame's stores drained at
# every loop header, a side effect of vmcnt's issue order) vs kGopEntryWait (the prefetched loads only,
# stores left in flight), in one process per geometry.
mkdir -p gpurun_out/wait && export TMPDIR=/tmp
O=gpurun_out/wait
for m in "420 3840 2160 300 50" "420 1920 1080 300 100" "422 7680 4320 48 100" "444 640 480 300 200" "444 1920 1080 48 200"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_OPT=1 PROBE_WAIT=1 PROBE_DELTAS=1 PROBE_WARM_S=1.0 timeout -k 10 240 ./tools/probe $m > $O/wait_$1_$2.log 2>&1 || { cat $O/wait_$1_$2.log; exit 1; }
  echo "== $1 $2x$3 x$4"; grep -E "median|vs production" $O/wait_$1_$2.log
done
echo "r03_wait done"
