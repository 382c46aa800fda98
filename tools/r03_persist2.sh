#!/bin/bash
# Round 3: loop-per-workgroup against one-shot at equal occupancy and code (the batch kernel with the
# stream kernel's LDS and int32 forms, persistent or not), the stream kernel beside them.
mkdir -p gpurun_out/persist2 && export TMPDIR=/tmp
O=gpurun_out/persist2
for m in "420 3840 2160 300 20" "420 1920 1080 300 60"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_PERSIST=1 PROBE_DELTAS=1 PROBE_WARM_S=1.5 timeout -k 10 240 ./tools/probe $m > $O/persist_$1_$2.log 2>&1 || { cat $O/persist_$1_$2.log; exit 1; }
  echo "== $1 $2x$3"; grep -E "one-shot|persistent|stream kernel" $O/persist_$1_$2.log
done
echo "r03_persist2 done"
