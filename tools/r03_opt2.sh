#!/bin/bash
# Round 3: SIMD placement of the waves of 4-wave workgroups (tools/hwid_probe), then the stream-kernel
# variants of PROBE_OPT (production, optimistic at six per CU, exact and optimistic with the early
# prefetch) checked against production and timed in one process.
mkdir -p gpurun_out/opt2 && export TMPDIR=/tmp
O=gpurun_out/opt2
timeout -k 10 60 ./tools/hwid_probe > $O/hwid.log 2>&1 || { cat $O/hwid.log; exit 1; }
cat $O/hwid.log
for m in "444 640 480 300 200" "420 1920 1080 300 60" "420 3840 2160 300 20" "422 7680 4320 15 60" "444 1920 1080 300 40"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_OPT=1 PROBE_DELTAS=1 PROBE_WARM_S=1.5 timeout -k 10 240 ./tools/probe $m > $O/$1_$2.log 2>&1 || { cat $O/$1_$2.log; exit 1; }
  echo "== $1 $2x$3"; grep -E "optimistic|production|re-run|exact" $O/$1_$2.log
done
echo "r03_opt2 done"
