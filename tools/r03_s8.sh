#!/bin/bash
# Round 3: int8 LDS state for the stream kernel (six workgroups per CU at 4:2:0 / 4:4:4) against
# production: outputs compared first (real P-frame deltas), then timed in one process.
mkdir -p gpurun_out/s8 && export TMPDIR=/tmp
for m in "444 640 480 300 200" "420 1920 1080 300 60" "420 3840 2160 300 20" "422 7680 4320 15 60"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_S8=1 PROBE_DELTAS=1 PROBE_WARM_S=1.5 timeout -k 10 240 ./tools/probe $m > gpurun_out/s8/$1_$2.log 2>&1 || { cat gpurun_out/s8/$1_$2.log; exit 1; }
  echo "== $1 $2x$3"; grep -E "int8|production|round" gpurun_out/s8/$1_$2.log
done
