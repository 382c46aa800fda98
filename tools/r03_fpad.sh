#!/bin/bash
# Round 3 diagnostic: gaps between consecutive frames of the coefficient and output buffers
# (PROBE_FPAD bytes) under the batch kernel, the one-shot orders and the stream kernel.
mkdir -p gpurun_out/fpad && export TMPDIR=/tmp
O=gpurun_out/fpad
for m in "420 3840 2160 300 40" "420 1920 1080 300 80"; do
  set -- $m
  for pad in 0 2048 8448 1052672 4096; do
    PROBE_R03=1 PROBE_GOP=24 PROBE_FPAD=$pad PROBE_DELTAS=1 PROBE_WARM_S=0.5 timeout -k 10 200 ./tools/probe $m > $O/fpad_$2_$pad.log 2>&1 || { cat $O/fpad_$2_$pad.log; exit 1; }
    echo "== $2x$3 pad $pad"; grep -E "one-shot|stream kernel|order xcd" $O/fpad_$2_$pad.log | grep median
  done
done
echo "r03_fpad done"
