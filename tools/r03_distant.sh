#!/bin/bash
# Round 3 diagnostic: the one-shot body with eight XCDs in eight distant parts of the batch, each holding
# tiles across frames (order 5), beside XCD-contiguous, bands, band walks and the stream kernel in
# tile and XCD-contiguous job orders; two processes per size.
mkdir -p gpurun_out/distant && export TMPDIR=/tmp
O=gpurun_out/distant
for run in 1 2; do
for m in "420 3840 2160 300 40" "420 1920 1080 300 80"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_FPAD=0 PROBE_DELTAS=1 PROBE_WARM_S=0.5 timeout -k 10 200 ./tools/probe $m > $O/distant_$2_$run.log 2>&1 || { cat $O/distant_$2_$run.log; exit 1; }
  echo "== $2x$3 run $run"; grep -E "one-shot|stream kernel" $O/distant_$2_$run.log | grep median
done
done
echo "r03_distant done"
