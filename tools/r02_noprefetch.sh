#!/bin/bash
# GPU box: stream-kernel prefetch placement, production vs loads at the top of each frame, every mode.
export TMPDIR=/tmp
O=gpurun_out/r02np; mkdir -p $O
for g in "420 3840 2160 300" "420 1920 1080 300" "422 7680 4320 15" "444 640 480 300" "444 1920 1080 240"; do
  PROBE_GOP=24 timeout -k 10 200 ./tools/probe $g 9 > "$O/np_${g// /_}.txt" 2>&1 || { cat "$O/np_${g// /_}.txt"; exit 1; }
  echo "== $g"; grep "jitter\|xcd order\|no prefetch ldsqt static" "$O/np_${g// /_}.txt"
done
