#!/bin/bash
# GPU box: record-input stream kernel (compact 64-B block records instead of dense planes),
# checked against production, then timed beside it.
export TMPDIR=/tmp
O=gpurun_out/r02rec; mkdir -p $O
for g in "420 3840 2160 300" "420 1920 1080 300" "444 640 480 300" "444 1920 1080 240"; do
  PROBE_GOP=24 PROBE_REC=1 timeout -k 10 300 ./tools/probe $g 7 > "$O/rec_${g// /_}.txt" 2>&1 || { cat "$O/rec_${g// /_}.txt"; exit 1; }
  echo "== $g"; grep "records\|record-input\|gop<" "$O/rec_${g// /_}.txt"
done
