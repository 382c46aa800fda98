#!/bin/bash
# GPU box: stream kernel production vs its arithmetic and store ablations, same process.
export TMPDIR=/tmp
O=gpurun_out/r02abl; mkdir -p $O
for g in "420 3840 2160 300" "420 1920 1080 300" "444 640 480 300" "444 1920 1080 240"; do
  PROBE_GOP=24 PROBE_GOP_ORDERS=1 timeout -k 10 200 ./tools/probe $g 7 > "$O/a_${g// /_}.txt" 2>&1 || { cat "$O/a_${g// /_}.txt"; exit 1; }
  echo "== $g"; grep "order tile" "$O/a_${g// /_}.txt"
done
