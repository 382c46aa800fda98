#!/bin/bash
# GPU box: 4:4:4 stream-kernel tiles of 128 MCUs / 512 lanes against production (64 / 256).
export TMPDIR=/tmp
O=gpurun_out/r02s444; mkdir -p $O
for r in 1 2; do for g in "444 640 480 300" "444 1920 1080 240"; do
  PROBE_GOP=24 PROBE_GOP_ORDERS=1 timeout -k 10 200 ./tools/probe $g 9 > "$O/t_${g// /_}_$r.txt" 2>&1 || { cat "$O/t_${g// /_}_$r.txt"; exit 1; }
  echo "== $g"; grep "order tile  \|MCU tiles" "$O/t_${g// /_}_$r.txt"
done; done
