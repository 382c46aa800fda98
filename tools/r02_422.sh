#!/bin/bash
# GPU box: 4:2:2 stream-kernel tile shapes (64 MCUs / 256 lanes production, 32 / 128, 32 / 256), 8K and 1080p.
export TMPDIR=/tmp
O=gpurun_out/r02s422; mkdir -p $O
for r in 1 2; do for g in "422 7680 4320 15" "422 1920 1080 240"; do
  PROBE_GOP=24 PROBE_GOP_ORDERS=1 timeout -k 10 200 ./tools/probe $g 9 > "$O/t_${g// /_}_$r.txt" 2>&1 || { cat "$O/t_${g// /_}_$r.txt"; exit 1; }
  echo "== $g"; grep "order tile  \|MCU tiles" "$O/t_${g// /_}_$r.txt"
done; done
