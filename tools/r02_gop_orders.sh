#!/bin/bash
# GPU box: stream-kernel workgroup orders, same process and buffers, every stream config, two runs.
export TMPDIR=/tmp
O=gpurun_out/r02gord; mkdir -p $O
rocm-smi --showserial 2>/dev/null | grep -i "serial number" | head -1
for r in 1 2; do for g in "420 3840 2160 300" "420 1920 1080 300" "422 7680 4320 15" "444 640 480 300" "444 1920 1080 240"; do
  PROBE_GOP=24 PROBE_GOP_ORDERS=1 timeout -k 10 200 ./tools/probe $g 9 > "$O/o_${g// /_}_$r.txt" 2>&1 || { cat "$O/o_${g// /_}_$r.txt"; exit 1; }
  echo "== $g"; grep "order" "$O/o_${g// /_}_$r.txt"
done; done
