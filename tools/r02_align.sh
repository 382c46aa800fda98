#!/bin/bash
# GPU box: balanced vs 2-KiB-aligned 4:2:0 tiles, batch and stream kernels, two runs.
export TMPDIR=/tmp
O=gpurun_out/r02al; mkdir -p $O
rocm-smi --showserial 2>/dev/null | grep -i "serial number" | head -1
for r in 1 2; do for g in "420 3840 2160 300" "420 1920 1080 300"; do
  PROBE_GOP=24 PROBE_ALIGN=1 timeout -k 10 200 ./tools/probe $g 9 > "$O/al_${g// /_}_$r.txt" 2>&1 || { cat "$O/al_${g// /_}_$r.txt"; exit 1; }
  echo "== $g"; grep "tiles" "$O/al_${g// /_}_$r.txt"
done; done
