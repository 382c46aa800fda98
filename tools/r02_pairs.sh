#!/bin/bash
# GPU box: the production batch kernel on several separately allocated buffer pairs in one
# process (physical-placement sensitivity), 4K and 1080p 4:2:0.
export TMPDIR=/tmp
O=gpurun_out/r02pairs; mkdir -p $O
rocm-smi --showserial 2>/dev/null | grep -i "serial number" | head -1
for g in "420 3840 2160 300" "420 1920 1080 300"; do
  PROBE_PAIRS=6 timeout -k 10 300 ./tools/probe $g 9 > "$O/pairs_${g// /_}.txt" 2>&1 || { cat "$O/pairs_${g// /_}.txt"; exit 1; }
  echo "== $g"; grep "pair" "$O/pairs_${g// /_}.txt"
done
