#!/bin/bash
# GPU box: global-state stream kernel (decode_gop_gs_kernel) checked against production, then
# timed beside it, every stream config.
export TMPDIR=/tmp
O=gpurun_out/r02gs; mkdir -p $O
rocm-smi --showserial 2>/dev/null | grep -i "serial number" | head -1
for g in "420 3840 2160 300" "420 1920 1080 300" "444 640 480 300" "444 1920 1080 240" "422 7680 4320 15"; do
  PROBE_GOP=24 PROBE_GS=1 timeout -k 10 300 ./tools/probe $g 7 > "$O/gs_${g// /_}.txt" 2>&1 || { cat "$O/gs_${g// /_}.txt"; exit 1; }
  echo "== $g"; grep "global-state\|gop<\|batch" "$O/gs_${g// /_}.txt"
done
