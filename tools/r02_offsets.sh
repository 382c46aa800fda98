#!/bin/bash
# GPU box: output-buffer offset sensitivity of the production batch and stream kernels.
export TMPDIR=/tmp
O=gpurun_out/r02off; mkdir -p $O
rocm-smi --showserial 2>/dev/null | grep -i "serial number" | head -1
for g in "420 3840 2160 300" "420 1920 1080 300" "444 640 480 300"; do
  PROBE_GOP=24 PROBE_OFFSETS=0,2048,4096,8192,16384,65536,262144,1048576,3158016 timeout -k 10 300 ./tools/probe $g 5 > "$O/off_${g// /_}.txt" 2>&1 || { cat "$O/off_${g// /_}.txt"; exit 1; }
  echo "== $g"; grep "out +" "$O/off_${g// /_}.txt"
done
