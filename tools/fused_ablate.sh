#!/bin/bash
# Time of the fused .mpg kernel with one part left out (tools/variants/abl{1,2,3}: no IDCT / no CSC /
# no block decode; outputs wrong), kernel traces of bench.py --mode file (GPU box; measurement only).
O=gpurun_out/ablate; mkdir -p $O && export TMPDIR=/tmp
for v in base abl1 abl2 abl3; do
  lib=mjpeg423-video-decoder-software_amd/libmj423gpu.so; [ $v != base ] && lib=tools/variants/$v/libmj423gpu.so
  MJ423_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt_$v -o kt --output-format csv -- python bench.py --mode file --config f2 --frontend gpu --steps 10 --no-cpu --no-verify > $O/kt_$v.log 2>&1 || { echo "STOP $v"; tail -3 $O/kt_$v.log; exit 1; }
  echo "$v: $(python tools/kt_summary.py $O/kt_$v 13 | head -1)"
done
