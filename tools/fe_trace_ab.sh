#!/bin/bash
# Per-kernel time of the whole-file GPU decode, this tree against an earlier build (BASE, default
# tools/variants/base): rocprofv3 kernel traces of bench.py --mode file --frontend gpu (GPU box).
O=gpurun_out/fe_ab; mkdir -p $O && export TMPDIR=/tmp
BASE=${BASE-tools/variants/base/libmj423gpu.so}
[ "${AB-1}" = 0 ] || timeout -k 10 300 python tools/ab_file.py ${AB_ROUNDS-3} -- $BASE mjpeg423-video-decoder-software_amd/libmj423gpu.so@MJ423_GPU_FE_FUSED=0 mjpeg423-video-decoder-software_amd/libmj423gpu.so@MJ423_FUSED_IDCT32=1 mjpeg423-video-decoder-software_amd/libmj423gpu.so > $O/ab_file.log 2>&1 || { echo "STOP ab"; tail -5 $O/ab_file.log; exit 1; }
[ "${AB-1}" = 0 ] || cat $O/ab_file.log
for v in ${KT-new base}; do
  lib=mjpeg423-video-decoder-software_amd/libmj423gpu.so; [ $v = base ] && lib=$BASE
  MJ423_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$v -o kt --output-format csv -- python bench.py --mode file --config f2 --frontend gpu --steps 10 --no-cpu --no-verify > $O/kt_$v.log 2>&1 || { echo "STOP kt $v"; tail -5 $O/kt_$v.log; exit 1; }
  tail -1 $O/kt_$v.log | cut -c1-300
done
echo fe_trace_ab done
