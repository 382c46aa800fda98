#!/bin/bash
# A/B of GPU front-end builds (tools/variants/*), interleaved rounds (GPU box).
mkdir -p gpurun_out
for r in 1 2; do
  for v in ${VARIANTS}; do
    echo -n "$v: "
    MJ423_LIB=tools/variants/$v/libmj423gpu.so timeout -k 10 200 python tools/gpu_fe_probe.py 1920 1080 ${COUNTS:-240} 2>/dev/null | grep x || exit 1
  done
done
