#!/bin/bash
# A/B builds of libmj423gpu.so with compile-time overrides, for measurements only:
#   tools/build_variant.sh NAME '-DMJ423_GOP_SHAPE420=32,256'
# -> tools/variants/NAME/libmj423gpu.so; select it with MJ423_LIB=tools/variants/NAME/libmj423gpu.so
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
pkg=$root/mjpeg423-video-decoder-software_amd
out=$root/tools/variants/$name
mkdir -p "$out"
flags="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-command-line-argument $*"
objs=()
for src in mj423_kernels.hip mj423_entropy.hip mj423_runtime.cpp mj423_accel.cpp mj423_io.cpp mj423_pipeline.cpp mj423_gpu_frontend.cpp mj423_multi.cpp mj423_dropin.cpp mj423_margin.hip mj423_fused.hip; do
  o=$out/${src%.*}.o
  /opt/rocm/bin/hipcc $flags -x hip -c "$pkg/csrc/$src" -o "$o" &
  objs+=("$o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/libmj423gpu.so" "${objs[@]}" -lpthread -ldl
rm -f "${objs[@]}"
echo "$out/libmj423gpu.so"
