#!/bin/bash
# Stream-kernel experiment (run on the GPU box): how does decode_gop_kernel's bandwidth
# depend on the GOP length (frames each workgroup walks in sequence)?
set -o pipefail
mkdir -p gpurun_out
for cfg in c3 c2; do
  for gop in 1 2 4 8 24 100; do
    echo "== $cfg gop $gop"
    timeout -k 10 240 python bench.py --config $cfg --mode stream --gop $gop --no-cpu --verify ends --steps 10 || exit $?
  done
  echo "== $cfg batch"
  timeout -k 10 240 python bench.py --config $cfg --no-cpu --verify ends --steps 10 || exit $?
done
