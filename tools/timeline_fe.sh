#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out/tl
for wv in 1,2,2 1,1,1 1,2,2 1,1,1; do
  i=$((i+1))
  MJ423_GPU_FE_WINDOWS=$wv timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace -d gpurun_out/tl/${wv}_$i -o kt --output-format csv -- python bench.py --mode file --config f2 --frontend gpu --steps 4 --warmup 1 --no-cpu --no-verify > gpurun_out/tl/${wv}_$i.log 2>&1 || exit 1
  tail -1 gpurun_out/tl/${wv}_$i.log | cut -c1-200
done
