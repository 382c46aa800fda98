#!/bin/bash
# Round-end evidence refresh (GPU box): tools/gpu_check.sh over every bench config with kernel
# traces + PMC passes, then the file-mode benches and a kernel trace of the GPU front end.
# Outputs under gpurun_out/; copied into profiles/r02 afterwards.
export TMPDIR=/tmp
mkdir -p gpurun_out
CONFIGS="c3 c2 c5 c1 c3s c2s c5s c1s" PROFILE="c3 c2 c5 c1 c3s c2s" bash tools/gpu_check.sh > gpurun_out/check.log 2>&1
grep -q "gpu_check done" gpurun_out/check.log || { tail -20 gpurun_out/check.log; exit 1; }
for v in host:"--sink host" device:"--sink device" gpufrontend:"--frontend gpu"; do
  n=${v%%:*}; args=${v#*:}
  timeout -k 10 300 python bench.py --mode file --config f2 --steps 20 $args > gpurun_out/f2_$n.json 2> gpurun_out/f2_$n.err || exit 1
  tail -1 gpurun_out/f2_$n.json | cut -c1-200
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_f2g_kt -o kt --output-format csv -- python bench.py --mode file --config f2 --frontend gpu --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/prof_f2g_kt.log 2>&1 || exit 1
echo "refresh done"
