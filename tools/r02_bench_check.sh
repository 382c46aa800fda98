#!/bin/bash
# Default bench (new CPU-baseline leg) + host CPU facts on the GPU box.
export TMPDIR=/tmp
mkdir -p gpurun_out/r02b
python - > gpurun_out/r02b/host.txt 2>&1 <<'PY'
import os
print("nproc", os.cpu_count(), "affinity", len(os.sched_getaffinity(0)), "OMP", os.environ.get("OMP_NUM_THREADS"))
for f in ("/sys/fs/cgroup/cpu.max", "/proc/self/cgroup"):
    try: print(f, open(f).read().strip())
    except OSError as e: print(f, e)
PY
cat gpurun_out/r02b/host.txt
timeout -k 10 300 python bench.py > gpurun_out/r02b/bench.json 2> gpurun_out/r02b/bench.err || { tail gpurun_out/r02b/bench.err; exit 1; }
tail -1 gpurun_out/r02b/bench.json
timeout -k 10 300 python bench.py --gpus 1 --config c2 --cpu-seconds 8 > gpurun_out/r02b/bench_c2.json 2> gpurun_out/r02b/bench_c2.err || { tail gpurun_out/r02b/bench_c2.err; exit 1; }
tail -1 gpurun_out/r02b/bench_c2.json
