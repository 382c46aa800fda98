#!/bin/bash
# Round-2 opening check on the GPU box: GPU parity suite, smoke, default bench, kernel trace.
export TMPDIR=/tmp
mkdir -p gpurun_out/r02a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02a/pytest_gpu.log 2>&1 || { tail -20 gpurun_out/r02a/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r02a/pytest_gpu.log
timeout -k 10 300 python bench.py > gpurun_out/r02a/bench.json 2> gpurun_out/r02a/bench.err || { tail gpurun_out/r02a/bench.err; exit 1; }
tail -1 gpurun_out/r02a/bench.json
echo done
