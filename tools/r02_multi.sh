#!/bin/bash
# GPU box: the multi-GPU group tests, the C driver at the headline size, then the whole GPU suite.
export TMPDIR=/tmp
mkdir -p gpurun_out/r02c
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -x -v --timeout 120 --timeout-method thread > gpurun_out/r02c/pytest_multi.log 2>&1 || { tail -40 gpurun_out/r02c/pytest_multi.log; exit 1; }
tail -3 gpurun_out/r02c/pytest_multi.log
timeout -k 10 200 ./mjpeg423-video-decoder-software_amd/mj423_multigpu > gpurun_out/r02c/multigpu_c3.json 2> gpurun_out/r02c/multigpu_c3.err || { cat gpurun_out/r02c/multigpu_c3.err; exit 1; }
tail -1 gpurun_out/r02c/multigpu_c3.json
timeout -k 10 200 ./mjpeg423-video-decoder-software_amd/mj423_multigpu --total-frames 2400 --steps 5 --warmup 1 > gpurun_out/r02c/multigpu_c4_strong.json 2> gpurun_out/r02c/multigpu_c4_strong.err || { cat gpurun_out/r02c/multigpu_c4_strong.err; exit 1; }
tail -1 gpurun_out/r02c/multigpu_c4_strong.json
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r02c/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/r02c/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/r02c/pytest_gpu.log
