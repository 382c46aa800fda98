#!/bin/bash
# Whole-file decode check (GPU box): parity suite, then the file benchmark with each sink
# and front end (synthetic 1080p 4:4:4 .mpg, BASELINE-independent; never the headline).
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --mode file --config f2 > gpurun_out/f2_host.json 2> gpurun_out/f2_host.err || exit 1
timeout -k 10 300 python bench.py --mode file --config f2 --sink device > gpurun_out/f2_device.json 2> gpurun_out/f2_device.err || exit 1
timeout -k 10 300 python bench.py --mode file --config f2 --sink device --frontend gpu > gpurun_out/f2_gpufrontend.json 2> gpurun_out/f2_gpufrontend.err || exit 1
