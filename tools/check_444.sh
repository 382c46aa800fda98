#!/bin/bash
# 4:4:4 change check (GPU box): parity suite, C1 bench, probes, stream/file benches.
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --config c1 > gpurun_out/c1.json 2> gpurun_out/c1.err || exit 1
timeout -k 10 300 python bench.py --config c1 --mode stream --no-cpu > gpurun_out/c1s.json 2> gpurun_out/c1s.err || exit 1
timeout -k 10 200 ./tools/probe 444 640 480 300 7 > gpurun_out/p444a.txt 2>&1 || exit 1
timeout -k 10 200 ./tools/probe 444 1920 1080 240 7 > gpurun_out/p444b.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --mode file --config f2 --sink device --no-cpu > gpurun_out/f2d.json 2> gpurun_out/f2d.err || exit 1
