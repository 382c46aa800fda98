#!/bin/bash
# Round 6: bench.py's whole-file line on a 240-frame reference-encoded clean static 1080p scene (10 GOPs).
set -o pipefail
O=gpurun_out/r06/real_bench; mkdir -p $O && export TMPDIR=/tmp
MJ423_LIB=tools/variants/r6count/libmj423gpu.so MJ423_ENTPAR_DEBUG=1 timeout -k 10 120 python bench.py --mode file --frontend gpu --mpg realdata/clean_1080p_240.mpg --steps 1 --warmup 0 --no-cpu --no-verify > $O/clean240_debug.log 2>&1 || { echo STOP debug; exit 1; }
grep "entpar: window" $O/clean240_debug.log | head -6
timeout -k 10 300 python bench.py --mode file --frontend gpu --mpg realdata/clean_1080p_240.mpg --steps 20 > $O/clean240_bench.log 2>&1 || { echo STOP bench; tail -5 $O/clean240_bench.log; exit 1; }
tail -1 $O/clean240_bench.log | cut -c1-300
