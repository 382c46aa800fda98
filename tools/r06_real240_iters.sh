#!/bin/bash
# Round 6: synchronisation iterations on the 240-frame reference-encoded clean scene (bench.py --mpg).
set -o pipefail
O=gpurun_out/r06/real_bench; mkdir -p $O && export TMPDIR=/tmp
for it in 10 6 5 4; do
  MJ423_GPU_FE_ITERS=$it timeout -k 10 300 python bench.py --mode file --frontend gpu --mpg realdata/clean_1080p_240.mpg --steps 20 --no-cpu > $O/clean240_it$it.log 2>&1 || { echo STOP $it; tail -5 $O/clean240_it$it.log; exit 1; }
  echo "iters $it: $(tail -1 $O/clean240_it$it.log | cut -c1-260 | grep -o '"ms_per_step": [0-9.]*')"
done
