#!/bin/bash
# Environment settings of the whole-file GPU decode, one process per run, ROUNDS interleaved rounds:
#   tools/env_ab.sh "MJ423_GPU_FE_RESERVE=0" "MJ423_GPU_FE_RESERVE=32 MJ423_GPU_FE_PREP=0" ...   (GPU box)
O=gpurun_out/envab; mkdir -p $O
for r in $(seq ${ROUNDS-2}); do
  for v in "$@"; do
    env $v timeout -k 10 120 python bench.py --mode file --config f2 --frontend gpu --steps 20 --no-cpu --no-verify > $O/r.log 2>&1 || { echo "STOP $v"; tail -3 $O/r.log; exit 1; }
    echo "[$v]: $(tail -1 $O/r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
