#!/bin/bash
# Whole-file GPU decode (240 x 1080p 4:4:4, mj423_mpg_decode_gpu), library builds A/B one process per
# run (tools/ab_file.py with a single build: no shared hardware queues), ROUNDS interleaved rounds.
O=gpurun_out/file_ab; mkdir -p $O
for r in $(seq ${ROUNDS-3}); do
  for l in "$@"; do
    timeout -k 10 120 python tools/ab_file.py 3 -- $l > $O/r.log 2>&1 || { echo "STOP $l"; tail -3 $O/r.log; exit 1; }
    grep "^file" $O/r.log | sed "s|^|round $r $l: |" | tee -a $O/all.log
  done
done
