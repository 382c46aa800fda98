#!/bin/bash
# Builds of libmj423gpu.so on the whole-file GPU decode (bench.py --mode file --frontend gpu, f2),
# one process per run, ROUNDS interleaved rounds; the first round verifies every frame against
# the oracle (--verify all).  Args: library paths (tools/build_variant.sh).  GPU box.
O=gpurun_out/libab; mkdir -p $O
for r in $(seq ${ROUNDS-2}); do
  for l in "$@"; do
    v=--no-verify; [ $r = 1 ] && v="--verify all"
    MJ423_LIB=$l timeout -k 10 180 python bench.py --mode file --config f2 --frontend gpu --steps 20 --no-cpu $v > $O/l.log 2>&1 || { echo "STOP $l"; tail -3 $O/l.log; exit 1; }
    echo "$l: $(tail -1 $O/l.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d.get("parity_verified"), d.get("parity_frames_checked"))')"
  done
done
