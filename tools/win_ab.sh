#!/bin/bash
# Window schedules of the whole-file GPU decode (MJ423_GPU_FE_WINDOWS), one process per run (the
# contexts of a multi-build process share the 4 hardware queues -- tools/ab_file.py's position
# artifact), ROUNDS interleaved rounds.  GPU box.
O=gpurun_out/win; mkdir -p $O
for r in $(seq ${ROUNDS-2}); do
  for w in "$@"; do
    MJ423_GPU_FE_WINDOWS=$w timeout -k 10 120 python bench.py --mode file --config f2 --frontend gpu --steps 20 --no-cpu --no-verify > $O/w.log 2>&1 || { echo "STOP $w"; tail -3 $O/w.log; exit 1; }
    echo "windows $w: $(tail -1 $O/w.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
  done
done
