#!/bin/bash
# Which buffer sets the batch kernel's level (tools/placement_probe.py), then the pooled policy,
# then the default bench line for context.  GPU box; every step has its own limit.
mkdir -p gpurun_out/placement && export TMPDIR=/tmp
timeout -k 10 300 python tools/placement_probe.py ${N-6} > gpurun_out/placement/split.jsonl 2>&1 || { echo "STOP split"; tail -5 gpurun_out/placement/split.jsonl; exit 1; }
tail -1 gpurun_out/placement/split.jsonl
timeout -k 10 300 python tools/placement_probe.py ${N-6} --pool > gpurun_out/placement/pool.jsonl 2>&1 || { echo "STOP pool"; tail -5 gpurun_out/placement/pool.jsonl; exit 1; }
tail -1 gpurun_out/placement/pool.jsonl
for m in contig contig-out; do
  timeout -k 10 300 python tools/placement_probe.py ${N-6} --$m > gpurun_out/placement/$m.jsonl 2>&1 || { echo "STOP $m"; tail -5 gpurun_out/placement/$m.jsonl; exit 1; }
  tail -1 gpurun_out/placement/$m.jsonl
done
timeout -k 10 300 python bench.py --steps 20 > gpurun_out/placement/bench_c3.log 2>&1 || { echo "STOP bench"; exit 1; }
tail -1 gpurun_out/placement/bench_c3.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench c3', d['value'], d['roofline']['frac'])"
echo placement_check done
