#!/bin/bash
# Pipeline chunk size A/B (file mode, 240 x 1080p 4:4:4): 24 vs 48 frames per chunk, host and
# device sinks, alternating, two rounds.
mkdir -p gpurun_out/chunk && export TMPDIR=/tmp
for r in 1 2; do for c in 24 48; do for sk in host device; do
  timeout -k 10 300 python bench.py --mode file --config f2 --steps 10 --sink $sk --chunk $c --no-cpu > gpurun_out/chunk/${sk}_${c}_$r.json 2>/dev/null || exit 1
  tail -1 gpurun_out/chunk/${sk}_${c}_$r.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('round $r chunk $c $sk', d['value'], d['roofline']['frac'], d['parity_verified'])"
done; done; done
