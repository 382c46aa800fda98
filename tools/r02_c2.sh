#!/bin/bash
# GPU box: bench roofline vs number of warm-up steps (clock ramp?), C2 and C3.
export TMPDIR=/tmp
O=gpurun_out/r02w; mkdir -p $O
for cfg in c2 c3 c1; do for w in 3 30 3 100; do
timeout -k 10 300 python bench.py --config $cfg --no-cpu --no-verify --steps 20 --warmup $w > $O/b.json 2>$O/b.err || { tail $O/b.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/b.json'));r=d['roofline'];print('$cfg warmup $w', r['frac'], r['frac_median'], r['kernel_ms_avg'], r['kernel_ms_median'])"
done; done
