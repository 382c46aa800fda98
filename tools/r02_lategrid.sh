#!/bin/bash
# GPU box: GPU front-end parity tests with the LDS-staged walk window, the whole-file decode
# bench A/B (window on, MJ423_GPU_FE_LATE_GRID=0 off), then a kernel trace of the default.
export TMPDIR=/tmp
O=gpurun_out/r02lg; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -x -v --timeout 120 --timeout-method thread -m gpu -k "gpu_entropy or mpg" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in 1 2; do
  for mode in on off; do
    if [ $mode = off ]; then export MJ423_GPU_FE_LATE_GRID=0; else unset MJ423_GPU_FE_LATE_GRID; fi
    timeout -k 10 200 python -u bench.py --mode file --config f2 --frontend gpu --steps 20 > $O/f2_${mode}_$r.json 2> $O/f2_${mode}_$r.err || { tail -20 $O/f2_${mode}_$r.err; exit 1; }
    python -c "import json; d=json.loads(open('$O/f2_${mode}_$r.json').read().strip().splitlines()[-1]); print('$mode', d['value'], d['unit'], d['ms_per_step'], d.get('parity_verified'))"
  done
done
unset MJ423_GPU_FE_LATE_GRID
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof -o fe --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --mode file --config f2 --frontend gpu --steps 20 > $GRAFT_REPO_ROOT/$O/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$O/prof.log; exit 1; }
echo done
