#!/bin/bash
# GPU box: stream-kernel parity with the start jitter on (default), then bench A/B
# (MJ423_GOP_JITTER = 1 | 0 default) at the BASELINE stream configs, then the probe.
export TMPDIR=/tmp
O=gpurun_out/r02jt; mkdir -p $O
rocm-smi --showserial 2>/dev/null | grep -i serial | head -1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -x -q --timeout 120 --timeout-method thread -m gpu -k "stream or gop or mpg or pipeline or gpu_entropy or multi" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for c in c3 c2 c5 c1; do
    for j in 1 0; do
      MJ423_GOP_JITTER=$j timeout -k 10 200 python bench.py --config $c --mode stream --steps 20 --no-cpu > $O/${c}s_j${j}_$r.json 2> $O/${c}s_j${j}_$r.err || { tail -5 $O/${c}s_j${j}_$r.err; exit 1; }
      python -c "import json; d=json.loads(open('$O/${c}s_j${j}_$r.json').read().strip().splitlines()[-1]); print('$c', 'jitter=$j', d['roofline']['frac'], d['parity_verified'])"
    done
  done
done
