#!/bin/bash
# GPU box: stream-kernel parity with the default workgroup order, then bench A/B of the orders
# (MJ423_GOP_ORDER = eighths (default) | tile) at the BASELINE stream configs.
export TMPDIR=/tmp
O=gpurun_out/r02go; mkdir -p $O
rocm-smi --showserial 2>/dev/null | grep -i serial | head -1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -x -q --timeout 120 --timeout-method thread -m gpu -k "stream or gop or mpg or pipeline or gpu_entropy or multi" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for c in c3 c2 c5 c1; do
    for o in eighths tile; do
      MJ423_GOP_ORDER=$o timeout -k 10 200 python bench.py --config $c --mode stream --steps 20 --no-cpu > $O/${c}s_${o}_$r.json 2> $O/${c}s_${o}_$r.err || { tail -5 $O/${c}s_${o}_$r.err; exit 1; }
      python -c "import json; d=json.loads(open('$O/${c}s_${o}_$r.json').read().strip().splitlines()[-1]); print('$c', '$o', d['roofline']['frac'], d['parity_verified'])"
    done
  done
done
