#!/bin/bash
# GPU box: timing-totals test, then file-mode benches whose roofline now covers every
# stream-kernel launch of the timed passes.
export TMPDIR=/tmp
O=gpurun_out/r02fm; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "timing or mpg" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for v in "host:--sink host" "device:--sink device" "gpufe:--frontend gpu"; do
  n=${v%%:*}; args=${v#*:}
  timeout -k 10 300 python bench.py --mode file --config f2 $args --steps 5 --no-cpu > $O/f2_$n.json 2> $O/f2_$n.err || { tail -5 $O/f2_$n.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/f2_$n.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$n', d['value'], r['frac'], r['kernel_launches'], r['kernel_ms_avg'], d['parity_verified'])"
done
