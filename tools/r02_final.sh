#!/bin/bash
# GPU box: the round-end gate on this tree -- the whole GPU suite, smoke, the default bench and
# the stream benches, a kernel trace of the default bench.
export TMPDIR=/tmp
O=gpurun_out/final; mkdir -p $O
rocm-smi --showserial 2>/dev/null | grep -i "serial number" | head -1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
for m in "--config c3 --mode stream" "--config c2 --mode stream" "--config c2"; do
  n=$(echo $m | tr -d ' -'); timeout -k 10 300 python bench.py $m --steps 20 > $O/bench_$n.json 2> $O/bench_$n.err || { tail -5 $O/bench_$n.err; exit 1; }
done
for f in $O/bench_*.json; do python -c "import json; d=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', d['value'], d['roofline']['frac'], d['parity_verified'])"; done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_c3 -o kt --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --no-cpu > $GRAFT_REPO_ROOT/$O/prof_c3.log 2>&1 || { tail -5 $GRAFT_REPO_ROOT/$O/prof_c3.log; exit 1; }
echo final done
