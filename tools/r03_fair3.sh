#!/bin/bash
# Round 3: the fair-priority rule extended to grids whose frame fills the resident workgroups (4K 4:2:0,
# 8K 4:2:2): library benches with the rule and with MJ423_GOP_FAIR=0, interleaved, then the stream tests.
mkdir -p gpurun_out/fair3 && export TMPDIR=/tmp
O=gpurun_out/fair3
stop() { echo "STOP: $1 rc=$2"; exit "$2"; }
for run in 1 2; do
  for b in c3s c5s c2s; do
    for fair in auto 0; do
      e=""; [ $fair != auto ] && e="MJ423_GOP_FAIR=$fair"
      env $e timeout -k 10 300 python bench.py --config ${b%s} --mode stream --steps 20 --no-cpu > $O/${b}_fair${fair}_$run.json 2>$O/${b}_fair${fair}_$run.err || stop $b $?
      echo "$b fair=$fair run $run $(python -c "import json; d=json.loads(open('$O/${b}_fair${fair}_$run.json').read().strip().splitlines()[-1]); print(d['roofline']['frac'], d['parity_verified'], d['stream_reruns'])")"
    done
  done
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_switches.py -m gpu -x -q -k "stream or switch" --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest.log
echo "r03_fair3 done"
