#!/bin/bash
# Round 3: GPU suite, then the file paths and stream configs after the three-round fair-priority rule.
mkdir -p gpurun_out/check5 && export TMPDIR=/tmp
O=gpurun_out/check5
stop() { echo "STOP: $1 rc=$2"; exit "$2"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $O/pytest_gpu.log
[ $rc -ne 0 ] && stop pytest $rc
for fe in gpu host; do
  timeout -k 10 300 python bench.py --mode file --config f2 --frontend $fe --sink device > $O/f2_$fe.json 2>$O/f2_$fe.err || stop f2_$fe $?
  echo "f2 $fe $(python -c "import json; d=json.loads(open('$O/f2_$fe.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['parity_verified'])")"
done
for b in c1s c2s c3s; do
  timeout -k 10 300 python bench.py --config ${b%s} --mode stream --steps 20 > $O/${b}.json 2>$O/${b}.err || stop $b $?
  echo "$b $(python -c "import json; d=json.loads(open('$O/${b}.json').read().strip().splitlines()[-1]); print(d['roofline']['frac'], d['parity_verified'], d['stream_reruns'])")"
done
echo "r03_check5 done"
