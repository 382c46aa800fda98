#!/bin/bash
# Round 3: the library with automatic fair priority (one-round stream grids): the stream benches,
# the whole-file paths, then the GPU suite.
mkdir -p gpurun_out/fair2 && export TMPDIR=/tmp
O=gpurun_out/fair2
stop() { echo "STOP: $1 rc=$2"; exit "$2"; }
for b in c1s c2s c3s c5s; do
  for fair in auto 0; do
    e=""; [ $fair != auto ] && e="MJ423_GOP_FAIR=$fair"
    env $e timeout -k 10 300 python bench.py --config ${b%s} --mode stream --steps 20 > $O/${b}_fair$fair.json 2>$O/${b}_fair$fair.err || stop $b $?
    echo "$b fair=$fair $(python -c "import json; d=json.loads(open('$O/${b}_fair$fair.json').read().strip().splitlines()[-1]); print(d['roofline']['frac'], d['parity_verified'], d['ms_per_step'])")"
  done
done
for fe in host gpu; do
  for fair in auto 0; do
    e=""; [ $fair != auto ] && e="MJ423_GOP_FAIR=$fair"
    env $e timeout -k 10 300 python bench.py --mode file --frontend $fe --sink device > $O/file_${fe}_fair$fair.json 2>$O/file_${fe}_fair$fair.err || stop file_$fe $?
    echo "file $fe fair=$fair $(python -c "import json; d=json.loads(open('$O/file_${fe}_fair$fair.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['frac'], d['parity_verified'])")"
  done
done
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $O/pytest_gpu.log
echo "r03_fair2 done"
