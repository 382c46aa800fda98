#!/bin/bash
mkdir -p gpurun_out/win
[ -n "$NOTEST" ] || timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "upload_windows or mixed_static or entropy" > gpurun_out/win/pytest.log 2>&1 || { tail -20 gpurun_out/win/pytest.log; exit 1; }
[ -n "$NOTEST" ] || tail -2 gpurun_out/win/pytest.log
for r in ${ROUNDS:-1 2}; do
  for wv in ${WV:-2 1,2,3 1,2,4 1,2,3,4 1,1,2,4}; do
    MJ423_GPU_FE_WINDOWS=$wv timeout -k 10 200 python bench.py --mode file --config f2 --frontend gpu --steps 10 --warmup 2 --no-cpu --no-verify > gpurun_out/win/b_${wv}_$r.json 2>gpurun_out/win/b_${wv}_$r.err || exit 1
    python -c "import json,sys;d=json.loads(open('gpurun_out/win/b_${wv}_$r.json').read().strip().splitlines()[-1]);print('$wv r$r', d['value'], d['ms_per_step'])"
  done
done
