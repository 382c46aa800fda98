#!/bin/bash
# A/B of stream-mode benches across tools/variants builds (measurement only).
mkdir -p gpurun_out
for v in default ${VARIANTS}; do
  for cfg in ${CONFIGS:-c3 c2}; do
    if [ $v = default ]; then lib=""; else lib=tools/variants/$v/libmj423gpu.so; fi
    MJ423_LIB=$lib timeout -k 10 200 python bench.py --mode ${MODE:-stream} --no-cpu --config $cfg > gpurun_out/ab_${v}_$cfg.log 2>&1 || { echo "FAIL $v $cfg"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/ab_${v}_$cfg.log').read().strip().splitlines()[-1]); print('$v $cfg', d['value'], d['roofline']['frac'], d['parity_verified'])"
  done
done
