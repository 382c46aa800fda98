#!/bin/bash
# A/B of an environment switch on stream-mode benches, interleaved rounds (GPU box).
#   AB_VAR=MJ423_GOP_XCD CONFIGS="c3 c2" ROUNDS=2 tools/ab_env.sh
mkdir -p gpurun_out
var=${AB_VAR:-MJ423_GOP_XCD}
for r in $(seq ${ROUNDS:-2}); do
  for val in ${VALS:-0 1}; do
    for cfg in ${CONFIGS:-c3 c2}; do
      env $var=$val timeout -k 10 200 python bench.py --mode ${MODE:-stream} --no-cpu --verify ends --config $cfg ${BENCH_ARGS} > gpurun_out/abenv.log 2>&1 || { echo "FAIL $val $cfg"; tail -5 gpurun_out/abenv.log; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/abenv.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$var=$val $cfg', d['value'], r['frac'], r['frac_median'], d['parity_verified'])"
    done
  done
done
