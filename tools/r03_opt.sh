#!/bin/bash
# Round 3: the optimistic stream kernel (int8 state, int16 IDCT with escape, six workgroups per CU)
# plus the exact re-run of marked jobs, against production: outputs compared first (real P-frame
# deltas, then absolute frames fed as deltas so that nearly every job is marked), then timed in
# one process; then the library path (bench.py --mode stream) with the optimistic form on and off.
mkdir -p gpurun_out/opt && export TMPDIR=/tmp
O=gpurun_out/opt
for m in "444 640 480 300 200" "420 1920 1080 300 60" "420 3840 2160 300 20" "422 7680 4320 15 60" "444 1920 1080 300 40"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_OPT=1 PROBE_DELTAS=1 PROBE_WARM_S=1.5 timeout -k 10 240 ./tools/probe $m > $O/$1_$2.log 2>&1 || { cat $O/$1_$2.log; exit 1; }
  echo "== $1 $2x$3"; grep -E "optimistic|production|re-run" $O/$1_$2.log
done
PROBE_R03=1 PROBE_GOP=24 PROBE_OPT=1 timeout -k 10 240 ./tools/probe 420 1920 1080 60 5 > $O/abs_420_1920.log 2>&1 || { cat $O/abs_420_1920.log; exit 1; }
echo "== absolute frames as deltas"; grep -E "optimistic|production|re-run" $O/abs_420_1920.log
for b in c3 c2 c1 c5; do
  for opt in 1 0; do
    MJ423_GOP_OPT=$opt timeout -k 10 300 python bench.py --config $b --mode stream --steps 20 > $O/bench_${b}s_opt$opt.log 2>&1 || { tail -5 $O/bench_${b}s_opt$opt.log; exit 1; }
    echo "bench $b stream opt=$opt: $(python -c "import json,sys; d=json.loads(open('$O/bench_${b}s_opt$opt.log').read().strip().splitlines()[-1]); print(d['roofline']['frac'], d['parity_verified'], d['ms_per_step'])")"
  done
done
echo "r03_opt done"
