#!/bin/bash
# Round 3: int16-workspace IDCT + 16-bit CSC -- GPU suite, A/B probe (same process) against
# the round-2 forms, benches.  Limits per step; stop at the first timeout/abort.
mkdir -p gpurun_out/idct && export TMPDIR=/tmp
O=gpurun_out/idct
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for m in "420 3840 2160 300" "444 640 480 300" "420 1920 1080 300" "422 7680 4320 15"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 timeout -k 10 240 ./tools/probe $m 9 > $O/probe_$1_$2.log 2>&1 || { cat $O/probe_$1_$2.log; exit 1; }
  grep -E "round|IDCT|CSC" $O/probe_$1_$2.log
done
for b in c3 c1s c3s c2s; do
  cfg=${b%s}; args="--config $cfg"; [ "$b" != "$cfg" ] && args="$args --mode stream"
  timeout -k 10 300 python bench.py $args --steps 20 > $O/bench_$b.log 2>&1 || { tail -5 $O/bench_$b.log; exit 1; }
  tail -1 $O/bench_$b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$b', d['value'], d['roofline']['frac'], d['parity_verified'])"
done
