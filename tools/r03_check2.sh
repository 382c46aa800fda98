#!/bin/bash
# Round-3 check after the stream-kernel prefetch fix and the 4:2:2 optimistic kernel: GPU suite,
# smoke, benches for every config (batch and stream), the phase trace.
mkdir -p gpurun_out/check2 && export TMPDIR=/tmp
O=gpurun_out/check2
stop() { echo "STOP: $1 rc=$2"; exit "$2"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; tail -3 $O/pytest_gpu.log
[ $rc -ge 124 ] && stop pytest $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || stop smoke $?
tail -1 $O/smoke.log
for b in c3 c2 c5 c1 c3s c2s c5s c1s; do
  cfg=${b%s}; args="--config $cfg"; [ "$b" != "$cfg" ] && args="$args --mode stream"
  timeout -k 10 300 python bench.py $args --steps 20 > $O/${b}_bench.log 2>&1 || stop bench_$b $?
  echo "$b $(python -c "import json; d=json.loads(open('$O/${b}_bench.log').read().strip().splitlines()[-1]); print(d['roofline']['frac'], d['parity_verified'], d['ms_per_step'], d['value'])")"
done
for m in "444 640 480 300" "420 3840 2160 300"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_TRACE=1 PROBE_DELTAS=1 timeout -k 10 120 ./tools/probe $m > $O/trace_$1_$2.log 2>&1 || stop trace $?
  grep trace $O/trace_$1_$2.log
done
echo "r03_check2 done"
