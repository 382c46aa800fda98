#!/bin/bash
# Round GPU check: the whole GPU suite (BASELINE configs first, per-test time limit),
# smoke, then the benches named in CONFIGS (default: c3 and the 640x480 4:4:4 stream).
# Every GPU step has its own limit; a timeout/abort ends the script (no retries).
mkdir -p gpurun_out && export TMPDIR=/tmp
stop() { echo "STOP: $1 rc=$2"; exit "$2"; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
[ $rc -ge 124 ] && stop pytest $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || stop smoke $?
tail -1 gpurun_out/smoke.log
for b in ${CONFIGS-c3 c1s}; do
  cfg=${b%s}; args="--config $cfg"; [ "$b" != "$cfg" ] && args="$args --mode stream"
  timeout -k 10 300 python bench.py $args --steps 20 > gpurun_out/bench_$b.log 2>&1 || stop bench_$b $?
  tail -1 gpurun_out/bench_$b.log
done
echo "round_check done"
