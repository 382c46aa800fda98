#!/bin/bash
# GPU-box round check: parity tests, smoke, benches for each BASELINE config, rocprofv3
# kernel trace + separate PMC passes for the headline config.  Every GPU step has its
# own time limit; a fault/abort/timeout ends the script (no retries).
mkdir -p gpurun_out && export TMPDIR=/tmp
stop() { echo "STOP: $1 rc=$2"; exit "$2"; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -ge 124 ] && stop pytest $rc
  timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || stop smoke $?
  cat gpurun_out/smoke.log | tail -1
fi
for b in ${CONFIGS-c3 c2 c5 c1 c3s c2s c5s c1s}; do
  cfg=${b%s}; args="--config $cfg"; [ "$b" != "$cfg" ] && args="$args --mode stream"
  timeout -k 10 300 python bench.py $args --steps 20 > gpurun_out/bench_$b.log 2>&1 || stop bench_$b $?
  tail -1 gpurun_out/bench_$b.log
done
# PROFILE="c3 c3s": rocprofv3 kernel trace + separate FETCH_SIZE / WRITE_SIZE passes per
# entry (KT_ONLY=1: the kernel trace only); a trailing "s" profiles the stream (GOP) mode.
for pr in ${PROFILE}; do
  cfg=${pr%s}; args="--config $cfg"; [ "$pr" != "$cfg" ] && args="$args --mode stream"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${pr}_kt -o kt --output-format csv -- python bench.py $args --steps 10 --no-cpu --no-verify > gpurun_out/prof_${pr}_kt.log 2>&1 || stop prof_kt_$pr $?
  if [ -n "$KT_ONLY" ]; then echo "profile $pr (kernel trace) done"; continue; fi
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/prof_${pr}_fetch -o f --output-format csv -- python bench.py $args --steps 3 --warmup 1 --no-cpu --no-verify > gpurun_out/prof_${pr}_fetch.log 2>&1 || stop prof_fetch_$pr $?
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/prof_${pr}_write -o w --output-format csv -- python bench.py $args --steps 3 --warmup 1 --no-cpu --no-verify > gpurun_out/prof_${pr}_write.log 2>&1 || stop prof_write_$pr $?
  echo "profile $pr done"
done
echo "gpu_check done"
