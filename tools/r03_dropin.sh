#!/bin/bash
# Round 3: per-block drop-in -- its GPU tests, then tools/dropin_bench.c through the library
# (immediate and deferred) and through the reference's own C on the same host.
mkdir -p gpurun_out/dropin && export TMPDIR=/tmp
O=gpurun_out/dropin
timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread \
  -k "symbol or dropin or accelerator or accel" > $O/pytest.log 2>&1; rc=$?
tail -3 $O/pytest.log; [ $rc -ge 124 ] && exit $rc
timeout -k 10 120 ./oracle/_ref/dropin_bench_ref 50 > $O/ref.json 2>&1 || { cat $O/ref.json; exit 1; }
MJ423_DROPIN_DEFER=1 timeout -k 10 120 ./oracle/_ref/dropin_bench 50 > $O/defer.json 2>&1 || { cat $O/defer.json; exit 1; }
MJ423_DROPIN_DEFER=0 timeout -k 10 120 ./oracle/_ref/dropin_bench 3 > $O/now.json 2>&1 || { cat $O/now.json; exit 1; }
cat $O/ref.json $O/defer.json $O/now.json
