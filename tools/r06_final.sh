#!/bin/bash
# Round 6 final-tree evidence: full GPU suite, smoke(), the default bench line (C3), the whole-file line.
set -o pipefail
O=gpurun_out/r06/${TAG:-final}; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $O/pytest_gpu.log; tail -3 $O/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo STOP smoke; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py > $O/c3_bench.log 2>&1 || { echo STOP c3; exit 1; }
tail -1 $O/c3_bench.log | cut -c1-200
timeout -k 10 300 python bench.py --mode file --config f2 --frontend gpu --steps 20 > $O/f2_bench.log 2>&1 || { echo STOP f2; exit 1; }
tail -1 $O/f2_bench.log | cut -c1-200
