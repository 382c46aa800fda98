#!/bin/bash
# GPU box: front-end tests, per-pass wall times of the whole-GPU .mpg decode (twice), and
# one pass series under a kernel + memory-copy + HIP-runtime trace.
export TMPDIR=/tmp
O=gpurun_out/r02f; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_frontend.py -x -q --timeout 120 --timeout-method thread -m gpu -k "gpu or mpg or frontend" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for i in 1 2 3; do
timeout -k 10 200 python tools/fe_pass_times.py 100 > $O/plain$i.txt 2>&1 || { cat $O/plain$i.txt; exit 1; }
tail -1 $O/plain$i.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace -d $O/trace -o fe --output-format csv -- python3 tools/fe_pass_times.py 60 > $O/traced.txt 2>&1 || { tail -20 $O/traced.txt; exit 1; }
grep -v "^W20\|^E20\|amdgpu.ids" $O/traced.txt | tail -1
