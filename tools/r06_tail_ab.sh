#!/bin/bash
# Round 6: iteration-0 tail walks of the synchronisation (MJ423_SYNC_TAIL_BYTES builds): parity of each
# build on the whole-file tests, convergence (MJ423_ENTPAR_DEBUG), then the whole-file A/B.
set -o pipefail
O=gpurun_out/r06/tail; mkdir -p $O && export TMPDIR=/tmp
for v in $VARIANTS; do
  MJ423_LIB=tools/variants/$v/libmj423gpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread \
    -k "entropy_decode or block_of_more or any_frame_size or reference_bmps" > $O/pytest_$v.log 2>&1 || { echo STOP pytest $v; tail -20 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
  MJ423_LIB=tools/variants/$v/libmj423gpu.so MJ423_ENTPAR_DEBUG=1 timeout -k 10 120 python bench.py --mode file --config f2 --frontend gpu --steps 1 --warmup 0 --no-cpu --no-verify > $O/debug_$v.log 2>&1 || { echo STOP debug $v; exit 1; }
  grep "entpar: window" $O/debug_$v.log | head -3
done
rm -f gpurun_out/file_ab/all.log
ROUNDS=${ROUNDS:-3} bash tools/file_ab_proc.sh $(for v in $VARIANTS; do echo tools/variants/$v/libmj423gpu.so; done) || exit 1
cp gpurun_out/file_ab/all.log $O/file_ab.log
