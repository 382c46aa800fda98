#!/bin/bash
# Round 6: synchronisation convergence (walks per iteration, -DMJ423_SYNC_COUNT builds, MJ423_ENTPAR_DEBUG)
# on the bench file and the golden files, without and with chain following (MJ423_SYNC_FOLLOW), the
# parity tests on the follow builds, then the whole-file pass A/B.
set -o pipefail
O=gpurun_out/r06/iters; mkdir -p $O && export TMPDIR=/tmp
for v in r6count r6fol16c; do
  L=tools/variants/$v/libmj423gpu.so
  MJ423_LIB=$L MJ423_ENTPAR_DEBUG=1 timeout -k 10 120 python bench.py --mode file --config f2 --frontend gpu --steps 1 --warmup 0 --no-cpu --no-verify > $O/debug_f2_$v.log 2>&1 || { echo STOP debug $v; tail -5 $O/debug_f2_$v.log; exit 1; }
  echo "== $v"; grep "entpar: window" $O/debug_f2_$v.log | head -12
  MJ423_LIB=$L MJ423_ENTPAR_DEBUG=1 timeout -k 10 120 python tools/golden_conv.py > $O/debug_golden_$v.log 2>&1 || { echo STOP golden; tail -5 $O/debug_golden_$v.log; exit 1; }
  grep "entpar: window.*flags\|^file" $O/debug_golden_$v.log | head -24
done
for v in $FOLLOW_TESTS; do
  MJ423_LIB=tools/variants/$v/libmj423gpu.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread \
    -k "entropy_decode or block_of_more or any_frame_size or reference_bmps" > $O/pytest_$v.log 2>&1 || { echo STOP pytest $v; tail -20 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
rm -f gpurun_out/file_ab/all.log
P=mjpeg423-video-decoder-software_amd/libmj423gpu.so
F4=tools/variants/r6fol4/libmj423gpu.so
F16=tools/variants/r6fol16/libmj423gpu.so
ROUNDS=${ROUNDS:-3} bash tools/file_ab_proc.sh $P $P@MJ423_GPU_FE_ITERS=6 $F4 $F16 $F16@MJ423_GPU_FE_ITERS=6 || exit 1
cp gpurun_out/file_ab/all.log $O/file_ab.log
