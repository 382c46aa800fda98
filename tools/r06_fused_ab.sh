#!/bin/bash
# Round 6: the fused .mpg kernel with column-major dequantized slots -- its parity tests, then the
# whole-file decode A/B against the round's base build (one process per run, interleaved rounds), and
# a kernel trace of the new build.
set -o pipefail
O=gpurun_out/r06/${TAG:-fused}; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 250 --timeout-method thread \
  -k "entropy_decode or block_of_more or any_frame_size or bounds or reference_bmps or decode_file" > $O/pytest.log 2>&1 \
  || { echo STOP pytest; grep -E "FAIL|Error|passed|failed" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
ROUNDS=${ROUNDS:-3} bash tools/file_ab_proc.sh ${AB_LIBS:-tools/variants/r6base/libmj423gpu.so tools/variants/r6fused/libmj423gpu.so} || exit 1
cp gpurun_out/file_ab/all.log $O/file_ab.log
OUT=r06/${TAG:-fused}/file KT_ONLY=1 bash tools/file_trace.sh || exit 1
python tools/kt_summary.py gpurun_out/r06/${TAG:-fused}/file/kt 20 > $O/file/kt_summary.txt; head -3 $O/file/kt_summary.txt
