#!/bin/bash
# Round 6: fused-path parity, A/B of the latest fused build against the previous one, then the
# upload-window schedules on the latest build (one process per run).
set -o pipefail
O=gpurun_out/r06/${TAG:-sweep}; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 250 --timeout-method thread \
  -k "entropy_decode or block_of_more or any_frame_size or bounds or reference_bmps or decode_file" > $O/pytest.log 2>&1 \
  || { echo STOP pytest; grep -E "FAIL|Error|passed|failed" $O/pytest.log | head -20; exit 1; }
tail -1 $O/pytest.log
rm -f gpurun_out/file_ab/all.log
ROUNDS=${ROUNDS:-3} bash tools/file_ab_proc.sh $AB_LIBS || exit 1
cp gpurun_out/file_ab/all.log $O/file_ab.log
if [ -n "$WINDOWS" ]; then ROUNDS=2 bash tools/win_ab.sh $WINDOWS > $O/windows.log 2>&1 || { echo STOP windows; tail -3 $O/windows.log; exit 1; }; cat $O/windows.log; fi
