#!/bin/bash
# Round 6: the synchronisation's list iterations (work-list layout A/B) -- parity (whole-file tests,
# bounds build), convergence and pass time on the reference-encoded files, synthetic A/B ($LIBS).
set -o pipefail
O=gpurun_out/r06/qlist; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "static_scene or entropy_decode or block_of_more or any_frame_size or reference_bmps or bounds_checks" > $O/pytest.log 2>&1 || { echo STOP pytest; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
P=mjpeg423-video-decoder-software_amd/libmj423gpu.so
B=tools/variants/r6mc/libmj423gpu.so
REAL_LIBS="${LIBS:-$B $P}" bash tools/r06_real.sh || exit 1
cp gpurun_out/r06/real/* $O/
rm -f gpurun_out/file_ab/all.log
ROUNDS=3 bash tools/file_ab_proc.sh ${LIBS:-$B $P} || exit 1
cp gpurun_out/file_ab/all.log $O/file_ab.log
