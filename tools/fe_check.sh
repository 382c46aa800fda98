#!/bin/bash
# GPU entropy front end round check (GPU box): the GPU test suite (SKIP_TESTS=1 skips it), a
# same-process A/B of the whole-file GPU decode against AB_LIBS (default tools/variants/base),
# then tools/file_trace.sh (bench line, convergence log, kernel + copy trace, FETCH/WRITE passes).
mkdir -p gpurun_out && export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log
  [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
fi
timeout -k 10 300 python tools/ab_file.py ${AB_ROUNDS-5} -- ${AB_LIBS-tools/variants/base/libmj423gpu.so} mjpeg423-video-decoder-software_amd/libmj423gpu.so@MJ423_GPU_FE_FUSED=0 mjpeg423-video-decoder-software_amd/libmj423gpu.so@MJ423_FUSED_PREFETCH=0 mjpeg423-video-decoder-software_amd/libmj423gpu.so > gpurun_out/ab_file.log 2>&1 || { echo "STOP ab"; tail -5 gpurun_out/ab_file.log; exit 1; }
cat gpurun_out/ab_file.log
[ -n "$NO_TRACE" ] && exit 0
bash tools/file_trace.sh
