# Full GPU suite, then tools/file_trace.sh (GPU box).
mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
bash tools/file_trace.sh
