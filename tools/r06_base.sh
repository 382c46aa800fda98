set -o pipefail
mkdir -p gpurun_out/r06/base && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 250 --timeout-method thread -k "bounds or dropin_adaptive" > gpurun_out/r06/base/pytest_new.log 2>&1 || { echo STOP pytest; tail -20 gpurun_out/r06/base/pytest_new.log; exit 1; }
tail -2 gpurun_out/r06/base/pytest_new.log
OUT=r06/base/file KT_ONLY=1 bash tools/file_trace.sh || exit 1
python tools/kt_summary.py gpurun_out/r06/base/file/kt 20 > gpurun_out/r06/base/file/kt_summary.txt
timeout -k 10 300 python bench.py --steps 20 > gpurun_out/r06/base/c3_bench.log 2>&1 || { echo STOP c3; exit 1; }
tail -1 gpurun_out/r06/base/c3_bench.log | cut -c1-300
