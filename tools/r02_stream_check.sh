#!/bin/bash
# GPU box: stream-kernel parity (GOP streams at every size, BASELINE sizes, front end), then the
# prefetch-placement probe once more.
export TMPDIR=/tmp
O=gpurun_out/r02sc; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "stream or gop or mpg or pipeline or gpu_entropy" > $O/pytest_stream.log 2>&1 || { tail -40 $O/pytest_stream.log; exit 1; }
tail -2 $O/pytest_stream.log
bash tools/r02_noprefetch.sh
