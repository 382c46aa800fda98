#!/bin/bash
# GPU box: stream-kernel parity tests, then the stream-kernel probe at the BASELINE geometries.
export TMPDIR=/tmp
O=gpurun_out/r02s; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "stream or gop or mpg or pipeline" > $O/pytest_stream.log 2>&1 || { tail -40 $O/pytest_stream.log; exit 1; }
tail -2 $O/pytest_stream.log
for g in "420 3840 2160 300" "420 1920 1080 300" "444 640 480 300" "422 7680 4320 15" "444 1920 1080 240"; do
    PROBE_GOP=24 timeout -k 10 200 ./tools/probe $g 5 > "$O/probe_gop_${g// /_}.txt" 2>&1 || { cat "$O/probe_gop_${g// /_}.txt"; exit 1; }
    echo "== $g"; grep -v "^copy\|only" "$O/probe_gop_${g// /_}.txt"
done
