#!/bin/bash
# GPU box: the whole GPU suite, then stream-kernel probes (args: geometries as "mode w h frames").
export TMPDIR=/tmp
O=gpurun_out/r02p; mkdir -p $O
if [ -z "$NOTEST" ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
fi
for g in "$@"; do
    PROBE_GOP=${GOP:-24} timeout -k 10 200 ./tools/probe $g 5 > "$O/probe_gop_${g// /_}.txt" 2>&1 || { cat "$O/probe_gop_${g// /_}.txt"; exit 1; }
    echo "== $g"; grep -v "^copy" "$O/probe_gop_${g// /_}.txt"
done
