#!/bin/bash
# GPU box: buffer placement x workgroup order (XCD-contiguous, frame groups of 8, frame-major),
# batch kernel, 4K 4:2:0, six buffer pairs in one process.
export TMPDIR=/tmp
O=gpurun_out/r02po; mkdir -p $O
PROBE_PAIRS=6 PROBE_PAIRS_ORDERS=1 timeout -k 10 400 ./tools/probe 420 3840 2160 300 5 > "$O/po.txt" 2>&1 || { cat "$O/po.txt"; exit 1; }
grep "pair" "$O/po.txt"
