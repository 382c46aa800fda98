#!/bin/bash
# GPU box: stream-kernel tail experiment -- per-frame time vs frame count (jobs/slots rounding).
export TMPDIR=/tmp
O=gpurun_out/r02t; mkdir -p $O
for g in "420 1920 1080 240" "420 1920 1080 300" "420 1920 1080 360" "420 3840 2160 288" "420 3840 2160 300" "420 3840 2160 312"; do
    PROBE_GOP=24 timeout -k 10 200 ./tools/probe $g 5 > "$O/probe_${g// /_}.txt" 2>&1 || { cat "$O/probe_${g// /_}.txt"; exit 1; }
    echo "== $g"; grep "production\|static" "$O/probe_${g// /_}.txt"
done
