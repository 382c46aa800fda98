#!/bin/bash
# GPU box: stream-kernel time vs GOP length (1 = every frame an I-frame: one frame per workgroup).
export TMPDIR=/tmp
O=gpurun_out/r02g; mkdir -p $O
for gop in 1 2 4 8 24 300; do
    PROBE_GOP=$gop timeout -k 10 200 ./tools/probe 420 3840 2160 300 5 > "$O/probe_gop$gop.txt" 2>&1 || { cat "$O/probe_gop$gop.txt"; exit 1; }
    echo "== gop $gop"; grep "production\|static\|r1" "$O/probe_gop$gop.txt"
done
