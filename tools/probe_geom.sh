#!/bin/bash
# Geometry sweep for the 4:2:0 ceiling (run on the GPU box): does the C2 vs C3 gap follow
# frame size, batch length or output row stride?
set -o pipefail
mkdir -p gpurun_out
run() { echo "== $*"; timeout -k 10 200 env "$@" || exit $?; }
{
run PROBE_COPY=1 ./tools/probe 420 1920 1080 300 5
run ./tools/probe 420 1920 1080 1200 5
run PROBE_PITCH=2048 ./tools/probe 420 1920 1080 300 5
run ./tools/probe 420 3840 2160 300 5
run PROBE_PITCH=4096 ./tools/probe 420 3840 2160 300 5
} > gpurun_out/probe_geom.txt 2>&1
