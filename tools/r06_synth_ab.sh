#!/bin/bash
# Round 6: synthetic whole-file A/B only (one process per build, $ROUNDS interleaved rounds) of $LIBS.
set -o pipefail
O=gpurun_out/r06/synth_ab; mkdir -p $O && export TMPDIR=/tmp
rm -f gpurun_out/file_ab/all.log
ROUNDS=${ROUNDS:-5} bash tools/file_ab_proc.sh $LIBS || exit 1
cp gpurun_out/file_ab/all.log $O/${TAG:-ab}.log
