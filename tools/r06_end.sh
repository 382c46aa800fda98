#!/bin/bash
# Round 6 end-of-round evidence: the full GPU suite, smoke(), C3 and whole-file bench lines
# (tools/r06_final.sh), then 600 damaged streams through the bounds-check build.
set -o pipefail
TAG=${TAG:-end} bash tools/r06_final.sh || exit 1
O=gpurun_out/r06/${TAG:-end}; mkdir -p $O/fz && export TMPDIR=/tmp
MJ423_LIB=mjpeg423-video-decoder-software_amd/libmj423gpu_bounds.so MJ423_BOUNDS_FUZZ=600 timeout -k 10 600 python -u tests/bounds_child.py $O/fz > $O/bounds_fuzz600.log 2>&1 || { echo STOP fuzz; tail -5 $O/bounds_fuzz600.log; exit 1; }
rm -rf $O/fz
tail -1 $O/bounds_fuzz600.log
