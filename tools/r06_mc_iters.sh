#!/bin/bash
# Round 6: synchronisation iterations before the multi-class resolution, on the synthetic bench file
# (one process per run) and the reference-encoded files.
set -o pipefail
O=gpurun_out/r06/mc_iters; mkdir -p $O && export TMPDIR=/tmp
P=mjpeg423-video-decoder-software_amd/libmj423gpu.so
SET="$P $P@MJ423_GPU_FE_ITERS=7 $P@MJ423_GPU_FE_ITERS=5 $P@MJ423_GPU_FE_ITERS=4"
for f in clean static pan; do
  AB_FILE=realdata/${f}_1080p.mpg timeout -k 10 300 python tools/ab_file.py 3 -- $SET > $O/time_$f.log 2>&1 || { echo STOP time $f; tail -5 $O/time_$f.log; exit 1; }
  grep "^file" $O/time_$f.log
done
rm -f gpurun_out/file_ab/all.log
ROUNDS=${ROUNDS:-3} bash tools/file_ab_proc.sh $SET || exit 1
cp gpurun_out/file_ab/all.log $O/file_ab.log
