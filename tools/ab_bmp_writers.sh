#!/bin/bash
# GPU box, measurements only: mjpeg423_decode (oracle/_ref/mjdrop_file) with 4 / 8 (default) / 16
# BMP writer threads -- library builds tools/variants/w4, the default, tools/variants/w16
# (tools/build_variant.sh NAME -DMJ423_BMP_WRITERS=n) picked by LD_LIBRARY_PATH (the binary's
# RUNPATH yields to it) -- interleaved, REPS rounds, on seeded synthetic files.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/writers
W=/tmp/mj423_writers; rm -rf $W; mkdir -p $W
python -c "import sys; sys.path.insert(0, 'tools'); import mpg_synth; mpg_synth.build(); mpg_synth.write('$W/a.mpg', 1920, 1080, 240, gop=24); mpg_synth.write('$W/b.mpg', 640, 480, 240, gop=24)" || exit 1
for r in $(seq ${REPS:-3}); do
  for f in a b; do
    for v in w4 default w16; do
      lp=""; [ $v != default ] && lp=tools/variants/$v
      rm -rf $W/o; mkdir -p $W/o
      t0=$(date +%s%N)
      LD_LIBRARY_PATH=$lp timeout -k 10 120 oracle/_ref/mjdrop_file $W/$f.mpg $W/o/d0000.bmp 2>/dev/null || { echo "STOP $v $f"; exit 1; }
      t1=$(date +%s%N)
      echo "$f $v $(( (t1 - t0) / 1000 ))" | tee -a gpurun_out/writers/times.txt
    done
  done
done
rm -rf $W
