#!/bin/bash
# Round 3: the two multi-GPU configurations at their full size on ONE GPU (the N = 1 points of their
# curves): SURVEY §8(d) C4 = 2400 4K 4:2:0 frames (strong scaling total), C5 = 120 8K 4:2:2 frames
# (8 x 15); batch and I/P stream (GOP 24), every frame checked against the oracle after timing.
mkdir -p gpurun_out/fullsize && export TMPDIR=/tmp
O=gpurun_out/fullsize
stop() { echo "STOP: $1 rc=$2"; exit "$2"; }
for m in ${MODES-batch stream}; do
  timeout -k 10 400 python bench.py --config c3 --total-frames 2400 --mode $m --steps 10 --cpu-seconds 6 > $O/c4_$m.log 2>&1 || stop c4_$m $?
  tail -1 $O/c4_$m.log
  timeout -k 10 300 python bench.py --config c5 --frames 120 --mode $m --steps 20 --cpu-seconds 6 > $O/c5x120_$m.log 2>&1 || stop c5_$m $?
  tail -1 $O/c5x120_$m.log
done
echo "r03_fullsize done"
