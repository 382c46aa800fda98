#!/bin/bash
# Round 6: bench.py's whole-file line on the reference-encoded 1080p files (tools/real_mpg.py; made in
# the build container, not committed), with the reference-loop CPU baseline.
set -o pipefail
O=gpurun_out/r06/real_bench; mkdir -p $O && export TMPDIR=/tmp
for f in clean static pan; do
  timeout -k 10 300 python bench.py --mode file --frontend gpu --mpg realdata/${f}_1080p.mpg --steps 20 > $O/${f}_bench.log 2>&1 || { echo STOP $f; tail -5 $O/${f}_bench.log; exit 1; }
  tail -1 $O/${f}_bench.log | cut -c1-160
done
