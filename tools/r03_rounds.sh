#!/bin/bash
# Round 3: priority by frames left against production as a function of the grid's rounds of
# resident workgroups (1080p 4:4:4: 510 jobs per GOP of 24 frames, 1 024 resident workgroups).
mkdir -p gpurun_out/rounds && export TMPDIR=/tmp
O=gpurun_out/rounds
for nf in 48 72 96 144 240; do
  PROBE_R03=1 PROBE_GOP=24 PROBE_OPT=1 PROBE_DELTAS=1 PROBE_WARM_S=1.0 timeout -k 10 240 ./tools/probe 444 1920 1080 $nf 60 > $O/opt_444_1920_$nf.log 2>&1 || { cat $O/opt_444_1920_$nf.log; exit 1; }
  echo "== 1080p 4:4:4 x $nf"; grep -E "\(production\)|priority by frames left  " $O/opt_444_1920_$nf.log | grep -v "vs production"
done
for nf in 48 96 144; do
  PROBE_R03=1 PROBE_GOP=24 PROBE_OPT=1 PROBE_DELTAS=1 PROBE_WARM_S=1.0 timeout -k 10 240 ./tools/probe 420 1920 1080 $nf 60 > $O/opt_420_1920_$nf.log 2>&1 || { cat $O/opt_420_1920_$nf.log; exit 1; }
  echo "== 1080p 4:2:0 x $nf"; grep -E "\(production\)|priority by frames left" $O/opt_420_1920_$nf.log | grep -v "vs production"
done
echo "r03_rounds done"
