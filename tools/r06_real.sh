#!/bin/bash
# Round 6: the whole-file GPU decode on reference-encoded 1080p files (tools/real_mpg.py: clean,
# static with sensor noise, panning; 24 frames, one GOP each): convergence per window
# (MJ423_ENTPAR_DEBUG, the -DMJ423_SYNC_COUNT build) and pass time per build in $REAL_LIBS.
set -o pipefail
O=gpurun_out/r06/real; mkdir -p $O && export TMPDIR=/tmp
for f in clean static pan; do
  MJ423_LIB=tools/variants/r6count/libmj423gpu.so MJ423_ENTPAR_DEBUG=1 AB_FILE=realdata/${f}_1080p.mpg \
    timeout -k 10 120 python tools/ab_file.py 1 -- tools/variants/r6count/libmj423gpu.so > $O/debug_$f.log 2>&1 || { echo STOP debug $f; tail -5 $O/debug_$f.log; exit 1; }
  echo "== $f"; grep "entpar: window" $O/debug_$f.log | head -4
done
rm -f $O/time_*.log
for r in 1 2; do
  for f in clean static pan; do
    for l in $REAL_LIBS; do  # one process per build (several contexts in one process share hardware queues)
      AB_FILE=realdata/${f}_1080p.mpg timeout -k 10 300 python tools/ab_file.py 3 -- $l > $O/t.log 2>&1 || { echo STOP time $f $l; tail -5 $O/t.log; exit 1; }
      grep "^file" $O/t.log | sed "s|^|round $r $f: |" | tee -a $O/time_$f.log
    done
  done
done
