#!/bin/bash
# GPU box: per-block symbol tests, then their cost per call and per 640x480 frame:
# round-1 library (tools/variants/dropin_r1), this tree, this tree with deferred idct().
export TMPDIR=/tmp
O=gpurun_out/r02d; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -k "symbol or dropin or accel" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
LD_LIBRARY_PATH=tools/variants/dropin_r1 timeout -k 10 300 ./tools/dropin_bench 2 > $O/r1.json 2>&1 || { cat $O/r1.json; exit 1; }
cat $O/r1.json
MJ423_DROPIN_DEFER=0 timeout -k 10 300 ./tools/dropin_bench 3 > $O/now.json 2>&1 || { cat $O/now.json; exit 1; }
cat $O/now.json
MJ423_DROPIN_DEFER=1 timeout -k 10 300 ./tools/dropin_bench 3 > $O/defer.json 2>&1 || { cat $O/defer.json; exit 1; }
cat $O/defer.json
mkdir -p /tmp/d0 /tmp/d1
for d in 0 1; do
  s=$(date +%s.%N)
  MJ423_DROPIN_DEFER=$d timeout -k 10 300 ./oracle/_ref/mjdrop_blocks tests/golden/stream_320x240.mpg /tmp/d$d/x0000.bmp || exit 1
  e=$(date +%s.%N)
  echo "mjdrop_blocks 320x240 x30 frames (incl. BMP writes), defer=$d: $(python3 -c "print(round($e - $s, 3))") s" >> $O/mjdrop.txt
done
cat $O/mjdrop.txt
