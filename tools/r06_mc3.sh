#!/bin/bash
# Round 6: multi-class resolution variants -- whole-file parity subset, the reference-encoded files
# (24 frames, one process per build), the 240-frame clean scene, synthetic A/B ($LIBS; first = base).
set -o pipefail
O=gpurun_out/r06/mc3; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "static_scene or entropy_decode or block_of_more or any_frame_size or reference_bmps or bounds_checks" > $O/pytest.log 2>&1 || { echo STOP pytest; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
REAL_LIBS="$LIBS" bash tools/r06_real.sh > $O/real.log 2>&1 || { echo STOP real; tail -5 $O/real.log; exit 1; }
grep "fallback" $O/real.log | head -6
cp gpurun_out/r06/real/time_*.log $O/
for l in $LIBS; do
  p=${l%%@*}; v=""; [ "$p" != "$l" ] && v=${l#*@}
  env $v MJ423_LIB=$p timeout -k 10 300 python bench.py --mode file --frontend gpu --mpg realdata/clean_1080p_240.mpg --steps 20 --no-cpu > $O/c240.log 2>&1 || { echo STOP c240 $l; tail -5 $O/c240.log; exit 1; }
  echo "clean240 $l: $(tail -1 $O/c240.log | grep -o '"ms_per_step": [0-9.]*')" | tee -a $O/clean240.log
done
rm -f gpurun_out/file_ab/all.log
ROUNDS=3 bash tools/file_ab_proc.sh $LIBS || exit 1
cp gpurun_out/file_ab/all.log $O/file_ab.log
