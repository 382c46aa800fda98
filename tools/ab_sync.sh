#!/bin/bash
# GPU front end: parity of the whole-GPU decode tests (MJ423_ENTPAR_LEAD: lead-in bits of an
# experimental build, ignored otherwise), then interleaved
# end-to-end A/B of library variants x lead-in (GPU box).  VARIANTS="name:lead ..." where
# name "cur" is the in-tree library, anything else tools/variants/<name>.
mkdir -p gpurun_out/sync
for L in ${TEST_LEADS:-0}; do
  MJ423_ENTPAR_LEAD=$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 \
    --timeout-method thread -k "gpu_entropy or mjpeg423_decode_file or seek_into_gop" > gpurun_out/sync/pytest_$L.log 2>&1 \
    || { tail -30 gpurun_out/sync/pytest_$L.log; exit 1; }
  echo "lead $L: $(tail -1 gpurun_out/sync/pytest_$L.log)"
done
for r in ${ROUNDS:-1 2}; do
  for v in ${VARIANTS:-base:0 cur:0}; do
    n=${v%%:*}; L=${v##*:}; lib=""
    [ "$n" != cur ] && lib=tools/variants/$n/libmj423gpu.so
    f=gpurun_out/sync/b_${n}_${L}_$r.json
    MJ423_LIB=$lib MJ423_ENTPAR_LEAD=$L timeout -k 10 200 python bench.py --mode file --config f2 --frontend gpu \
      --steps 10 --warmup 2 --no-cpu --no-verify > $f 2> ${f%.json}.err || exit 1
    python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$n lead $L r$r', d['value'], d['ms_per_step'])"
  done
done
if [ -n "$PROF" ]; then
  export TMPDIR=/tmp
  for v in $PROF; do
    n=${v%%:*}; L=${v##*:}; lib=""
    [ "$n" != cur ] && lib=tools/variants/$n/libmj423gpu.so
    MJ423_LIB=$lib MJ423_ENTPAR_LEAD=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/sync/kt_${n}_$L -o kt \
      --output-format csv -- python bench.py --mode file --config f2 --frontend gpu --steps 3 --warmup 1 --no-cpu --no-verify \
      > gpurun_out/sync/kt_${n}_$L.log 2>&1 || exit 1
  done
fi
