#!/bin/bash
# LDS-DMA stream kernel (decode_gop_dma_kernel, MJ423_GOP_DMA=1|2) against the production stream
# kernels: parity of the stream tests under each form, then interleaved bench rounds per config
# (GPU box).  Every GPU step has its own limit; a fault/abort/timeout ends the script.
mkdir -p gpurun_out/dma && export TMPDIR=/tmp
stop() { echo "STOP: $1 rc=$2"; exit "$2"; }
for form in ${FORMS-2 1}; do
  MJ423_GOP_DMA=$form timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -v --timeout 120 \
    --timeout-method thread -k "stream or gop or pipelin or mpg or extreme or entropy" > gpurun_out/dma/pytest_form$form.log 2>&1
  rc=$?; tail -3 gpurun_out/dma/pytest_form$form.log; grep -E "^FAILED|Error" gpurun_out/dma/pytest_form$form.log | head -20
  [ $rc -ge 124 ] && stop pytest_form$form $rc
done
for round in ${ROUNDS-1 2}; do
  for b in ${CONFIGS-c3 c2 c1 c5}; do
    for form in 0 ${FORMS-2 1}; do
      MJ423_GOP_DMA=$form timeout -k 10 200 python bench.py --config $b --mode stream --steps 20 --no-cpu --verify ends \
        > gpurun_out/dma/bench_${b}_f${form}_r$round.log 2>&1 || stop bench_${b}_$form $?
      python - "$b" "$form" gpurun_out/dma/bench_${b}_f${form}_r$round.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[1]} form {sys.argv[2]}: frac {r['frac']:.4f} median {r['frac_median']:.4f} kernel_ms {r['kernel_ms_avg']} "
      f"parity {d['parity_verified']} reruns {d.get('stream_reruns')}", flush=True)
PY
    done
  done
done
echo "ab_dma done"
