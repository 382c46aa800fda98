#!/bin/bash
# The multi-rank bench path rehearsed on one GPU: N gloo ranks share the card (MJ423_BENCH_BACKEND=gloo,
# collectives on the host), launched as the driver launches bench.py; the rank-0 JSON line must carry
# cpu_baseline and an attributed roofline.traffic.  Then the per-block drop-in with no environment
# (the default deferred mode) beside the reference's own C.  GPU box.
mkdir -p gpurun_out/gloo && export TMPDIR=/tmp
for n in ${RANKS-2 8}; do
  port=$((29500 + n))
  MJ423_BENCH_BACKEND=gloo timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node=$n \
    --master-addr=127.0.0.1 --master-port=$port bench.py --gpus $n --steps 10 --verify ends \
    > gpurun_out/gloo/bench_gloo$n.log 2>&1 || { echo "STOP gloo $n"; tail -20 gpurun_out/gloo/bench_gloo$n.log; exit 1; }
  grep '^{"metric"' gpurun_out/gloo/bench_gloo$n.log > gpurun_out/gloo/bench_gloo$n.json
  python - gpurun_out/gloo/bench_gloo$n.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
c, r = d["cpu_baseline"], d["roofline"]
print(f"ranks {d['n_gpus']}: value {d['value']} frac {r['frac']} traffic {r['traffic']} ({r['traffic_source']['status']}) "
      f"cpu {c['value']} {c['unit']} on {c['cores']} threads ({c['threads_limited_by']}), world {c['world_size']}, "
      f"parity {d['parity_verified']} ({d['parity_frames_checked']} frames)")
PY
done
if [ -x oracle/_ref/dropin_bench ]; then
  (unset MJ423_DROPIN_DEFER; timeout -k 10 120 oracle/_ref/dropin_bench 20 > gpurun_out/gloo/dropin_default.json 2> gpurun_out/gloo/dropin_default.err) || { echo "STOP dropin"; exit 1; }
  timeout -k 10 120 oracle/_ref/dropin_bench_ref 20 > gpurun_out/gloo/dropin_ref.json
  cat gpurun_out/gloo/dropin_default.json gpurun_out/gloo/dropin_ref.json; cat gpurun_out/gloo/dropin_default.err
fi
echo "gloo_rehearsal done"
