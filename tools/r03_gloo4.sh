#!/bin/bash
# Round 3: the multi-rank bench path rehearsed on one GPU (4 ranks over gloo sharing cuda:0):
# batch C3 and a stream C2 whose ranks 1-3 start mid-GOP; every rank's frames verified.
mkdir -p gpurun_out/gloo4 && export TMPDIR=/tmp
O=gpurun_out/gloo4
export MJ423_BENCH_BACKEND=gloo HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29517 \
  bench.py --gpus 4 --config c3 --frames 60 --steps 5 > $O/c3_batch.log 2>&1 || { tail -20 $O/c3_batch.log; exit 1; }
grep '^{' $O/c3_batch.log | tail -1 | cut -c1-400
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29518 \
  bench.py --gpus 4 --config c2 --frames 50 --mode stream --steps 5 > $O/c2_stream.log 2>&1 || { tail -20 $O/c2_stream.log; exit 1; }
grep '^{' $O/c2_stream.log | tail -1 | cut -c1-400
echo "r03_gloo4 done"
