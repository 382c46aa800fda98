#!/bin/bash
# The whole-file GPU decode (bench.py --mode file --frontend gpu, mj423_mpg_decode_gpu) on the GPU
# box: the bench line, the entropy front end's convergence log, a rocprofv3 kernel + memory-copy
# trace (per-kernel time and the H2D upload spans of every pass), and separate FETCH_SIZE /
# WRITE_SIZE passes (per dispatch, every kernel of the pass).  ARGS overrides the workload.
O=gpurun_out/${OUT-file}
mkdir -p $O && export TMPDIR=/tmp
args="--mode file --config f2 --frontend gpu ${ARGS}"
timeout -k 10 300 python bench.py $args --steps 20 > $O/bench.log 2>&1 || { echo "STOP bench"; tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log
MJ423_ENTPAR_DEBUG=1 timeout -k 10 300 python bench.py $args --steps 1 --warmup 0 --no-cpu --no-verify > $O/debug.log 2>&1 || { echo "STOP debug"; tail -5 $O/debug.log; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $O/kt -o kt --output-format csv -- python bench.py $args --steps 20 --no-cpu --no-verify > $O/kt.log 2>&1 || { echo "STOP kt"; tail -5 $O/kt.log; exit 1; }
[ -n "$KT_ONLY" ] && { echo "file_trace done (kernel trace only)"; exit 0; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $O/fetch -o f --output-format csv -- python bench.py $args --steps 3 --warmup 1 --no-cpu --no-verify > $O/fetch.log 2>&1 || { echo "STOP fetch"; tail -5 $O/fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $O/write -o w --output-format csv -- python bench.py $args --steps 3 --warmup 1 --no-cpu --no-verify > $O/write.log 2>&1 || { echo "STOP write"; tail -5 $O/write.log; exit 1; }
echo "file_trace done"
