#!/bin/bash
# The whole-file GPU decode's evidence (GPU box): the bench line, a rocprofv3 kernel trace with
# --stats of the same command, then the PMC passes (tools/fe_pmc.sh).  Every step has its own limit.
O=gpurun_out/file_prof; mkdir -p $O && export TMPDIR=/tmp
args="--mode file --config f2 --frontend gpu --no-cpu --no-verify"
timeout -k 10 200 python bench.py --mode file --config f2 --frontend gpu --steps 20 > $O/bench_f2.log 2>&1 || { echo "STOP bench"; exit 1; }
tail -1 $O/bench_f2.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- python bench.py $args --steps 10 > $O/kt.log 2>&1 || { echo "STOP kt"; exit 1; }
grep '^{"metric"' $O/kt.log | cut -c1-200
bash tools/fe_pmc.sh || exit 1
echo file_profile done
