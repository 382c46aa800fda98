#!/bin/bash
# Counters of the whole-file GPU decode's kernels (bench.py --mode file --frontend gpu), one rocprofv3
# --pmc pass per counter set (GPU box): SQ instruction mix / wave cycles, then FETCH_SIZE, then
# WRITE_SIZE (MI355X_MICROARCH.md §HBM: separate passes).  tools/pmc_file_summary.py reads them.
O=gpurun_out/fe_pmc; mkdir -p $O && export TMPDIR=/tmp
args="--mode file --config f2 --frontend gpu --steps 3 --warmup 1 --no-cpu --no-verify"
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set -d $O/p$i -o p --output-format csv -- python bench.py $args > $O/p$i.log 2>&1 || { echo "STOP pmc $i"; tail -5 $O/p$i.log; exit 1; }
  echo "pmc pass $i done"
done
echo fe_pmc done
