#!/bin/bash
# GPU box: SQ/GRBM counters of the batch and stream kernels at C3 (effective clock, where the
# waves' time goes, LDS bank conflicts).  One counter pass per run, each under its own limit.
export TMPDIR=/tmp
O=$GRAFT_REPO_ROOT/gpurun_out/r02sq; mkdir -p $O
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -o "SQ_[A-Z_0-9]*\|GRBM_[A-Z_0-9]*" $O/counters.txt | sort -u > $O/names.txt || true
for m in batch stream; do
  a="--no-cpu --steps 5 --warmup 3"; [ $m = stream ] && a="$a --mode stream"
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES -d $O/p1_$m -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $a > $O/p1_$m.log 2>&1 || { tail -5 $O/p1_$m.log; exit 1; }
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAVES -d $O/p2_$m -o p --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py $a > $O/p2_$m.log 2>&1 || { tail -5 $O/p2_$m.log; exit 1; }
done
echo sq done
