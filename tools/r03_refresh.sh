#!/bin/bash
# Round-3 evidence refresh (GPU box): tools/gpu_check.sh over the bench configs with kernel
# traces + FETCH/WRITE passes, SQ instruction counters of the batch kernel (C3, C1), the
# drop-in bench.  Outputs under gpurun_out/; copied into profiles/r03 afterwards.
export TMPDIR=/tmp
mkdir -p gpurun_out/sq
CONFIGS="${CONFIGS-c3 c2 c5 c1 c3s c2s c5s c1s}" PROFILE="${PROFILE-c3 c2 c1 c3s c1s}" bash tools/gpu_check.sh > gpurun_out/check.log 2>&1
grep -q "gpu_check done" gpurun_out/check.log || { tail -20 gpurun_out/check.log; exit 1; }
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/sq
for c in c3 c1; do
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/$c -o p --output-format csv -- python3 $R/bench.py --config $c --no-cpu --no-verify --steps 5 --warmup 3 > $O/$c.log 2>&1) || { tail -5 $O/$c.log; exit 1; }
done
MJ423_DROPIN_DEFER=1 timeout -k 10 120 ./oracle/_ref/dropin_bench 50 > gpurun_out/dropin_defer.json 2>&1 || exit 1
timeout -k 10 120 ./oracle/_ref/dropin_bench_ref 50 > gpurun_out/dropin_ref.json 2>&1 || exit 1
echo "refresh done"
