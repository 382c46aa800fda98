#!/bin/bash
# Round 3 diagnostic: memory-side TCC counters of the one-shot body in XCD-contiguous / frame-major /
# bands order and of the stream kernel (PROBE_PMC case list), one rocprofv3 --pmc pass per counter set.
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/pmcx; mkdir -p $O
sets=("TCC_EA0_WRREQ_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_EA0_WRREQ_LEVEL_sum"
      "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_TAG_STALL_sum")
for m in "3840 2160 300" "1920 1080 300"; do
  set -- $m
  i=0
  for s in "${sets[@]}"; do
    i=$((i+1))
    (cd /tmp && PROBE_GOP=24 PROBE_PMC=1 PROBE_DELTAS=1 timeout -s KILL 120 rocprofv3 --pmc $s -d $O/p_$1_$i -o p --output-format csv -- $R/tools/probe 420 $1 $2 $3 3 > $O/p_$1_$i.log 2>&1) || { tail -5 $O/p_$1_$i.log; exit 1; }
    grep median $O/p_$1_$i.log
  done
done
echo "r03_pmcx done"
