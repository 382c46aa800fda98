#!/bin/bash
# Counters of the LDS-DMA stream kernel (MJ423_GOP_DMA=2) against the production stream kernel
# (MJ423_GOP_DMA=0) on the bench's stream workloads: one rocprofv3 --pmc pass per counter set
# (GPU box).  Outputs gpurun_out/pmcdma/<cfg>_f<form>_<set>/.
export TMPDIR=/tmp
O=gpurun_out/pmcdma; mkdir -p $O
sets=("FETCH_SIZE" "WRITE_SIZE"
      "TCC_EA0_WRREQ_LEVEL_sum TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
      "SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU")
for cfg in ${CONFIGS-c3 c2}; do
  for form in 0 2; do
    i=0
    for s in "${sets[@]}"; do
      i=$((i+1))
      MJ423_GOP_DMA=$form timeout -s KILL 120 rocprofv3 --pmc $s -d $O/${cfg}_f${form}_$i -o p --output-format csv -- \
        python bench.py --config $cfg --mode stream --steps 3 --warmup 2 --no-cpu --no-verify > $O/${cfg}_f${form}_$i.log 2>&1 \
        || { echo "STOP $cfg $form $i"; tail -5 $O/${cfg}_f${form}_$i.log; exit 1; }
      echo "$cfg form $form set $i done"
    done
  done
done
echo "pmc_dma done"
