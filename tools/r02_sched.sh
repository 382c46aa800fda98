#!/bin/bash
# GPU box: the production kernels compiled with the default scheduler and with
# -amdgpu-sched-strategy=max-memory-clause (tools/probe_default, tools/probe_memclause), ABA order.
export TMPDIR=/tmp
O=gpurun_out/r02sched; mkdir -p $O
for b in default memclause default; do
  for g in "420 3840 2160 300" "420 1920 1080 300" "444 640 480 300" "444 1920 1080 240"; do
    PROBE_GOP=24 PROBE_GOP_ORDERS=1 timeout -k 10 200 ./tools/probe_$b $g 7 > "$O/s_${b}_${g// /_}.txt" 2>&1 || { cat "$O/s_${b}_${g// /_}.txt"; exit 1; }
    PROBE_PAIRS=1 timeout -k 10 200 ./tools/probe_$b $g 7 > "$O/b_${b}_${g// /_}.txt" 2>&1 || { cat "$O/b_${b}_${g// /_}.txt"; exit 1; }
    echo "$b $g: $(grep 'order tile  ' $O/s_${b}_${g// /_}.txt | grep -o '(0.[0-9]*') stream, $(grep 'pair 0' $O/b_${b}_${g// /_}.txt | grep -o '(0.[0-9]*') batch"
  done
done
