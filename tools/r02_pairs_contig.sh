#!/bin/bash
# GPU box: default vs physically contiguous (hipDeviceMallocContiguous) buffer pairs, batch kernel.
export TMPDIR=/tmp
O=gpurun_out/r02pc; mkdir -p $O
for r in 1 2; do
  PROBE_PAIRS=7 PROBE_PAIRS_CONTIG=1 timeout -k 10 300 ./tools/probe 420 3840 2160 300 7 > "$O/pc_$r.txt" 2>&1 || { cat "$O/pc_$r.txt"; exit 1; }
  echo "== run $r"; grep "pair" "$O/pc_$r.txt"
done
