#!/bin/bash
# GPU box: which buffer's placement sets the batch kernel's rate: one coefficient buffer with
# eight output buffers, then one output buffer with eight coefficient buffers (4K 4:2:0).
export TMPDIR=/tmp
O=gpurun_out/r02pk; mkdir -p $O
for k in coef out; do
  PROBE_PAIRS=8 PROBE_PAIRS_KEEP=$k timeout -k 10 300 ./tools/probe 420 3840 2160 300 7 > "$O/keep_$k.txt" 2>&1 || { cat "$O/keep_$k.txt"; exit 1; }
  echo "== same $k"; grep "pair" "$O/keep_$k.txt"
done
