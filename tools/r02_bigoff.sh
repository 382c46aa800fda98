#!/bin/bash
# GPU box: batch kernel rate against the output's offset from the coefficients inside one
# physically contiguous allocation (4K 4:2:0), two runs.
export TMPDIR=/tmp
O=gpurun_out/r02bo; mkdir -p $O
for r in 1 2; do
  PROBE_BIGOFF=0,2,4,8,16,32,64,128,256,512,1024,1536,2048,3072,4096 timeout -k 10 400 ./tools/probe 420 3840 2160 300 5 > "$O/bo_$r.txt" 2>&1 || { cat "$O/bo_$r.txt"; exit 1; }
  echo "== run $r"; grep "big\|out at" "$O/bo_$r.txt"
done
