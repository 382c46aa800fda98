#!/bin/bash
# Round 3: one-shot chain stream kernel (state handed between workgroups of one XCD) against the
# production stream kernel and the batch kernel, same frames (GOP 24, 288 frames), band sizes.
mkdir -p gpurun_out/chain && export TMPDIR=/tmp
O=gpurun_out/chain
for m in "420 3840 2160 288 20 120" "420 3840 2160 288 20 60" "420 1920 1080 288 60 68" "420 1920 1080 288 60 136"; do
  set -- $m
  PROBE_R03=1 PROBE_GOP=24 PROBE_CHAIN=1 PROBE_CHAIN_B=$6 PROBE_DELTAS=1 PROBE_WARM_S=1.5 timeout -k 10 120 ./tools/probe $1 $2 $3 $4 $5 > $O/chain_$2_B$6.log 2>&1 || { cat $O/chain_$2_B$6.log; exit 1; }
  echo "== $1 $2x$3 B=$6"; grep -E "chain|production" $O/chain_$2_B$6.log
done
echo "r03_chain done"
