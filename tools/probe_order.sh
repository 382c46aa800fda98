#!/bin/bash
# Tile-order experiment (GPU box): frame-interleaved (fgroup) and XCD-chunked orders.
mkdir -p gpurun_out
{
for args in "420 3840 2160 300" "420 1920 1080 300" "420 3840 2160 300" "420 1920 1080 300"; do
  echo "== $args"; timeout -k 10 200 ./tools/probe $args 7 || exit $?
done
} > gpurun_out/probe_order.txt 2>&1
