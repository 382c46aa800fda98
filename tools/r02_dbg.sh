#!/bin/bash
export TMPDIR=/tmp
for v in "" tools/variants/oobhigh/libmj423gpu.so; do
  for st in 1 0; do
    MJ423_LIB=$v MJ423_GOP_STATIC=$st timeout -k 10 120 python tools/debug_stream.py 420 200 120 || exit 1
  done
done
MJ423_GOP_STATIC=1 timeout -k 10 120 python tools/debug_stream.py 444 72 40 || exit 1
MJ423_GOP_STATIC=1 timeout -k 10 120 python tools/debug_stream.py 422 136 56 || exit 1
MJ423_GOP_STATIC=1 timeout -k 10 120 python tools/debug_stream.py 420 1920 1080 || exit 1
