#!/bin/bash
# Round 6 whole-file evidence on the current tree: bench line + kernel trace (tools/file_trace.sh,
# KT_ONLY), then the per-kernel PMC passes (tools/fe_pmc.sh).
set -o pipefail
OUT=r06/${TAG:-file_final}/file KT_ONLY=1 bash tools/file_trace.sh || exit 1
python tools/kt_summary.py gpurun_out/r06/${TAG:-file_final}/file/kt 20 > gpurun_out/r06/${TAG:-file_final}/file/kt_summary.txt
head -4 gpurun_out/r06/${TAG:-file_final}/file/kt_summary.txt
bash tools/fe_pmc.sh || exit 1
mkdir -p gpurun_out/r06/${TAG:-file_final}/pmc && cp -r gpurun_out/fe_pmc/* gpurun_out/r06/${TAG:-file_final}/pmc/
