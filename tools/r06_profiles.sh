#!/bin/bash
# Round 6 final rocprofv3 summaries: the default bench (C3 batch kernel) and the whole-file decode.
set -o pipefail
O=gpurun_out/r06/final_prof; mkdir -p $O && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c3 -o c3 --output-format csv -- python bench.py --steps 20 > $O/c3_bench.log 2>&1 || { echo STOP c3; tail -5 $O/c3_bench.log; exit 1; }
tail -1 $O/c3_bench.log | cut -c1-200
OUT=r06/final_prof/file KT_ONLY=1 bash tools/file_trace.sh || exit 1
python tools/kt_summary.py gpurun_out/r06/final_prof/file/kt 20 > $O/file/kt_summary.txt
head -6 $O/file/kt_summary.txt
