#!/bin/bash
# The PCIe-inclusive and whole-file paths on this tree (GPU box): host-buffer entry points
# (tools/latency_probe.py) and bench.py --mode file with the host front end (host and device sinks)
# and the GPU front end.  None of these is the headline value.
mkdir -p gpurun_out/paths && export TMPDIR=/tmp
timeout -k 10 300 python tools/latency_probe.py > gpurun_out/paths/latency.log 2>&1 || { echo "STOP latency"; tail -5 gpurun_out/paths/latency.log; exit 1; }
cat gpurun_out/paths/latency.log
for v in "host host" "device host" "host gpu"; do
  set -- $v
  timeout -k 10 300 python bench.py --mode file --config f2 --sink $1 --frontend $2 --steps 5 \
    > gpurun_out/paths/file_$1_$2.log 2>&1 || { echo "STOP file $v"; tail -5 gpurun_out/paths/file_$1_$2.log; exit 1; }
  grep '^{"metric"' gpurun_out/paths/file_$1_$2.log > gpurun_out/paths/file_$1_$2.json
  python -c "import json,sys; d=json.load(open('gpurun_out/paths/file_$1_$2.json')); print('$v', d['value'], d['unit'], 'launch frac', d['roofline']['frac'], 'parity', d['parity_verified'])"
done
echo "paths_check done"
