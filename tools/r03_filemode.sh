#!/bin/bash
# Round 3: the whole-file paths (--mode file) after the pipeline's two-GOP chunks: host sink,
# device sink, GPU front end; the stream-kernel roofline summed over every launch.
mkdir -p gpurun_out/filemode && export TMPDIR=/tmp
for v in host:"--sink host" device:"--sink device" gpufrontend:"--frontend gpu"; do
  n=${v%%:*}; args=${v#*:}
  timeout -k 10 300 python bench.py --mode file --config f2 --steps 10 $args > gpurun_out/filemode/f2_$n.json 2> gpurun_out/filemode/f2_$n.err || { tail -5 gpurun_out/filemode/f2_$n.err; exit 1; }
  tail -1 gpurun_out/filemode/f2_$n.json | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$n', d['value'], d['unit'], d['roofline']['frac'], d.get('config',{}).get('chunks'), d['parity_verified'])"
done
