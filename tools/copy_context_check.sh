export TMPDIR=/tmp; mkdir -p gpurun_out/cc
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --no-cpu --verify ends > gpurun_out/cc/c3_$i.log 2>&1 || exit 1
  grep '^{"metric"' gpurun_out/cc/c3_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3', d['roofline']['frac'], 'copy', d['copy_context']['frac'], d['copy_context']['ms'])"
done
for c in c2 c5 c1; do
  timeout -k 10 200 python bench.py --config $c --steps 20 --no-cpu --verify ends > gpurun_out/cc/$c.log 2>&1 || exit 1
  grep '^{"metric"' gpurun_out/cc/$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['roofline']['frac'], 'copy', d['copy_context']['frac'], d['copy_context']['ms'])"
done
timeout -k 10 200 python bench.py --mode stream --steps 20 --no-cpu --verify ends > gpurun_out/cc/c3s.log 2>&1 || exit 1
grep '^{"metric"' gpurun_out/cc/c3s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('c3s', d['roofline']['frac'], 'copy', d['copy_context']['frac'], d['copy_context']['ms'])"
