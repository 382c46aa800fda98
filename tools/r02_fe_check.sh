export TMPDIR=/tmp
O=gpurun_out/fec; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multi.py -x -q --timeout 120 --timeout-method thread -m gpu -k "gpu_entropy or mpg or multi" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --mode file --config f2 --frontend gpu --steps 20 > $O/f2_$r.json 2> $O/f2_$r.err || { tail -5 $O/f2_$r.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/f2_$r.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['parity_verified'])"
done
