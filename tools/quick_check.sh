mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
for c in c3 c2 c5; do timeout -k 10 300 python bench.py --config $c --no-cpu > gpurun_out/q_$c.json 2>gpurun_out/q_$c.err || exit 1; done
timeout -k 10 200 ./tools/probe 420 3840 2160 300 7 > gpurun_out/q_probe.txt 2>&1
