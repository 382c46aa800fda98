#!/bin/bash
# GPU box: the library's threaded host paths under ThreadSanitizer -- tools/asan_host_paths.cpp
# built with the host code instrumented by -fsanitize=thread (`make -C
# mjpeg423-video-decoder-software_amd tsan`); reports from inside the HIP runtime (uninstrumented,
# its own threads) are suppressed by tools/tsan.supp, every other report is kept.  Two seeded
# 640x480 streams as in tools/asan_host_paths.sh; output in gpurun_out/tsan/.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/tsan
W=/tmp/mj423_tsan; rm -rf $W; mkdir -p $W/out
python - $W <<'PY' || exit 1
import sys
import numpy as np
sys.path.insert(0, "tools")
import mpg_synth
d = sys.argv[1]
mpg_synth.build()
mpg_synth.write(f"{d}/sparse.mpg", 640, 480, 30, gop=7, seed=11)
a, s, t = mpg_synth.generate(640, 480, 8, gop=4, seed=12)
rng = np.random.default_rng(12)
s[:] = rng.integers(1, 2048, size=s.shape) * rng.choice([-1, 1], size=s.shape)
mpg_synth.write_coef(f"{d}/dense.mpg", 640, 480, t, s)
PY
TSAN_OPTIONS=suppressions=tools/tsan.supp:report_thread_leaks=0:halt_on_error=0 timeout -k 10 240 \
  tools/tsan_host_paths $W/sparse.mpg $W/dense.mpg $W/out > gpurun_out/tsan/host_paths.jsonl 2> gpurun_out/tsan/host_paths.err
rc=$?
echo "tsan_host_paths rc=$rc, reports: $(grep -c 'WARNING: ThreadSanitizer' gpurun_out/tsan/host_paths.err)"
cat gpurun_out/tsan/host_paths.jsonl
rm -rf $W
exit $rc
