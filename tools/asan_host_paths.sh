#!/bin/bash
# GPU box: the library's threaded host paths under AddressSanitizer (tools/asan_host_paths.cpp,
# host code instrumented, device code not; built here by `make -C mjpeg423-video-decoder-software_amd
# asan`).  Two seeded 640x480 streams -- synthetic content with GOP 7, and fully populated planes --
# then one run of the driver; its JSON line goes to gpurun_out/asan/host_paths.jsonl.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/asan
W=/tmp/mj423_asan; rm -rf $W; mkdir -p $W/out
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
ASAN_OPTIONS=detect_leaks=0:abort_on_error=0 timeout -k 10 240 tools/asan_host_paths $W/sparse.mpg $W/dense.mpg $W/out \
  > gpurun_out/asan/host_paths.jsonl 2> gpurun_out/asan/host_paths.err
rc=$?
echo "asan_host_paths rc=$rc"
cat gpurun_out/asan/host_paths.jsonl
tail -20 gpurun_out/asan/host_paths.err
rm -rf $W
exit $rc
