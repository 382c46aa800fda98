"""Host time of the whole-file GPU decode per call (diagnostic): decodes the bench's synthetic
240 x 1080p .mpg N times with MJ423_FE_HOSTTIME=1 (the library prints its own host timestamps) and
prints the Python-side wall time per call beside them.  python tools/hosttime_probe.py [N]"""
import os
import sys
import tempfile
import time

os.environ["MJ423_FE_HOSTTIME"] = "1"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mjpeg423-video-decoder-software_amd"), os.path.join(REPO, "tools")]
import torch  # noqa: E402

import mj423  # noqa: E402
import mpg_synth  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
path = os.path.join(tempfile.mkdtemp(), "h.mpg")
mpg_synth.write(path, 1920, 1080, 240, gop=24, seed=0x4D4A3432, nthreads=16)
m = mj423.Mpg(path)
ctx = mj423.Context(0)
out = torch.empty((240, 1080, 1920), dtype=torch.int32, device="cuda:0")
torch.cuda.synchronize()
for i in range(n):
    t = time.perf_counter()
    m.decode_gpu(ctx, 0, 240, out.data_ptr())
    print(f"call {i}: {1e3 * (time.perf_counter() - t):.3f} ms wall", file=sys.stderr, flush=True)
