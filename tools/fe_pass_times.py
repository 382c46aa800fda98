"""Per-pass wall times of the whole-GPU .mpg decode (measurements only): finds one-off
stalls that an average over K passes hides."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("mjpeg423-video-decoder-software_amd", "tools"):
    sys.path.insert(0, os.path.join(REPO, p))
import torch  # noqa: E402

import mj423  # noqa: E402
import mpg_synth  # noqa: E402

w, h, n, passes = 1920, 1080, 240, int(sys.argv[1]) if len(sys.argv) > 1 else 30
path = "/tmp/fpt.mpg"
mpg_synth.write(path, w, h, n, 24, 7)
m = mj423.Mpg(path)
ctx = mj423.Context(0)
out = torch.empty((n, h, w), dtype=torch.int32, device="cuda:0")
ts = []
for i in range(passes):
    t = time.perf_counter()
    m.decode_gpu(ctx, 0, n, out.data_ptr())
    ts.append((time.perf_counter() - t) * 1e3)
print(" ".join("%.2f" % x for x in ts), flush=True)
