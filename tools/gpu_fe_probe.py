"""Whole-GPU decode throughput (measurements only): entropy_kernel + stream kernel on a
synthetic 4:4:4 .mpg, frames left in HBM, for several frame counts (the GPU front end
is as parallel as the batch has bitstreams: 3 per frame)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("mjpeg423-video-decoder-software_amd", "tools"):
    sys.path.insert(0, os.path.join(REPO, p))
import torch  # noqa: E402

import mj423  # noqa: E402
import mpg_synth  # noqa: E402

w, h = int(sys.argv[1]), int(sys.argv[2])
counts = [int(x) for x in sys.argv[3].split(",")]
path = "/tmp/gfe.mpg"
mpg_synth.write(path, w, h, max(counts), 24, 7)
m = mj423.Mpg(path)
ctx = mj423.Context(0)
ctx.enable_timing(True)
for n in counts:
    out = torch.empty((n, h, w), dtype=torch.int32, device="cuda:0")
    m.decode_gpu(ctx, 0, n, out.data_ptr())  # warm-up
    best = 1e9
    for _ in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        m.decode_gpu(ctx, 0, n, out.data_ptr())
        best = min(best, time.perf_counter() - t)
    print(f"{w}x{h} x{n}: {best * 1e3:8.2f} ms  {n * w * h / best / 1e6:9.0f} Mpix/s  "
          f"(last stream-kernel launch {ctx.kernel_ms():.2f} ms)", flush=True)
    del out
