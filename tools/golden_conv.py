"""Whole-file GPU decode of each golden .mpg (diagnostic: run with MJ423_ENTPAR_DEBUG=1 to print the
synchronisation's iterations per window)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mjpeg423-video-decoder-software_amd"))
import torch  # noqa: E402

import mj423  # noqa: E402

ctx = mj423.Context(0)
gold = os.path.join(REPO, "tests", "golden")
for name in sorted(os.listdir(gold)):
    if not name.endswith(".mpg"):
        continue
    m = mj423.Mpg(os.path.join(gold, name))
    w, h, n = m.header.width, m.header.height, m.header.num_frames
    out = torch.empty((n, h, w), dtype=torch.int32, device="cuda:0")
    torch.cuda.synchronize()
    print(f"file {name} {w}x{h} {n} frames", flush=True)
    m.decode_gpu(ctx, 0, n, out.data_ptr())
    torch.cuda.synchronize()
    m.close()
ctx.close()
