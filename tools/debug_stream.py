"""Stream-kernel mismatch map (GPU box): decodes a seeded I/P stream and prints which
(frame, row, column) ranges differ from the oracle.  Measurement/debug tool only.
usage: python tools/debug_stream.py CHROMA W H"""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "mjpeg423-video-decoder-software_amd"), os.path.join(REPO, "oracle")]
import torch  # noqa: E402
import mj423  # noqa: E402
import oracle as orc  # noqa: E402

chroma, w, h = (int(a) for a in sys.argv[1:4])
rng = np.random.default_rng(chroma + w)
types = np.array([0, 1, 1, 1, 0, 1, 1, 0, 0, 1], np.uint8)
n = len(types)
A = orc.random_quantized_planes(rng, w, h, chroma, nframes=n).reshape(n, -1)
inp = A.copy()
for f in range(1, n):
    if types[f]:
        inp[f] = (A[f].astype(np.int32) - A[f - 1].astype(np.int32)).astype(np.int16)
with mj423.Context(0) as ctx:
    d_in = torch.from_numpy(inp.reshape(-1)).to("cuda:0")
    d_out = torch.full((n * w * h,), 0x7eadbeef, dtype=torch.int32, device="cuda:0")
    torch.cuda.synchronize()
    ctx.decode_stream_device(d_in.data_ptr(), d_out.data_ptr(), n, w, h, chroma, types)
    ctx.synchronize()
    got = d_out.cpu().numpy().view(np.uint32).reshape(n, h, w)
exp = orc.decode_frames_mt(A, n, w, h, chroma, nthreads=4)
bad = got != exp
print(f"{chroma} {w}x{h} lib={os.environ.get('MJ423_LIB', 'tree')} static={os.environ.get('MJ423_GOP_STATIC', '1')}:"
      f" {int(bad.sum())} bad pixels, untouched {int((got == 0x7eadbeef).sum())}")
for f in range(n):
    rows = np.nonzero(bad[f].any(axis=1))[0]
    if len(rows):
        cols = np.nonzero(bad[f].any(axis=0))[0]
        print(f"  frame {f}: rows {rows[:24].tolist()}{'...' if len(rows) > 24 else ''} ({len(rows)}),"
              f" cols {cols.min()}..{cols.max()} ({len(cols)})")
