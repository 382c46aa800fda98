"""Debug helper (GPU box): fused-kernel CSC over all 2^24 triples vs a numpy restatement
of ycbcr_to_rgb.c:26-49; prints the first mismatches.  Measurement/debug only."""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "mjpeg423-video-decoder-software_amd"))
import mj423  # noqa: E402


def csc_np(Y, Cb, Cr):
    Y, Cb, Cr = (np.asarray(a, np.int64) for a in (Y, Cb, Cr))
    cbb, crr, yy = Cb - 128, Cr - 128, Y << 14
    norm = lambda v: np.where(v < 0, 0, np.minimum(v >> 14, 255))
    return (norm(yy + 29032 * cbb) | norm(yy - 5638 * cbb - 11700 * crr) << 8 | norm(yy + 22970 * crr) << 16).astype(np.uint32)


chroma = int(sys.argv[1]) if len(sys.argv) > 1 else 444
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
W = H = 8 * B
g = mj423.geometry(W, H, chroma)
ctx = mj423.Context(0)
dev = torch.device("cuda:0")
r = torch.arange(B, device=dev, dtype=torch.int64)[:, None]
c = torch.arange(B, device=dev, dtype=torch.int64)[None, :]
if chroma == 444:
    t, ypm, j = r * B + c, 1, 0
elif chroma == 422:
    t, ypm, j = r * (B // 2) + (c >> 1), 2, c & 1
else:
    t, ypm, j = (r >> 1) * (B // 2) + (c >> 1), 4, 2 * (r & 1) + (c & 1)
yv = ((t >> 16) * ypm + j).expand(B, B)
coef = torch.zeros(g.y_blocks + 2 * g.c_blocks, 64, dtype=torch.int16, device=dev)
coef[:g.y_blocks, 0] = (8 * yv).reshape(-1).to(torch.int16)
tc = torch.arange(g.c_blocks, device=dev, dtype=torch.int64)
coef[g.y_blocks:g.y_blocks + g.c_blocks, 0] = (8 * ((tc >> 8) & 255)).to(torch.int16)
coef[g.y_blocks + g.c_blocks:, 0] = (8 * (tc & 255)).to(torch.int16)
out = torch.empty(H * W, dtype=torch.int32, device=dev)
torch.cuda.synchronize(dev)
ctx.decode_batch_device(coef.data_ptr(), out.data_ptr(), 1, W, H, chroma, input_form=1)
ctx.synchronize()
o = out.view(H, W)
samp = o[::8, ::8].cpu().numpy().view(np.uint32)
# also check constancy inside a few blocks
blk_var = int((o[:64, :64].reshape(8, 8, 8, 8) != o[:64:8, :64:8].reshape(8, 1, 8, 1)).sum().item())
Yh = yv.cpu().numpy()
tt = t.expand(B, B).cpu().numpy()
exp = csc_np(Yh, (tt >> 8) & 255, tt & 255)
bad = np.argwhere(samp != exp)
print(f"chroma {chroma} B {B}: {len(bad)} mismatching Y blocks of {B * B}; non-constant pixels in 8x8 corner blocks: {blk_var}")
for rr, cc in bad[:12]:
    print(f"  block ({rr},{cc}) Y {Yh[rr, cc]} Cb {(tt[rr, cc] >> 8) & 255} Cr {tt[rr, cc] & 255}: got {samp[rr, cc]:08x} exp {exp[rr, cc]:08x}")
if len(bad):
    rows = np.unique(bad[:, 0])
    cols = np.unique(bad[:, 1])
    print("rows with mismatches:", rows[:20], len(rows), "cols:", cols[:20], len(cols))
