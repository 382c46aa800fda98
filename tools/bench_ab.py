"""Batch-kernel timing under different process set-ups (measurements only): why the bench
reads a few % below tools/probe for the same library kernel.  usage: bench_ab.py CHROMA W H N"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mjpeg423-video-decoder-software_amd"))
import torch  # noqa: E402

import mj423  # noqa: E402

chroma, w, h, n = (int(x) for x in sys.argv[1:5])
g = mj423.geometry(w, h, chroma)
hip = ctypes.CDLL("libamdhip64.so")
ctx = mj423.Context(0)
ctx.enable_timing(True)


def hip_alloc(nbytes):
    p = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes)) == 0
    return p.value


def run(tag, coef, out, steps=20):
    for _ in range(3):
        ctx.decode_batch_device(coef, out, n, w, h, chroma)
    ctx.synchronize()
    ms = []
    for _ in range(steps):
        ctx.decode_batch_device(coef, out, n, w, h, chroma)
        ms.append(ctx.kernel_ms())
    fb = mj423.frame_bytes(w, h, chroma) * n
    print(f"{tag:48s} median {np.median(ms):.4f} ms mean {np.mean(ms):.4f} ms  frac {fb / (np.median(ms) * 1e-3) / 8e12:.3f}",
          flush=True)


tc = torch.empty(n * g.coef_per_frame, dtype=torch.int16, device="cuda:0")
to = torch.empty(n * w * h, dtype=torch.int32, device="cuda:0")
ctx.synth_frames_device(tc.data_ptr(), w, h, chroma, n, 0, 0x4D4A3432)
hc = hip_alloc(n * g.coef_per_frame * 2)
ho = hip_alloc(n * w * h * 4)
ctx.synth_frames_device(hc, w, h, chroma, n, 0, 0x4D4A3432)
ctx.synchronize()
for rnd in range(2):
    run("context stream, hipMalloc buffers", hc, ho)
    run("context stream, torch buffers", tc.data_ptr(), to.data_ptr())
    s = torch.cuda.Stream()
    ctx.set_stream(s.cuda_stream)
    run("torch stream, torch buffers", tc.data_ptr(), to.data_ptr())
    run("torch stream, hipMalloc buffers", hc, ho)
    ctx.set_stream(None)
