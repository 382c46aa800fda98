"""Does the output/input buffer placement change decode_kernel's bandwidth?  (GPU box.)
Times ctx.decode_batch_device on the same frames with buffers from torch's caching
allocator, from hipMalloc directly, and with offsets, interleaved, medians of N."""
import ctypes
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "mjpeg423-video-decoder-software_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mj423  # noqa: E402

hip = ctypes.CDLL("libamdhip64.so")


def hip_malloc(n):
    p = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(n)) == 0
    return p.value


def main():
    w, h, chroma, nfr = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    g = mj423.geometry(w, h, chroma)
    ctx = mj423.Context(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    ctx.set_stream(s.cuda_stream)
    cb = nfr * g.coef_per_frame * 2
    ob = nfr * w * h * 4
    t_coef = torch.empty(cb // 2 + (1 << 20), dtype=torch.int16, device="cuda")
    t_out = torch.empty(ob // 4 + (1 << 20), dtype=torch.int32, device="cuda")
    h_coef = hip_malloc(cb + (4 << 20))
    h_out = hip_malloc(ob + (4 << 20))
    print(f"torch coef {t_coef.data_ptr():#x} out {t_out.data_ptr():#x}; hip coef {h_coef:#x} out {h_out:#x}")
    cases = {
        "torch/torch": (t_coef.data_ptr(), t_out.data_ptr()),
        "hip/hip": (h_coef, h_out),
        "torch/hip": (t_coef.data_ptr(), h_out),
        "hip/torch": (h_coef, t_out.data_ptr()),
        "hip/hip+256": (h_coef, h_out + 256),
        "hip/hip+4096": (h_coef, h_out + 4096),
        "hip/hip+1M": (h_coef, h_out + (1 << 20)),
        "hip+1M/hip": (h_coef + (1 << 20), h_out),
    }
    for c, _ in cases.values():
        ctx.synth_frames_device(c, w, h, chroma, nfr, 0, 0x4D4A3432)
    torch.cuda.synchronize()
    res = {k: [] for k in cases}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    for r in range(8):
        for k, (c, o) in cases.items():
            ev[0].record(s)
            ctx.decode_batch_device(c, o, nfr, w, h, chroma)
            ev[1].record(s)
            ev[1].synchronize()
            if r:
                res[k].append(ev[0].elapsed_time(ev[1]))
    fb = mj423.frame_bytes(w, h, chroma) * nfr
    for k, v in res.items():
        m = float(np.median(v))
        print(f"{k:14s} median {m:.4f} ms  {fb / m / 1e6:.0f} GB/s  frac {fb / m / 1e6 / 8000:.3f}")


if __name__ == "__main__":
    main()
