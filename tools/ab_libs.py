"""Same-process A/B of library builds (measurements only): every build named on the command line
is loaded into ONE process (ctypes, RTLD_LOCAL: each keeps its own kernels) and decodes the SAME
device buffers, in interleaved rounds, so buffer placement (±4 % between processes)
is common to all of them.  Prints per build the median kernel time and fraction of 8 TB/s, and
checks that every build's output equals the first one's.

  python tools/ab_libs.py CONFIG ROUNDS lib_a.so lib_b.so ...
  CONFIG = c3 | c2 | c5 | c1 (bench.py's batch configs), ROUNDS = interleaved rounds of 10 launches
"""
import ctypes
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mjpeg423-video-decoder-software_amd"))
import torch  # noqa: E402

import mj423  # noqa: E402  (geometry and byte counts from the default build)

CONFIGS = {"c1": (640, 480, 444, 300), "c2": (1920, 1080, 420, 300), "c3": (3840, 2160, 420, 300),
           "c5": (7680, 4320, 422, 15)}
SEED = 0x4D4A3432


def main():
    cfg, rounds, paths = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
    w, h, chroma, n = CONFIGS[cfg]
    g = mj423.geometry(w, h, chroma)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    coef = torch.empty(n * g.coef_per_frame, dtype=torch.int16, device=dev)
    outs = [torch.empty(n * w * h, dtype=torch.int32, device=dev) for _ in paths]
    libs, ctxs = [], []
    for p in paths:
        L = ctypes.CDLL(os.path.abspath(p))
        L.mj423_ctx_kernel_ms.restype = ctypes.c_double
        c = ctypes.c_void_p()
        assert L.mj423_ctx_create(ctypes.byref(c), 0) == 0
        assert L.mj423_ctx_set_stream(c, ctypes.c_void_p(stream.cuda_stream)) == 0
        assert L.mj423_ctx_enable_timing(c, 1) == 0
        libs.append(L)
        ctxs.append(c)
    assert libs[0].mj423_synth_frames_device(ctxs[0], ctypes.c_void_p(coef.data_ptr()), w, h, chroma, n,
                                             ctypes.c_uint64(0), ctypes.c_uint64(SEED)) == 0
    torch.cuda.synchronize()

    def launch(i):
        y = coef.data_ptr()
        d = mj423.FramesDesc(y, y + 128 * g.y_blocks, y + 128 * (g.y_blocks + g.c_blocks), g.coef_per_frame,
                             outs[i].data_ptr(), w * h, w, n, w, h, chroma, 0)
        assert libs[i].mj423_decode_frames_device(ctxs[i], ctypes.byref(d)) == 0
        return libs[i].mj423_ctx_kernel_ms(ctxs[i])

    for i in range(len(paths)):  # warm-up: clocks ramp, code objects load
        for _ in range(30):
            launch(i)
    torch.cuda.synchronize()
    times = [[] for _ in paths]
    for _ in range(rounds):
        for i in range(len(paths)):
            for _ in range(10):
                times[i].append(launch(i))
    torch.cuda.synchronize()
    fb = mj423.frame_bytes(w, h, chroma) * n
    ref = outs[0].cpu()
    for i, p in enumerate(paths):
        ms = float(np.median(times[i]))
        same = bool(torch.equal(outs[i].cpu(), ref))
        print(f"{cfg} {os.path.basename(os.path.dirname(p)) or p}: median {ms:.4f} ms  frac {fb / (ms * 1e-3) / 8e12:.4f}"
              f"  output equal to the first build: {same}", flush=True)


if __name__ == "__main__":
    main()
