"""Per-call latency of the host-buffer entry points (PCIe included; measurements only):
decode_frame() and the accelerator API in the firmware's call order, at the reference's
native 640x480 4:4:4 and at 1080p 4:2:0; the reference's target is 24 fps (41.7 ms/frame,
c0/common/config.h:29)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mjpeg423-video-decoder-software_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

import mj423  # noqa: E402

YQ = np.array([16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55, 14, 13, 16, 24, 40, 57, 69, 56,
               14, 17, 22, 29, 51, 87, 80, 62, 18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113,
               92, 49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99], np.int32)  # tables.c:13-22


def planes(rng, nblocks):
    """Sparse quantized blocks (natural order), a few low-frequency coefficients each."""
    q = np.zeros((nblocks, 64), np.int16)
    q[:, 0] = rng.integers(0, 127, nblocks)
    for k in (1, 8, 2, 9, 16):
        m = rng.random(nblocks) < 0.4
        q[m, k] = rng.integers(-6, 7, int(m.sum()))
    return q


def med(f, reps=50):
    f()
    ts = []
    for _ in range(reps):
        t = time.perf_counter()
        f()
        ts.append(time.perf_counter() - t)
    return float(np.median(ts)) * 1e3


ctx = mj423.Context(0)
rng = np.random.default_rng(1)
for w, h, chroma in ((640, 480, 444), (1920, 1080, 420)):
    g = mj423.geometry(w, h, chroma)
    Y, Cb, Cr = planes(rng, g.y_blocks), planes(rng, g.c_blocks), planes(rng, g.c_blocks)
    ms = med(lambda: ctx.decode_frame(Y, Cb, Cr, w, h, chroma))
    print(f"decode_frame {w}x{h} {chroma}: {ms:.3f} ms/call ({1e3 / ms:.0f} frames/s, host buffers)", flush=True)
# accelerator API, firmware order (c0/playback.c:71-121), dequantized planes
acc = mj423.Accelerator(640, 480, mj423.CHROMA_444)
g = mj423.geometry(640, 480, 444)
dq = [(planes(rng, g.y_blocks).astype(np.int32) * YQ).astype(np.int16) for _ in range(3)]  # dct_block_t input
out = np.empty((480, 640), np.uint32)


def accel_frame():
    acc.idct_accel_calculate_buffer_cb(dq[1])
    acc.idct_accel_calculate_buffer_cr(dq[2])
    acc.idct_accel_calculate_buffer_y(dq[0])
    acc.ycbcr_to_rgb_accel_get_results(out)
    acc.wait_for_idct_y_finsh()
    acc.wait_for_ycbcr_to_rgb_finsh()


ms = med(accel_frame)
print(f"accelerator API 640x480 444 (firmware call order): {ms:.3f} ms/frame ({1e3 / ms:.0f} frames/s)", flush=True)

# host-buffer batches (decode_frames: H2D of the coefficients, one fused launch, D2H of the BGRA), the
# PCIe-inclusive rate of the boundary that hands over host memory -- never the headline value
for w, h, chroma, n in ((1920, 1080, 420, 60), (3840, 2160, 420, 30)):
    g = mj423.geometry(w, h, chroma)
    coef = np.concatenate([np.concatenate([planes(rng, g.y_blocks), planes(rng, 2 * g.c_blocks)]).reshape(-1)
                           for _ in range(n)])
    out = np.empty((n, h, w), np.uint32)
    out.fill(0)  # pages touched once: the timed calls measure the copies, not first-touch faults
    ms_fresh = med(lambda: ctx.decode_frames(coef, n, w, h, chroma), reps=5)
    ms = med(lambda: ctx.decode_frames(coef, n, w, h, chroma, out=out), reps=10)
    print(f"decode_frames {n} x {w}x{h} {chroma}, a fresh output array per call: {ms_fresh:.2f} ms/call", flush=True)
    mb = n * (2 * g.coef_per_frame + 4 * w * h) / 1e6
    print(f"decode_frames {n} x {w}x{h} {chroma} (host buffers re-used, PCIe both ways): {ms:.2f} ms/call, "
          f"{n * w * h / ms / 1e3:.0f} Mpix/s, {mb / ms:.1f} GB/s over PCIe", flush=True)
