"""Pipeline A/B for the streaming decoder (measurements only): chunk sizes, front-end
threads, and the raw PCIe rates of pinned copies on this box."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in ("mjpeg423-video-decoder-software_amd", "tools"):
    sys.path.insert(0, os.path.join(REPO, p))
import torch  # noqa: E402

import mj423  # noqa: E402
import mpg_synth  # noqa: E402

w, h, n = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
path = "/tmp/pp.mpg"
mpg_synth.write(path, w, h, n, 24, 7)
m = mj423.Mpg(path)
ctx = mj423.Context(0)
for nb in (64 << 20, 256 << 20):
    hbuf = torch.empty(nb, dtype=torch.uint8).pin_memory()
    dbuf = torch.empty(nb, dtype=torch.uint8, device="cuda")
    for _ in range(2):
        torch.cuda.synchronize(); t = time.perf_counter(); dbuf.copy_(hbuf, non_blocking=True); torch.cuda.synchronize()
        h2d = nb / (time.perf_counter() - t) / 1e9
        t = time.perf_counter(); hbuf.copy_(dbuf, non_blocking=True); torch.cuda.synchronize()
        d2h = nb / (time.perf_counter() - t) / 1e9
    print(f"pinned {nb >> 20} MiB: H2D {h2d:.1f} GB/s  D2H {d2h:.1f} GB/s", flush=True)
g = mj423.geometry(w, h, 444)
print(f"{w}x{h} 4:4:4 x{n}: coef {g.coef_per_frame * 2 / 1e6:.1f} MB/frame, BGRA {w * h * 4 / 1e6:.1f} MB/frame")
t = time.perf_counter(); m.entropy_decode_deltas(0, n, nthreads=16); fe = time.perf_counter() - t
print(f"front end alone (16 threads, one call): {fe * 1e3:.1f} ms = {n * w * h / fe / 1e6:.0f} Mpix/s", flush=True)
for chunk in [int(x) for x in os.environ.get("CHUNKS", "4 8 12 24 48").split()]:
    for th in (8, 16):
        best = None
        pipe = mj423.Pipeline(ctx, w, h, chunk_frames=chunk, nthreads=th)
        for _ in range(3):
            st = pipe.decode(m, 0, n, lambda fi, v: 0)
            best = st if best is None or st.wall_s < best.wall_s else best
        print(f"chunk {chunk:3d} threads {th:2d}: wall {best.wall_s * 1e3:7.1f} ms  "
              f"{n * w * h / best.wall_s / 1e6:7.0f} Mpix/s  fe_busy {best.frontend_busy_s * 1e3:6.1f} ms  "
              f"gpu_span {best.gpu_span_ms:6.1f} ms", flush=True)
        pipe.close()
