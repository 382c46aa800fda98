"""Launch cadence vs measured decode_kernel time (GPU box): the same batch decode timed
(a) with a host sync after every launch, (b) back to back with events around each
launch, (c) back to back with one event pair around all of them, (d) back to back
with a 1 ms device-side idle gap (torch.cuda._sleep) between launches."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "mjpeg423-video-decoder-software_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import mj423  # noqa: E402


def main():
    w, h, chroma, nfr = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    k = 10
    g = mj423.geometry(w, h, chroma)
    ctx = mj423.Context(0)
    s = torch.cuda.Stream()
    torch.cuda.set_stream(s)
    ctx.set_stream(s.cuda_stream)
    coef = torch.empty(nfr * g.coef_per_frame, dtype=torch.int16, device="cuda")
    out = torch.empty(nfr * w * h, dtype=torch.int32, device="cuda")
    ctx.synth_frames_device(coef.data_ptr(), w, h, chroma, nfr, 0, 0x4D4A3432)
    fb = mj423.frame_bytes(w, h, chroma) * nfr

    def launch():
        ctx.decode_batch_device(coef.data_ptr(), out.data_ptr(), nfr, w, h, chroma)

    def ev():
        return torch.cuda.Event(enable_timing=True)

    for _ in range(3):
        launch()
    torch.cuda.synchronize()
    res = {}
    for rnd in range(3):
        # (a) synced
        t = []
        for _ in range(k):
            a, b = ev(), ev()
            a.record(s)
            launch()
            b.record(s)
            b.synchronize()
            t.append(a.elapsed_time(b))
        res.setdefault("a synced", []).extend(t)
        # (b) back to back, per-launch events
        es = [(ev(), ev()) for _ in range(k)]
        for a, b in es:
            a.record(s)
            launch()
            b.record(s)
        torch.cuda.synchronize()
        res.setdefault("b back-to-back", []).extend(a.elapsed_time(b) for a, b in es)
        # (c) one pair around k
        a, b = ev(), ev()
        a.record(s)
        for _ in range(k):
            launch()
        b.record(s)
        torch.cuda.synchronize()
        res.setdefault("c one pair /k", []).append(a.elapsed_time(b) / k)
        # (d) idle gap on the device between launches
        es = [(ev(), ev()) for _ in range(k)]
        for a, b in es:
            torch.cuda._sleep(2_000_000)
            a.record(s)
            launch()
            b.record(s)
        torch.cuda.synchronize()
        res.setdefault("d device gap", []).extend(a.elapsed_time(b) for a, b in es)
    print(f"{w}x{h} {chroma} x{nfr}")
    for name, v in res.items():
        m = float(np.median(v))
        print(f"  {name:16s} median {m:.4f} ms  mean {np.mean(v):.4f}  frac {fb / m / 1e6 / 8000:.3f}  "
              f"first-of-run {v[0]:.4f}")


if __name__ == "__main__":
    main()
