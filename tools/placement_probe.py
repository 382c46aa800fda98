"""Which buffer sets the batch kernel's level: in ONE process,
the C3 decode (300 x 4K 4:2:0, decode_kernel<420>) is timed on a base pair of buffers, then with
only the coefficient buffer re-allocated N times (the output buffer kept), then with only the
output buffer re-allocated N times (the coefficients kept), then on a few cross pairs.  Every
allocation is kept alive until the end, so each lands on fresh pages.  Per pair: the median of
20 launches (HIP events on the launch stream) and the fraction of 8 TB/s.  Measurements only.

  python tools/placement_probe.py [N] [--pool | --contig | --contig-out]

--pool: the same with every coefficient/output pair carved out of ONE allocation (coefficients
first, output at the next 2-MiB boundary), N fresh pools -- the library-owned policy the review
asks to try.
--contig: every coefficient/output pair from hipExtMallocWithFlags(hipDeviceMallocContiguous);
--contig-out: only the output buffers so, the coefficients from torch.
--gap-sweep: ONE contiguous allocation per round (N rounds) holding the coefficients and then the
output at a swept gap after them (the relative offset of the read and write streams).
"""
import ctypes
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "mjpeg423-video-decoder-software_amd"))
import torch  # noqa: E402

import mj423  # noqa: E402

W, H, CH, NF = 3840, 2160, 420, 300
SEED = 0x4D4A3432


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 6
    pool = "--pool" in sys.argv
    contig = "--contig" in sys.argv
    contig_out = "--contig-out" in sys.argv
    hip = ctypes.CDLL("libamdhip64.so")
    g = mj423.geometry(W, H, CH)
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx = mj423.Context(0)
    ctx.set_stream(stream.cuda_stream)
    ctx.enable_timing(True)
    nco, npx = NF * g.coef_per_frame, NF * W * H
    fb = mj423.frame_bytes(W, H, CH) * NF
    keep = []

    def coef_buf():
        t = torch.empty(nco, dtype=torch.int16, device=dev)
        ctx.synth_frames_device(t.data_ptr(), W, H, CH, NF, 0, SEED)
        keep.append(t)
        return t

    def out_buf():
        t = torch.empty(npx, dtype=torch.int32, device=dev)
        keep.append(t)
        return t

    def pooled():
        cb = nco * 2
        ob = (cb + (2 << 20) - 1) // (2 << 20) * (2 << 20)
        t = torch.empty(ob + npx * 4, dtype=torch.uint8, device=dev)
        keep.append(t)
        c = t[:cb].view(torch.int16)
        o = t[ob:ob + npx * 4].view(torch.int32)
        ctx.synth_frames_device(c.data_ptr(), W, H, CH, NF, 0, SEED)
        return c, o

    class Raw:  # a hipExtMallocWithFlags allocation (kept until the end)
        def __init__(self, nbytes):
            p = ctypes.c_void_p()
            rc = hip.hipExtMallocWithFlags(ctypes.byref(p), ctypes.c_size_t(nbytes), ctypes.c_uint(0x4))
            assert rc == 0, f"hipExtMallocWithFlags(contiguous, {nbytes}) = {rc}"
            self.p = p.value
            keep.append(self)

        def data_ptr(self):
            return self.p

    def contig_pair(both):
        if both:
            c = Raw(nco * 2)
            ctx.synth_frames_device(c.data_ptr(), W, H, CH, NF, 0, SEED)
        else:
            c = coef_buf()
        return c, Raw(npx * 4)

    def timed(c, o):
        for _ in range(5):
            ctx.decode_batch_device(c.data_ptr(), o.data_ptr(), NF, W, H, CH)
        torch.cuda.synchronize(dev)
        ms = []
        for _ in range(20):
            ctx.decode_batch_device(c.data_ptr(), o.data_ptr(), NF, W, H, CH)
            ms.append(ctx.kernel_ms())
        med = float(np.median(ms))
        return {"ms": round(med, 4), "frac": round(fb / (med * 1e-3) / 8e12, 4),
                "coef_va": hex(c.data_ptr()), "out_va": hex(o.data_ptr())}

    rows = []

    def rec(kind, i, j, c, o):
        r = dict(kind=kind, coef=i, out=j, **timed(c, o))
        rows.append(r)
        print(json.dumps(r), flush=True)

    if "--gap-sweep" in sys.argv:
        gaps = [0, 4 << 10, 64 << 10, 256 << 10, 1 << 20, 2 << 20, 3 << 20, 4 << 20, 6 << 20, 8 << 20, 16 << 20,
                32 << 20, 64 << 20, 128 << 20]
        cb = (nco * 2 + (2 << 20) - 1) // (2 << 20) * (2 << 20)
        for i in range(n):
            base = Raw(cb + max(gaps) + npx * 4)
            ctx.synth_frames_device(base.data_ptr(), W, H, CH, NF, 0, SEED)

            class View:
                def __init__(self, p):
                    self.p = p

                def data_ptr(self):
                    return self.p
            for gp in gaps:
                rec(f"gap_{gp >> 10}k", i, i, View(base.data_ptr()), View(base.data_ptr() + cb + gp))
    elif pool:
        for i in range(n):
            c, o = pooled()
            rec("pool", i, i, c, o)
    elif contig or contig_out:
        for i in range(n):
            c, o = contig_pair(contig)
            rec("contig" if contig else "contig_out", i, i, c, o)
    else:
        coefs, outs = [coef_buf()], [out_buf()]
        rec("base", 0, 0, coefs[0], outs[0])
        for i in range(1, n + 1):
            coefs.append(coef_buf())
            rec("coef_only", i, 0, coefs[i], outs[0])
        for j in range(1, n + 1):
            outs.append(out_buf())
            rec("out_only", 0, j, coefs[0], outs[j])
        for i, j in ((1, 1), (2, 3), (n, n), (n // 2, 1)):
            rec("cross", i, j, coefs[i], outs[j])
        rec("base_again", 0, 0, coefs[0], outs[0])
    fr = {}
    for r in rows:
        fr.setdefault(r["kind"], []).append(r["frac"])
    print(json.dumps({"summary": {k: {"min": min(v), "max": max(v), "n": len(v)} for k, v in fr.items()}}), flush=True)


if __name__ == "__main__":
    main()
