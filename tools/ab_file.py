"""Same-process A/B of library builds on the whole-file GPU decode (mj423_mpg_decode_gpu,
bench.py --mode file --frontend gpu), measurements only.  Every build named on the command line
is loaded into ONE process (ctypes, RTLD_LOCAL: each keeps its own kernels and contexts), opens
the SAME seeded synthetic .mpg (tools/mpg_synth) and decodes it into its own HBM buffer, in
interleaved rounds; prints per build the median pass time and Gpix/s, and checks that every
build's frames equal the first build's.

  python tools/ab_file.py ROUNDS [W H FRAMES GOP] -- lib_a.so lib_b.so@MJ423_GPU_FE_FUSED=0 ...

A build may carry @VAR=VALUE settings: the library reads them (getenv) on every call, so they are
set in the environment around that build's calls only.

AB_FILE=path.mpg: time that file instead of a synthetic one.

AB_SAME_OUT=1: every build decodes into ONE output buffer, each build's frames compared after its
own final call.

Caveat (round 5): a position artifact -- one build of the list runs ~1 ms slower per pass, the
same build in every round -- is not its kernels (tools/ab_trace.py: equal kernel times) but its
context stream sharing a hardware queue with a copy stream (GPU_MAX_HW_QUEUES=4 for three
streams per context): its setup kernels wait behind the whole upload.  Settings that change the
schedule are compared one process per run instead (tools/win_ab.sh).
"""
import ctypes
import os
import sys
import tempfile
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import torch  # noqa: E402

import mpg_synth  # noqa: E402

SEED = 0x4D4A3432


def main():
    sep = sys.argv.index("--")
    args, paths = sys.argv[1:sep], sys.argv[sep + 1:]
    rounds = int(args[0])
    w, h, n, gop = (int(x) for x in args[1:5]) if len(args) >= 5 else (1920, 1080, 240, 24)
    given = os.environ.get("AB_FILE")  # an existing .mpg instead (e.g. tools/real_mpg.py's)
    if given:
        import struct
        with open(given, "rb") as fh:
            n, w, h = struct.unpack("<3I", fh.read(12))
        path = given
    else:
        path = os.path.join(tempfile.mkdtemp(prefix="mj423ab"), "ab.mpg")
        mpg_synth.write(path, w, h, n, gop=gop, seed=SEED, nthreads=16)
    dev = torch.device("cuda", 0)
    same = os.environ.get("AB_SAME_OUT") == "1"
    outs = [torch.empty((n, h, w), dtype=torch.int32, device=dev) for _ in (paths[:1] if same else paths)]
    outs = outs * len(paths) if same else outs
    libs, ctxs, mpgs, envs = [], [], [], []
    for spec in paths:
        p, *kv = spec.split("@")
        envs.append(dict(x.split("=", 1) for x in kv))
        L = ctypes.CDLL(os.path.abspath(p))
        c, m = ctypes.c_void_p(), ctypes.c_void_p()
        assert L.mj423_ctx_create(ctypes.byref(c), 0) == 0
        assert L.mj423_mpg_open(path.encode(), ctypes.byref(m)) == 0
        libs.append(L)
        ctxs.append(c)
        mpgs.append(m)

    def one(i):
        saved = {k: os.environ.get(k) for k in envs[i]}
        os.environ.update(envs[i])
        try:
            return _one(i)
        finally:
            for k, v in saved.items():
                if v is None:
                    os.environ.pop(k, None)
                else:
                    os.environ[k] = v

    def _one(i):
        t = time.perf_counter()
        rc = libs[i].mj423_mpg_decode_gpu(ctxs[i], mpgs[i], ctypes.c_uint32(0), ctypes.c_uint32(n),
                                          ctypes.c_void_p(outs[i].data_ptr()), ctypes.c_uint64(w * h),
                                          ctypes.c_uint32(0))
        assert rc == 0, rc
        return time.perf_counter() - t  # (the call synchronises its stream before returning)

    for i in range(len(paths)):  # warm-up: buffers, code objects, clocks
        for _ in range(5):
            one(i)
    times = [[] for _ in paths]
    for _ in range(rounds):
        for i in range(len(paths)):
            for _ in range(5):
                times[i].append(one(i))
    torch.cuda.synchronize()
    ref = None
    for i, spec in enumerate(paths):
        if same:
            one(i)  # this build's frames in the shared buffer
        ref = outs[0].cpu() if ref is None else ref
        ms = float(np.median(times[i])) * 1e3
        eq = bool(torch.equal(outs[i].cpu(), ref))
        p, *kv = spec.split("@")
        label = os.path.basename(os.path.dirname(os.path.abspath(p))) + "".join("@" + x for x in kv)
        print(f"file {w}x{h}x{n} {label}: median {ms:.3f} ms  min {min(times[i]) * 1e3:.3f} ms  "
              f"{n * w * h / (ms * 1e-3) / 1e9:.1f} Gpix/s  output equal to the first build: {eq}", flush=True)
    if not given:
        os.remove(path)


if __name__ == "__main__":
    main()
