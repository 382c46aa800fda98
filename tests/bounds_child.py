"""Child process of tests/test_gpu_parity.py::test_whole_file_decode_under_bounds_checks (not a test
module): the whole-file GPU decode paths through libmj423gpu_bounds.so, the bounds-check build
(csrc/mj423_check.hpp: every index the entropy, index, fused and margin kernels derive from a table is
checked against its allocation; a miss prints "mj423 bound: ..." and traps).  Every frame is compared
with the oracle; prints "bounds child OK" at the end.  Runs with MJ423_LIB pointing at that build."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
for p in (os.path.join(REPO, "mjpeg423-video-decoder-software_amd"), os.path.join(REPO, "oracle"),
          os.path.join(REPO, "tools"), HERE):
    sys.path.insert(0, p)
import torch  # noqa: E402

import mj423  # noqa: E402
import mpg_synth  # noqa: E402
import oracle  # noqa: E402
from conftest import GOLDEN, oracle_frames_any_size, static_scene  # noqa: E402


def frames(ctx, m, first, count, window=0):
    w, h = m.header.width, m.header.height
    out = torch.full((max(count, 1), h, w), -1, dtype=torch.int32, device="cuda:0")
    torch.cuda.synchronize()
    m.decode_gpu(ctx, first, count, out.data_ptr(), window_frames=window)
    torch.cuda.synchronize()
    return out[:count].cpu().numpy().view(np.uint32)


def main():
    assert "bounds" in mj423.LIB_PATH, mj423.LIB_PATH
    tmp = sys.argv[1]
    ctx = mj423.Context(0)
    n_checked = 0
    # the reference encoder's files: every frame, windows of 5, the default schedule, and a seek
    for name in ("stream_160x96", "stream_320x240", "stream_100x60"):
        m = mj423.Mpg(os.path.join(GOLDEN, f"{name}.mpg"))
        w, h, n = m.header.width, m.header.height, m.header.num_frames
        want = m.decode(ctx, 0, n)  # host entropy decode + the GPU transform (mj423_decode_mpg)
        for first, window in ((0, 5), (0, 0), (3, 1), (n - 1, 0)):
            got = frames(ctx, m, first, n - first, window)
            assert np.array_equal(got, want[first:]), (name, first, window)
            n_checked += n - first
        m.close()
    # synthetic files: window schedules that cut GOPs, sizes that are not multiples of 8
    for (w, h, n, gop, seed, windows) in ((320, 240, 14, 5, 11, "1,1,1,1,1,1,1"), (320, 240, 14, 5, 12, "5,1,1"),
                                          (100, 60, 9, 4, 13, "1,2,3"), (1921, 1083, 4, 3, 14, "1,2,3"),
                                          (96, 64, 30, 7, 51, "1,2,3")):
        a, s, t = mpg_synth.generate(w, h, n, gop=gop, seed=seed)
        path = os.path.join(tmp, f"b{w}x{h}_{seed}.mpg")
        mpg_synth.write_coef(path, w, h, t, s)
        m = mj423.Mpg(path)
        os.environ["MJ423_GPU_FE_WINDOWS"] = windows
        want = oracle_frames_any_size(oracle, a, n, w, h)
        for first in (0, 2):
            got = frames(ctx, m, first, n - first)
            assert np.array_equal(got, want[first:]), (w, h, windows, first)
            n_checked += n - first
        del os.environ["MJ423_GPU_FE_WINDOWS"]
        m.close()
    # static-scene P-frames: the multi-class resolution (entmc_* kernels), windows that cut the GOP
    for (w, h, n, seed, windows) in ((640, 480, 8, 21, "1,3,4"), (200, 120, 12, 22, "5,1,6")):
        a, s, t = static_scene(w, h, n, seed)
        path = os.path.join(tmp, f"static{w}x{h}_{seed}.mpg")
        mpg_synth.write_coef(path, w, h, t, s)
        m = mj423.Mpg(path)
        os.environ["MJ423_GPU_FE_WINDOWS"] = windows
        want = oracle_frames_any_size(oracle, a, n, w, h)
        for first in (0, 3):
            got = frames(ctx, m, first, n - first)
            assert np.array_equal(got, want[first:]), (w, h, windows, first)
            n_checked += n - first
        del os.environ["MJ423_GPU_FE_WINDOWS"]
        m.close()
    # damaged streams (the reference files and a synthetic one, bytes flipped inside the frames'
    # payloads): accepted or rejected exactly as the host front end accepts or rejects them, accepted
    # ones equal to the oracle's decode of the host's coefficients -- and no bound trips on any of them
    trials = int(os.environ.get("MJ423_BOUNDS_FUZZ", "60"))
    rng = np.random.default_rng(20261018)
    a, s, t = mpg_synth.generate(48, 32, 7, gop=4, seed=6)
    synth = os.path.join(tmp, "fz.mpg")
    mpg_synth.write_coef(synth, 48, 32, t, s)
    sources = [synth] + [os.path.join(GOLDEN, f"{nm}.mpg") for nm in ("stream_160x96", "stream_100x60")]
    agree = rejected = 0
    for trial in range(trials):
        raw = bytearray(open(sources[trial % len(sources)], "rb").read())
        for _ in range(int(rng.integers(1, 6))):
            raw[int(rng.integers(40, len(raw) - 600))] ^= int(rng.integers(1, 256))
        try:
            m = mj423.Mpg(bytes(raw))
        except mj423.Mj423Error:
            rejected += 1
            continue
        n, w, h = m.header.num_frames, m.header.width, m.header.height
        try:
            host = m.entropy_decode(0, n)
        except mj423.Mj423Error:
            host = None
        try:
            got = frames(ctx, m, 0, n, window=int(rng.integers(0, 4)))
        except mj423.Mj423Error:
            got = None
        assert (host is None) == (got is None), trial
        if host is not None:
            want = oracle_frames_any_size(oracle, host.reshape(n, -1), n, w, h)
            assert np.array_equal(got, want), trial
            agree += 1
        m.close()
    ctx.close()
    print(f"bounds child OK: {n_checked} frames through the bounds-check build, all equal to the oracle; "
          f"{trials} damaged streams: {agree} decoded equal to the oracle, {trials - agree - rejected} rejected by "
          f"both front ends, {rejected} rejected at open", flush=True)


if __name__ == "__main__":
    main()
