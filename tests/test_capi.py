"""CPU: the product C ABI library loads, exports every symbol include/mj423gpu.h
declares, and its host-only arithmetic (geometry, byte accounting) is right.
No compute call is made here (there is no GPU in the build container)."""
import ctypes
import os
import re

import pytest

from conftest import PKG, REPO

HEADERS = [os.path.join(REPO, "include", h) for h in sorted(os.listdir(os.path.join(REPO, "include")))
           if h.endswith(".h")]


def declared_functions():
    names = set()
    for hdr in HEADERS:
        src = open(hdr).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        src = re.sub(r"typedef[^;]*\(\s*\*[^;]*;", "", src)  # function-pointer typedefs declare no symbol
        names |= set(re.findall(r"\b([A-Za-z_][A-Za-z0-9_]*)\s*\([^;{]*\)\s*;", src))
    return sorted(n for n in names if n not in ("if", "sizeof"))


def test_header_declares_reference_surface():
    names = set(declared_functions())
    # mj/decoder/mjpeg423_decoder.h:15-16 and c0/idct_ycbcr_to_rgb_accel.h:13-22
    for ref in ("idct", "ycbcr_to_rgb", "init_idct_ycbcr_to_rgb_accel", "idct_accel_calculate_buffer_y",
                "idct_accel_calculate_buffer_cb", "idct_accel_calculate_buffer_cr", "ycbcr_to_rgb_accel_get_results",
                "ycbcr_to_rgb_accel_calculate_buffer", "wait_for_ycbcr_to_rgb_finsh", "wait_for_idct_y_finsh",
                "decode_frame", "decode_frames", "lossless_decode", "mjpeg423_decode", "encode_bmp"):
        assert ref in names


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(os.path.join(PKG, "libmj423gpu.so"))
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_geometry_and_bytes():
    import mj423
    g = mj423.geometry(1920, 1080, 420)
    assert (g.coded_w, g.coded_h, g.y_blocks, g.c_blocks) == (1920, 1088, 32640, 8160)
    # SURVEY §8(d) algorithmic bytes per frame
    assert mj423.frame_bytes(640, 480, 444) == 3_072_000
    assert mj423.frame_bytes(1920, 1080, 420) == 14_561_280
    assert mj423.frame_bytes(3840, 2160, 420) == 58_060_800
    assert mj423.frame_bytes(7680, 4320, 422) == 265_420_800
    g = mj423.geometry(7680, 4320, 422)
    assert (g.y_blocks, g.c_blocks) == (518400, 259200)
    for bad in ((0, 8, 444), (8, 8, 411), (8, 0, 420)):
        with pytest.raises(mj423.Mj423Error):
            mj423.geometry(*bad)


def test_geometry_matches_oracle(orc):
    import mj423
    for w, h, c in ((640, 480, 444), (1920, 1080, 420), (33, 17, 420), (100, 9, 422), (8, 8, 444)):
        a, b = mj423.geometry(w, h, c), orc.geometry(w, h, c)
        assert (a.coded_w, a.coded_h, a.y_bw, a.c_bw, a.y_blocks, a.c_blocks) == \
               (b.coded_w, b.coded_h, b.y_bw, b.c_bw, b.y_blocks, b.c_blocks)


def test_no_silent_cpu_fallback():
    """Without a HIP device the product refuses loudly instead of computing on the CPU."""
    import mj423
    try:
        import torch
        if torch.cuda.device_count() > 0:
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    with pytest.raises(mj423.Mj423Error) as e:
        mj423.Context(0)
    assert "no HIP device" in str(e.value) or "EHIP" in str(e.value)


def test_frame_range_matches_shard():
    """mj423_frame_range (C ABI, used by the C multi-GPU group) == shard.frame_range (torch ranks)."""
    import mj423
    import shard
    for world in (1, 2, 3, 4, 7, 8):
        for total in (0, 1, 5, 300, 601, 2400):
            rs = [mj423.frame_range(r, world, total) for r in range(world)]
            assert [(f, f + c) for f, c in rs] == [shard.frame_range(r, world, total) for r in range(world)]
    with pytest.raises(mj423.Mj423Error):
        mj423.frame_range(2, 2, 10)


def test_multi_group_refuses_without_gpu():
    """The multi-GPU group has no CPU path either."""
    import mj423
    try:
        import torch
        if torch.cuda.device_count() > 0:
            pytest.skip("a GPU is present")
    except ImportError:
        pass
    with pytest.raises(mj423.Mj423Error) as e:
        mj423.Multi(2)
    assert "no HIP device" in str(e.value)


def test_multigpu_c_driver_is_built():
    """The plain-C host driver of the multi-GPU group links against the product library."""
    exe = os.path.join(PKG, "mj423_multigpu")
    assert os.access(exe, os.X_OK), "run make -C mjpeg423-video-decoder-software_amd"
    import subprocess
    r = subprocess.run([exe, "--bogus"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2 and "unknown or incomplete argument" in r.stderr


def test_gop_ranges_start_at_iframes():
    """mj423_mpg_gop_ranges (host only): the multi-GPU .mpg split cuts at I-frames."""
    from conftest import GOLDEN
    import mj423
    m = mj423.Mpg(os.path.join(GOLDEN, "stream_320x240.mpg"))
    n = m.header.num_frames
    types = [m.frame(i).frame_type for i in range(n)]
    for world in (1, 2, 3, 4, 8):
        rs = mj423.mpg_gop_ranges(m, 0, n, world)
        assert rs[0][0] == 0 and sum(c for _, c in rs) == n
        assert all(a + c == b for (a, c), (b, _) in zip(rs, rs[1:]))
        assert all(types[f] == 0 for f, c in rs if c)
    # a range that starts inside a GOP keeps its start (that rank seeds from the GOP's I-frame)
    rs = mj423.mpg_gop_ranges(m, 5, n - 5, 2)
    assert rs[0][0] == 5 and rs[1][0] + rs[1][1] == n


def test_accelerator_submission_before_init_is_reported():
    """The reference's accelerator calls return void (c0/idct_ycbcr_to_rgb_accel.h:13-22):
    a submission the library cannot honour is recorded in mj423_accel_status(), never
    silently dropped.  No device is touched: the accelerator is not initialised here."""
    import mj423
    L = mj423.lib()
    buf = (ctypes.c_int16 * 64)()
    assert mj423.Accelerator.status() == 0
    L.idct_accel_calculate_buffer_y(ctypes.cast(buf, ctypes.c_void_p), ctypes.c_uint32(128))
    L.wait_for_idct_y_finsh()
    assert "init_idct_ycbcr_to_rgb_accel" in mj423.last_error()
    assert mj423.Accelerator.status() == -4  # MJ423_ESTATE
    assert "has not succeeded" in mj423.last_error()
    assert mj423.Accelerator.status() == 0  # read-and-clear
    L.ycbcr_to_rgb_accel_get_results(None, ctypes.c_uint32(0))
    assert mj423.Accelerator.status() == -4


def test_per_block_symbols_report_failures_without_a_device():
    """idct()/ycbcr_to_rgb() return void like the reference's (mjpeg423_decoder.h:15-16);
    with no HIP device they record the failure (mj423_dropin_status) instead of computing
    anything on the host: the product has no CPU fallback."""
    import mj423
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    L = mj423.lib()
    blk = (ctypes.c_int16 * 64)()
    out = (ctypes.c_uint8 * 64)(*([7] * 64))
    prev = L.mj423_dropin_defer(1)
    try:
        for defer in (1, 0):  # deferred mode and immediate mode
            L.mj423_dropin_defer(defer)
            L.mj423_dropin_status()
            L.idct(ctypes.cast(blk, ctypes.c_void_p), ctypes.cast(out, ctypes.c_void_p))
            assert L.mj423_dropin_flush() in (0, -2)
            assert L.mj423_dropin_status() == -2  # MJ423_EHIP
            assert "no CPU fallback" in mj423.last_error()
            assert list(out) == [7] * 64  # nothing written
            assert L.mj423_dropin_status() == 0
    finally:
        L.mj423_dropin_defer(prev if prev in (0, 1, 2) else 2)
