"""CPU: the oracle restatement (oracle/mj423_oracle.c) pinned against the golden
fixtures generated from the reference's own C (oracle/gen_golden.py), and -- when
oracle/_ref is built -- against the reference library directly."""
import ctypes
import os

import numpy as np
import pytest


@pytest.mark.parametrize("name", ["idct_directed.npz", "idct_realistic.npz", "idct_wrap.npz"])
def test_idct_fixtures(golden, manifest, orc, name):
    d = golden(name)
    out = orc.idct_blocks(d["inp"])
    assert np.array_equal(out, d["out"])
    assert orc.fnv1a64(out) == manifest["fixtures"][name[:-4]]["out_fnv1a64"]


def test_csc_sample(golden, orc):
    d = golden("csc_sample.npz")
    t = d["ycbcr"]
    got = orc.ycbcr_pixels(t[:, 0], t[:, 1], t[:, 2])
    assert np.array_equal(got, d["bgra"])


def test_csc_exhaustive_hash(manifest, orc):
    assert orc.csc_exhaustive_hash() == manifest["fixtures"]["csc_sample"]["exhaustive_fnv1a64"]


def test_tables_match_reference(manifest, orc):
    t = manifest["tables"]
    assert orc.YQUANT.tolist() == t["yquant"]
    assert orc.CQUANT.tolist() == t["cquant"]


def _stream(golden):
    return golden("stream_640x480.npz")


@pytest.mark.parametrize("frame", [0, 1])
def test_front_end_reference_semantics(golden, manifest, orc, frame):
    """lossless_decode restatement (dequantizing form) reproduces the reference's DCAC planes,
    I-frame then P-frame accumulating into the same buffers (decoder/lossless_decode.c:60-135)."""
    s = _stream(golden)
    nb = 4800
    quant = {"Y": orc.YQUANT, "Cb": orc.CQUANT, "Cr": orc.CQUANT}
    for plane in ("Y", "Cb", "Cr"):
        dcac = orc.lossless_decode_ref(nb, s[f"f0_{plane}_stream"], quant[plane], 0)
        if frame == 1:
            dcac = orc.lossless_decode_ref(nb, s[f"f1_{plane}_stream"], quant[plane], 1, prev=dcac)
        assert orc.fnv1a64(dcac) == manifest["fixtures"][f"stream_640x480_f{frame}"]["dcac_fnv1a64"][plane]


@pytest.mark.parametrize("frame", [0, 1])
def test_quantized_domain_identity(golden, manifest, orc, frame):
    """decoding to absolute quantized coefficients and dequantizing with
    (int16)(Q*q) equals the reference's dequantizing decoder, for I and P frames."""
    s = _stream(golden)
    nb = 4800
    quant = {"Y": orc.YQUANT, "Cb": orc.CQUANT, "Cr": orc.CQUANT}
    for plane in ("Y", "Cb", "Cr"):
        q = orc.lossless_decode_q(nb, s[f"f0_{plane}_stream"], 0)
        if frame == 1:
            q = orc.lossless_decode_q(nb, s[f"f1_{plane}_stream"], 1, prev=q)
        assert np.array_equal(q, s[f"f{frame}_{plane}_q"])  # the encoder's absolute coefficients
        deq = orc.dequant(q, quant[plane])
        assert orc.fnv1a64(deq) == manifest["fixtures"][f"stream_640x480_f{frame}"]["dcac_fnv1a64"][plane]


@pytest.mark.parametrize("frame", [0, 1])
def test_decode_frame_640x480(golden, manifest, orc, frame):
    """decode_frame on quantized planes == the reference pipeline's BGRA frame (BASELINE config 1)."""
    s = _stream(golden)
    out = orc.decode_frame(s[f"f{frame}_Y_q"], s[f"f{frame}_Cb_q"], s[f"f{frame}_Cr_q"], 640, 480, 444)
    assert np.array_equal(out[::16], s[f"f{frame}_bgra_rows16"])
    assert orc.fnv1a64(out) == manifest["fixtures"][f"stream_640x480_f{frame}"]["bgra_fnv1a64"]


def test_chroma_fetch_rule(orc):
    """4:2:0 / 4:2:2 extension: every pixel equals the 4:4:4 reference CSC
    of (Y(x,y), C(x/2, y/sy)) where the planes are the per-block IDCT outputs."""
    rng = np.random.default_rng(5)
    for chroma, sy in ((420, 2), (422, 1)):
        w, h = 48, 32
        g = orc.geometry(w, h, chroma)
        coef = orc.random_quantized_planes(rng, w, h, chroma)[0]
        Y, Cb, Cr = coef[:g.y_blocks], coef[g.y_blocks:g.y_blocks + g.c_blocks], coef[g.y_blocks + g.c_blocks:]
        out = orc.decode_frame(Y, Cb, Cr, w, h, chroma)
        yp = orc.idct_blocks(orc.dequant(Y, orc.YQUANT)).reshape(g.y_bh, g.y_bw, 8, 8).transpose(0, 2, 1, 3).reshape(g.y_bh * 8, g.y_bw * 8)
        cbp = orc.idct_blocks(orc.dequant(Cb, orc.CQUANT)).reshape(g.c_bh, g.c_bw, 8, 8).transpose(0, 2, 1, 3).reshape(g.c_bh * 8, g.c_bw * 8)
        crp = orc.idct_blocks(orc.dequant(Cr, orc.CQUANT)).reshape(g.c_bh, g.c_bw, 8, 8).transpose(0, 2, 1, 3).reshape(g.c_bh * 8, g.c_bw * 8)
        ys, xs = np.mgrid[0:h, 0:w]
        exp = orc.ycbcr_pixels(yp[ys, xs], cbp[ys // sy, xs // 2], crp[ys // sy, xs // 2]).reshape(h, w)
        assert np.array_equal(out, exp)


def test_oracle_vs_reference_random(orc):
    """Randomized equivalence against the reference library itself (build container only)."""
    ref = orc.ref_lib()
    if ref is None:
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    rng = np.random.default_rng(99)
    blocks = np.concatenate([rng.integers(-32768, 32768, size=(20000, 64), dtype=np.int16),
                             rng.integers(-2048, 2048, size=(20000, 64), dtype=np.int16)])
    exp = np.empty((len(blocks), 64), np.uint8)
    ref.ref_idct_batch(len(blocks), blocks.ctypes.data_as(ctypes.c_void_p), exp.ctypes.data_as(ctypes.c_void_p))
    assert np.array_equal(orc.idct_blocks(blocks), exp)
    # full 4:4:4 frame on dequantized planes
    w, h = 128, 64
    nb = (w // 8) * (h // 8)
    planes = [rng.integers(-1500, 1500, size=(nb, 64), dtype=np.int16) for _ in range(3)]
    scratch = np.empty(3 * nb * 64, np.uint8)
    exp = np.empty(w * h, np.uint32)
    ref.ref_decode_frame_444(w, h, *[p.ctypes.data_as(ctypes.c_void_p) for p in planes],
                             scratch.ctypes.data_as(ctypes.c_void_p), exp.ctypes.data_as(ctypes.c_void_p))
    got = orc.decode_frame(*planes, w, h, 444, dequantized=True)
    assert np.array_equal(got.ravel(), exp)


@pytest.mark.parametrize("chroma,w,h", [(420, 64, 48), (420, 40, 24), (422, 48, 40), (444, 24, 16)])
def test_reference_subsampled_frame_loop_matches_oracle(orc, chroma, w, h):
    """oracle/ref_harness.c ref_decode_frame_sub (the reference's own idct() + ycbcr_to_rgb()
    with the A7 chroma gather; bench.py's `kind: reference` CPU baseline for 4:2:x) equals
    the oracle frame decode, wrap regime included (build container only)."""
    ref = orc.ref_lib()
    if ref is None:
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    g = orc.geometry(w, h, chroma)
    rng = np.random.default_rng(7 + chroma)
    Y, Cb, Cr = (rng.integers(-32768, 32768, size=(n, 64), dtype=np.int16) if i == 0 else
                 rng.integers(-1500, 1500, size=(n, 64), dtype=np.int16)
                 for i, n in enumerate((g.y_blocks, g.c_blocks, g.c_blocks)))
    cw, ch = g.y_bw * 8, g.y_bh * 8
    scratch = np.empty(64 * (g.y_blocks + 2 * g.c_blocks), np.uint8)
    exp = np.empty((ch, cw), np.uint32)
    P = ctypes.c_void_p
    ref.ref_decode_frame_sub(ctypes.c_uint32(cw), ctypes.c_uint32(ch), ctypes.c_int(chroma),
                             Y.ctypes.data_as(P), Cb.ctypes.data_as(P), Cr.ctypes.data_as(P),
                             scratch.ctypes.data_as(P), exp.ctypes.data_as(P))
    got = orc.decode_frame(Y, Cb, Cr, w, h, chroma, dequantized=True)
    assert np.array_equal(got, exp[:h, :w])


@pytest.mark.parametrize("name", ["stream_160x96", "stream_320x240", "stream_100x60"])
def test_reference_decoder_loop_harness_matches_reference_bmps(manifest, orc, tmp_path, name):
    """oracle/ref_harness.c:ref_decode_mpg_frames -- the reference's decoder loop
    (mjpeg423_decoder.c:90-124: lossless_decode x3, idct, ycbcr_to_rgb; the file-mode CPU baseline
    of bench.py) -- over every frame of the reference-encoded golden files: each frame's BMP equals
    the one the reference decoder itself wrote (SHA-256 of the file, or of the coded region)."""
    import ctypes
    import struct
    import mj423
    from conftest import GOLDEN, coded_region_sha256
    ref = orc.ref_lib()
    if ref is None:
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    fx = manifest["fixtures"][name]
    data = np.fromfile(os.path.join(GOLDEN, f"{name}.mpg"), np.uint8)
    n, w, h = struct.unpack("<3I", data[:12].tobytes())
    m = mj423.Mpg(os.path.join(GOLDEN, f"{name}.mpg"))
    pos = np.array([m.frame(i).position for i in range(n)], np.uint64)
    P = ctypes.c_void_p
    for f in range(n):
        g0 = m.gop_start(f)
        rgb = np.zeros((h, w), np.uint32)
        got = ref.ref_decode_mpg_frames(data.ctypes.data_as(P), pos.ctypes.data_as(P), ctypes.c_uint32(g0),
                                        ctypes.c_uint32(f + 1), ctypes.c_uint32(w), ctypes.c_uint32(h),
                                        rgb.ctypes.data_as(P))
        assert got == f + 1 - g0
        p = tmp_path / "f.bmp"
        mj423.write_bmp(str(p), rgb)
        if "decoded_bmp_sha256" in fx:
            import hashlib
            assert hashlib.sha256(p.read_bytes()).hexdigest() == fx["decoded_bmp_sha256"][f], (name, f)
        else:
            assert coded_region_sha256(p.read_bytes(), w, h) == fx["decoded_coded_region_sha256"][f], (name, f)
    m.close()
