"""CPU: the product's host side (include/mj423io.h) -- entropy front end, .mpg
container, BMP sink -- against the reference's own outputs (golden fixtures made by
the reference encoder/decoder, oracle/gen_golden.py) and the oracle.  These are
host-only code paths (the reference runs them on its CPU too); no GPU is needed."""
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, check_bmp_against_fixture, coded_region_sha256, oracle_frames_any_size


def _mpg(name):
    import mj423
    return mj423.Mpg(os.path.join(GOLDEN, f"{name}.mpg"))


@pytest.mark.parametrize("frame", [0, 1])
def test_reference_lossless_decode_symbol(golden, manifest, orc, frame):
    """lossless_decode() (dequantizing, decoder/lossless_decode.c:60) reproduces the reference's
    DCAC planes of the 640x480 I+P stream bit for bit."""
    import mj423
    s = golden("stream_640x480.npz")
    quant = {"Y": orc.YQUANT, "Cb": orc.CQUANT, "Cr": orc.CQUANT}
    for plane in ("Y", "Cb", "Cr"):
        dcac = np.zeros((4800, 64), np.int16)
        mj423.lossless_decode(4800, s[f"f0_{plane}_stream"].tobytes(), dcac, quant[plane], False)
        if frame == 1:
            mj423.lossless_decode(4800, s[f"f1_{plane}_stream"].tobytes(), dcac, quant[plane], True)
        assert orc.fnv1a64(dcac) == manifest["fixtures"][f"stream_640x480_f{frame}"]["dcac_fnv1a64"][plane]


def test_quantized_front_end_matches_encoder(golden, orc):
    import mj423
    s = golden("stream_640x480.npz")
    for plane in ("Y", "Cb", "Cr"):
        q0 = mj423.lossless_decode_q(4800, s[f"f0_{plane}_stream"].tobytes(), False)
        assert np.array_equal(q0, s[f"f0_{plane}_q"])
        q1 = mj423.lossless_decode_q(4800, s[f"f1_{plane}_stream"].tobytes(), True, prev=q0)
        assert np.array_equal(q1, s[f"f1_{plane}_q"])
        assert np.array_equal(q1, orc.lossless_decode_q(4800, s[f"f1_{plane}_stream"], 1, prev=q0))


def test_front_end_random_streams_vs_reference(orc):
    """Randomized: bitstreams written by the reference's lossless_encode over random sparse
    quantized blocks (incl. ZRL runs and long amplitudes) decode exactly as the reference's
    own lossless_decode decodes them.  (The reference encoder's final flush can drop the
    last few bits of the stream -- e.g. 325 comes back as 320 -- and the reference decoder
    reproduces that; the oracle is the reference decoder, not the encoder's input.  The
    reference encoder also corrupts streams whose amplitudes need more than ~12 bits, after
    which its decoder indexes past the zig-zag table and crashes, so amplitudes stay within
    +/-2047 here; the product's front end guards that index instead of crashing.)"""
    import ctypes
    import mj423
    ref = orc.ref_lib()
    if ref is None:
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    ref.lossless_encode.restype = ctypes.c_uint32
    rng = np.random.default_rng(5)
    for trial in range(6):
        n = 300
        blocks = np.zeros((n, 64), np.int16)
        nz = rng.random((n, 64)) < [0.9, 0.5, 0.2, 0.05, 0.01][trial % 5]
        mag = rng.integers(-1023, 1024, size=(n, 64)) if trial < 3 else rng.integers(-2047, 2048, size=(n, 64))
        blocks[nz] = mag[nz]
        blocks[blocks == 0] = 0
        buf = np.zeros(n * 64 * 4 + 64, np.uint8)
        nbytes = ref.lossless_encode(n, blocks.ctypes.data_as(ctypes.c_void_p), buf.ctypes.data_as(ctypes.c_void_p))
        stream = buf[:nbytes + 8].copy()
        exp = np.zeros((n, 64), np.int16)  # reference decoder with a unit table = quantized domain
        one = np.ones(64, np.int16)
        ref.lossless_decode(n, stream.ctypes.data_as(ctypes.c_void_p), exp.ctypes.data_as(ctypes.c_void_p),
                            one.ctypes.data_as(ctypes.c_void_p), 0)
        # all but the stream's tail agree with the encoder's input (DC re-accumulated)
        enc = blocks.copy()
        enc[:, 0] = np.cumsum(blocks[:, 0].astype(np.int64)).astype(np.int16)
        assert np.array_equal(exp[:-1], enc[:-1])
        assert np.array_equal(mj423.lossless_decode_q(n, stream.tobytes(), False), exp), trial
        assert np.array_equal(orc.lossless_decode_q(n, stream, 0), exp), trial


def test_truncated_stream_is_reported():
    import mj423
    with pytest.raises(mj423.Mj423Error):
        mj423.lossless_decode_q(100, b"\x5f\xff", False)


@pytest.mark.parametrize("name", ["stream_160x96", "stream_320x240", "stream_100x60"])
def test_mpg_container(manifest, name):
    fx = manifest["fixtures"][name]
    m = _mpg(name)
    h = m.header
    assert [h.num_frames, h.width, h.height, h.num_iframes, h.payload_size] == fx["header"]
    types = [m.frame(i).frame_type for i in range(h.num_frames)]
    assert types[0] == 0 and sum(1 for t in types if t == 0) == h.num_iframes
    idx, pos = m.trailer()
    assert list(idx) == [i for i, t in enumerate(types) if t == 0]
    for i in idx:
        assert m.gop_start(int(i)) == int(i)
    for i in range(h.num_frames):
        g = m.gop_start(i)
        assert types[g] == 0 and all(t == 1 for t in types[g + 1:i + 1])
    with pytest.raises(Exception):
        m.frame(h.num_frames)


def test_mpg_trailer_positions_point_at_iframes(manifest):
    """The trailer's frame_position is relative to the end of the 20-byte header
    (mjpeg423_encoder.c:82-88, file_position starts counting at the header size)."""
    m = _mpg("stream_320x240")
    idx, pos = m.trailer()
    for i, p in zip(idx, pos):
        assert m.frame(int(i)).position == int(p)


def _oracle_decode_mpg(orc, m, first, count):
    """Oracle chain: quantized-domain front end from the GOP start + oracle frame decode."""
    w, h = m.header.width, m.header.height
    nb = (w // 8) * (h // 8)
    g0 = m.gop_start(first)
    import ctypes
    state = [None, None, None]
    out = []
    for f in range(g0, first + count):
        fr = m.frame(f)
        P = fr.frame_type != 0
        for pi, (ptr, size) in enumerate(((fr.y, fr.y_size), (fr.cb, fr.cb_size), (fr.cr, fr.cr_size))):
            bs = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint8)), shape=(size,)).copy()
            state[pi] = orc.lossless_decode_q(nb, np.concatenate([bs, np.zeros(8, np.uint8)]), P,
                                              prev=state[pi] if P else None)
        if f >= first:
            out.append(orc.decode_frame(state[0], state[1], state[2], w, h, 444))
    return np.stack(out)


@pytest.mark.parametrize("name", ["stream_160x96", "stream_320x240", "stream_100x60"])
def test_entropy_decode_threads_and_gop_seek(orc, name):
    m = _mpg(name)
    n = m.header.num_frames
    full = m.entropy_decode(0, n, nthreads=4)
    for first in (0, 1, 5, n - 1):
        part = m.entropy_decode(first, n - first, nthreads=3)
        assert np.array_equal(part, full[first:])
    one = m.entropy_decode(0, n, nthreads=1)
    assert np.array_equal(one, full)


def test_bmp_writer_matches_reference_bytes(tmp_path, golden, orc):
    """Oracle-decoded frame 0 written by the product's BMP sink is byte-identical to the
    BMP the reference's own decoder wrote (libbmp bmp_save)."""
    import mj423
    m = _mpg("stream_160x96")
    frame0 = _oracle_decode_mpg(orc, m, 0, 1)[0]
    p = tmp_path / "x0000.bmp"
    mj423.write_bmp(str(p), frame0)
    with open(os.path.join(GOLDEN, "stream_160x96_dec0000.bmp"), "rb") as f:
        assert p.read_bytes() == f.read()


@pytest.mark.parametrize("name", ["stream_160x96", "stream_320x240", "stream_100x60"])
def test_front_end_chain_reproduces_reference_decoder(tmp_path, manifest, orc, name):
    """Every frame: product front end -> oracle pixel path -> product BMP writer gives the
    SHA-256 of the BMP the reference's mjpeg423_decode wrote (P-frames included); at 100x60
    (not multiples of 8) the coded region's, i.e. the w/8 x h/8 whole blocks."""
    import mj423
    fx = manifest["fixtures"][name]
    m = _mpg(name)
    w, h, n = m.header.width, m.header.height, m.header.num_frames
    frames = oracle_frames_any_size(orc, m.entropy_decode(0, n), n, w, h)
    for f in range(n):
        p = tmp_path / f"o{f:04d}.bmp"
        mj423.write_bmp(str(p), frames[f])
        check_bmp_against_fixture(p.read_bytes(), fx, f)


@pytest.mark.parametrize("w,h", [(100, 60), (7, 20), (20, 3), (5, 5), (9, 17), (8, 8), (65, 8)])
def test_mpg_any_frame_size(tmp_path, w, h):
    """Any frame size opens (the reference's encoder writes any w_size/h_size and codes the
    w/8 x h/8 whole blocks, mjpeg423_encoder.c:21-24): the stream's planes are those of
    mj423_geometry(w & ~7, h & ~7), none below 8, and the front end decodes exactly them."""
    import mj423
    import mpg_synth
    n = 5
    a, s, t = mpg_synth.generate(w, h, n, gop=2, seed=w * 131 + h)
    path = tmp_path / "a.mpg"
    mpg_synth.write_coef(path, w, h, t, s)
    m = mj423.Mpg(path)
    assert (m.header.width, m.header.height) == (w, h)
    g = m.geometry()
    nb = (w // 8) * (h // 8)
    assert (g.width, g.height, g.y_blocks, g.c_blocks, g.coef_per_frame) == (w // 8 * 8, h // 8 * 8, nb, nb, 192 * nb)
    assert np.array_equal(m.entropy_decode(0, n), a) and np.array_equal(m.entropy_decode(1, n - 1, nthreads=2), a[1:])
    d, ty = m.entropy_decode_deltas(0, n)
    assert np.array_equal(d, s) and np.array_equal(ty, t)


def test_mpg_size_limits():
    """Zero and over-2^20 sizes are refused at open."""
    import struct
    import mj423
    for w, h in ((0, 8), (8, 0), ((1 << 20) + 1, 8)):
        with pytest.raises(mj423.Mj423Error):
            mj423.Mpg(struct.pack("<5I", 0, w, h, 0, 0) + bytes(512))


@pytest.mark.parametrize("name", ["stream_160x96", "stream_320x240", "stream_100x60"])
def test_entropy_deltas_accumulate_to_absolute(name):
    """Per-frame deltas (I absolute, P own deltas) summed mod 2^16 over each GOP equal the
    host-accumulated absolute planes."""
    m = _mpg(name)
    n = m.header.num_frames
    absq = m.entropy_decode(0, n)
    deltas, types = m.entropy_decode_deltas(0, n, nthreads=5)
    assert [m.frame(i).frame_type for i in range(n)] == list(types)
    acc = None
    for f in range(n):
        acc = deltas[f].copy() if types[f] == 0 else (acc.astype(np.int32) + deltas[f]).astype(np.int16)
        assert np.array_equal(acc, absq[f]), f


# ---------------------------------------------- synthetic streams (tools/mpg_synth.cpp)
def test_synthetic_stream_writer_matches_reference_decoder(tmp_path, orc):
    """A stream written by tools/mpg_synth decodes under the reference's own mjpeg423_decode
    (oracle/_ref/mjref_app) to the BMPs that the product front end + oracle pixel path +
    product BMP writer give: the writer emits the reference's format, so larger synthetic
    streams are valid inputs for the benchmarks and GPU tests."""
    import hashlib
    import mj423
    import mpg_synth
    app = os.path.join(os.path.dirname(GOLDEN), "..", "oracle", "_ref", "mjref_app")
    if not os.path.exists(app):
        pytest.skip("oracle/_ref not built (needs /root/reference)")
    import subprocess
    for w, h, n in ((48, 40, 11), (53, 43, 6)):  # (53 x 43: the 48 x 40 whole blocks are coded)
        a, s, t = mpg_synth.generate(w, h, n, gop=4, seed=11)
        path = tmp_path / f"s{w}.mpg"
        mpg_synth.write_coef(path, w, h, t, s)
        subprocess.run([app, "decode", str(path), str(tmp_path / f"r{w}_0000.bmp")], check=True, capture_output=True,
                       timeout=60)
        m = mj423.Mpg(path)
        coef = m.entropy_decode(0, n)
        assert np.array_equal(coef, a)
        frames = oracle_frames_any_size(orc, coef, n, w, h)
        for f in range(n):
            p = tmp_path / f"o{f:04d}.bmp"
            mj423.write_bmp(str(p), frames[f])
            ref = (tmp_path / f"r{w}_{f:04d}.bmp").read_bytes()
            if w % 8 == 0 and h % 8 == 0:
                assert hashlib.sha256(p.read_bytes()).digest() == hashlib.sha256(ref).digest(), f
            else:
                assert coded_region_sha256(p.read_bytes(), w, h) == coded_region_sha256(ref, w, h), f


@pytest.mark.parametrize("w,h,gop", [(64, 48, 5), (160, 96, 24), (8, 8, 3)])
def test_front_end_on_synthetic_streams(tmp_path, w, h, gop):
    """Product front end on larger seeded streams: absolute planes from any start frame,
    per-frame deltas, and the bitstream bytes of each plane equal to the writer's."""
    import mj423
    import mpg_synth
    n = 2 * gop + 3
    a, s, t = mpg_synth.generate(w, h, n, gop=gop, seed=w * h)
    path = tmp_path / "s.mpg"
    mpg_synth.write_coef(path, w, h, t, s)
    m = mj423.Mpg(path)
    assert m.header.num_frames == n and m.header.num_iframes == (n + gop - 1) // gop
    for first in (0, 1, gop, n - 1):
        assert np.array_equal(m.entropy_decode(first, n - first, nthreads=3), a[first:])
    d, ty = m.entropy_decode_deltas(0, n, nthreads=4)
    assert np.array_equal(d, s) and np.array_equal(ty, t)


def test_container_and_front_end_survive_corruption():
    """Mutated / truncated reference streams: opening either fails with Mj423Error or
    indexes; every frame either decodes or reports an overrun -- never a crash, never a
    read outside the file -- and whatever decodes is the same through the absolute and
    the per-frame-delta forms of the front end, at any thread count."""
    import mj423
    rng = np.random.default_rng(1234)
    raw = open(os.path.join(GOLDEN, "stream_160x96.mpg"), "rb").read()
    opened = decoded = 0
    for trial in range(150):
        b = bytearray(raw)
        kind = trial % 3
        if kind == 0:  # flip payload bytes
            for _ in range(int(rng.integers(1, 20))):
                b[int(rng.integers(20, len(b)))] ^= int(rng.integers(1, 256))
        elif kind == 1:  # truncate
            b = b[:int(rng.integers(0, len(b)))]
        else:  # damage a header / frame-header word
            o = int(rng.choice([0, 4, 8, 12, 16, 20, 24, 28, 32]))
            if o + 4 <= len(b):
                b[o:o + 4] = int(rng.integers(0, 2**32)).to_bytes(4, "little")
        try:
            m = mj423.Mpg(bytes(b))
        except mj423.Mj423Error:
            continue
        opened += 1
        n = m.header.num_frames
        if n == 0 or n > 64 or m.header.width * m.header.height > 1 << 20:
            continue
        try:
            absq = m.entropy_decode(0, n, nthreads=3)
        except mj423.Mj423Error:
            continue
        decoded += 1
        d, t = m.entropy_decode_deltas(0, n, nthreads=2)
        acc = None
        for f in range(n):
            acc = d[f].copy() if t[f] == 0 else (acc.astype(np.int32) + d[f]).astype(np.int16)
            assert np.array_equal(acc, absq[f])
        assert np.array_equal(m.entropy_decode(0, n, nthreads=1), absq)
    assert opened > 10 and decoded > 5


def test_frontend_fuzz_under_asan():
    """The library's .mpg parser and entropy walk on 20 000 mutated inputs (bit flips, field
    overwrites in the header / frame tables / trailer, truncation, extension) with the host code
    built under AddressSanitizer (tools/fuzz_frontend.cpp, `make fuzz`): no invalid access, damaged
    files either rejected or decoded within their bounds, and the unmutated files still decode."""
    import json
    from conftest import GOLDEN, PKG, REPO
    exe = os.path.join(REPO, "tools", "fuzz_frontend")
    if not os.path.exists(exe):
        subprocess.run(["make", "-C", PKG, "-j8", "fuzz"], check=True, capture_output=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=1")
    r = subprocess.run([exe, "20000", "0x4D4A3432", os.path.join(GOLDEN, "stream_160x96.mpg"),
                        os.path.join(GOLDEN, "stream_320x240.mpg")], capture_output=True, text=True, timeout=600,
                       env=env)
    assert r.returncode == 0, r.stderr[-4000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["iterations"] == 20000 and d["opened"] > 0 and d["rejected"] > 0 and d["decoded"] > 0


def test_transfer_bound_holds_for_tightest_streams():
    """The streaming decoder sizes its transfer buffers from bitstream sizes alone
    (mj423_pipeline.cpp chunk_xfer_bytes): a plane of nb bytes sets at most one DC entry per
    block plus one entry per 9 bits, because every AC entry costs RUN(4) + SIZE(4) + at least one
    amplitude bit.  Checked on the tightest streams there are (every coefficient +-1, so every AC
    symbol is exactly 9 bits) and on random dense and sparse ones, I and P."""
    import mj423
    import mpg_synth
    mpg_synth.build()
    rng = np.random.default_rng(9)
    n = 96
    cases = [np.where(rng.random((n, 64)) < 0.5, 1, -1).astype(np.int16)]  # every coefficient +-1
    for density, mag in ((1.0, 2047), (0.6, 15), (0.1, 300), (0.02, 3)):
        b = np.where(rng.random((n, 64)) < density, rng.integers(1, mag + 1, size=(n, 64)), 0)
        cases.append((b * rng.choice([-1, 1], size=(n, 64))).astype(np.int16))
    for blocks in cases:
        for P in (False, True):
            stream = mpg_synth.encode_plane(blocks, P)
            got = mj423.lossless_decode_q(n, stream, True)  # P form onto zeros: the entries themselves
            entries = int(np.count_nonzero(got))
            assert entries <= n + (8 * len(stream)) // 9, (entries, len(stream), P)


_HOST_ONLY_C = r"""
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
typedef struct mj423_mpg mj423_mpg;
int mj423_mpg_open(const char*, mj423_mpg**);
int mj423_mpg_entropy_decode(const mj423_mpg*, uint32_t, uint32_t, int16_t*, int);
int mj423_mpg_entropy_decode_deltas(const mj423_mpg*, uint32_t, uint32_t, int16_t*, uint8_t*, int);
void mj423_mpg_close(mj423_mpg*);
int main(int argc, char** argv) {
    (void)argc;
    mj423_mpg* m = 0;
    if (mj423_mpg_open(argv[1], &m)) return 2;
    int16_t* q = malloc((size_t)320 * 240 * 3 * 2 * 30);
    uint8_t t[30];
    int rc = mj423_mpg_entropy_decode(m, 0, 30, q, 2) | mj423_mpg_entropy_decode_deltas(m, 3, 20, q, t, 2);
    mj423_mpg_close(m);
    printf("rc=%d\n", rc);
    return rc;
}
"""


def test_host_only_mpg_use_makes_no_hip_call(tmp_path):
    """Opening, indexing and entropy-decoding a .mpg on the host (mj423_mpg_open,
    mj423_mpg_entropy_decode[_deltas], mj423_mpg_close) call no HIP API: no device query, no
    page-locking, no runtime initialisation.  Checked from the dynamic linker's lazy bindings
    (LD_DEBUG=bindings): the only libamdhip64 symbols libmj423gpu.so binds are the fat-binary
    registrations every HIP library makes at load.  (The whole-GPU decoder page-locks a copy of
    the file on its first use, mj423_mpg_pinned.)"""
    from conftest import PKG
    src = tmp_path / "host_only.c"
    src.write_text(_HOST_ONLY_C)
    exe = tmp_path / "host_only"
    subprocess.run(["gcc", "-O1", "-o", str(exe), str(src), f"-L{PKG}", "-lmj423gpu", f"-Wl,-rpath,{PKG}"], check=True)
    env = dict(os.environ, LD_DEBUG="bindings", LD_DEBUG_OUTPUT=str(tmp_path / "ld"))
    env.pop("LD_BIND_NOW", None)
    r = subprocess.run([str(exe), os.path.join(GOLDEN, "stream_320x240.mpg")], env=env, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and "rc=0" in r.stdout, r.stdout + r.stderr
    log = "".join(p.read_text() for p in tmp_path.iterdir() if p.name.startswith("ld"))
    bound = set()
    for line in log.splitlines():
        if "binding file" in line and "libmj423gpu.so" in line.split(" to ")[0] and "libamdhip64" in line:
            bound.add(line.split("symbol `")[1].split("'")[0])
    assert bound, "no binding seen: the check itself is not working"
    assert all(s.startswith("__hip") for s in bound), sorted(bound)
