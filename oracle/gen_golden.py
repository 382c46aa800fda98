#!/usr/bin/env python3
"""Generate tests/golden/* from the reference's own C (TEST INFRASTRUCTURE).

Runs ONLY in the build container, where /root/reference exists and
`make -C oracle ref` has compiled the reference sources in place into
oracle/_ref/libmjref.so.  Every expected output below is produced by the
reference's functions (idct, ycbcr_to_rgb, lossless_decode, and the encoder
rgb_to_ycbcr/fdct/quantize_I/quantize_P/lossless_encode for realistic inputs);
inputs come from numpy's PCG64 with the fixed seeds recorded in the manifest.
The committed .npz files are plain arrays (load with allow_pickle=False).

Fixture set (SURVEY §4 "Recommended fixture set"):
  idct_directed.npz   DC sweep, single-AC impulses, saturating and alternating blocks
  idct_realistic.npz  4096 dequantized blocks from the reference encoder pipeline
  idct_wrap.npz       1024 full-range int16 blocks (pins the int32 wrap regime, §0.6)
  csc_sample.npz      4096 (Y,Cb,Cr) triples -> BGRA; exhaustive 2^24 hash in manifest
  stream_640x480.npz  one I-frame + one P-frame at 640x480 4:4:4 (BASELINE config 1):
                      reference bitstreams, absolute quantized planes, every 16th row of the
                      decoded BGRA frames; hashes of the full frames and of the dequantized
                      planes lossless_decode produces
  stream_*.mpg        .mpg files written by the reference's own encoder (mjpeg423_encode,
                      via oracle/_ref/mjref_app) from synthetic BMP frames; the reference's own
                      decoder (mjpeg423_decode) output BMPs are pinned by SHA-256 in the manifest
                      (the first one of each stream is kept as a file for the BMP-writer test);
                      stream_100x60 (sizes not multiples of 8) pins only each BMP's coded region,
                      the w/8 x h/8 whole blocks -- the reference leaves the rest uninitialised
  manifest.json       seeds, shapes and FNV-1a-64 hashes of every expected output
"""
import ctypes
import hashlib
import json
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "tests", "golden")
REF = os.path.join(HERE, "_ref", "libmjref.so")
REF_APP = os.path.join(HERE, "_ref", "mjref_app")
P = ctypes.c_void_p


def fnv1a64(arr) -> str:
    h = 0xCBF29CE484222325
    data = np.ascontiguousarray(arr).view(np.uint8).ravel()
    # vectorised FNV is awkward; chunked pure python is fine at fixture sizes
    for b in data.tobytes():
        h ^= b
        h = (h * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return f"{h:016x}"


def ptr(a):
    return a.ctypes.data_as(P)


def load_ref():
    if not os.path.exists(REF):
        sys.exit(f"{REF} missing: run `make -C oracle ref` first (needs /root/reference)")
    lib = ctypes.CDLL(REF)
    lib.ref_csc_exhaustive_hash.restype = ctypes.c_uint64
    lib.lossless_encode.restype = ctypes.c_uint32
    return lib


def ref_idct(lib, blocks):
    blocks = np.ascontiguousarray(blocks, dtype=np.int16)
    out = np.zeros((len(blocks), 64), np.uint8)
    lib.ref_idct_batch(len(blocks), ptr(blocks), ptr(out))
    return out


def directed_blocks():
    blks = []
    for dc in range(-2048, 2048):  # DC-only sweep
        b = np.zeros(64, np.int16)
        b[0] = dc
        blks.append(b)
    for pos in range(64):  # single-coefficient impulses
        for amp in (1, -1, 7, -7, 64, -64, 1023, -1023):
            b = np.zeros(64, np.int16)
            b[pos] = amp
            blks.append(b)
    for dc in (-32768, -2048, 0, 1016, 2047, 4095, 32767):  # saturating / out-of-range
        b = np.zeros(64, np.int16)
        b[0] = dc
        blks.append(b)
        blks.append(np.full(64, dc, np.int16))
    sign = np.array([1 if ((i >> 3) + (i & 7)) % 2 == 0 else -1 for i in range(64)], np.int16)
    for amp in (1, 16, 255, 1023, 2047, 16383, 32767):  # alternating-sign checkerboards
        blks.append((sign * amp).astype(np.int16))
        blks.append((-sign * amp).astype(np.int16))
    return np.stack(blks)


def synth_rgb(rng, w, h, shift=0):
    """Smooth gradients + texture + noise + hard-edged rectangles -> BGRA uint32."""
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    x = x + shift
    r = 128 + 90 * np.sin(x / 37.0) * np.cos(y / 23.0) + 30 * np.sin((x + y) / 5.0)
    g = 40 + 160 * (x / max(w, 1)) + 20 * np.cos(y / 3.0)
    b = 200 - 150 * (y / max(h, 1)) + 25 * np.sin(x * y / 900.0)
    img = np.stack([b, g, r], axis=-1) + rng.normal(0, 6, size=(h, w, 3))
    for _ in range(12):
        x0, y0 = rng.integers(0, w - 8), rng.integers(0, h - 8)
        ww, hh = rng.integers(4, w // 3), rng.integers(4, h // 3)
        img[y0:y0 + hh, x0 + shift % 7:x0 + ww] = rng.integers(0, 256, size=3)
    img = np.clip(img, 0, 255).astype(np.uint32)
    return (img[..., 0] | (img[..., 1] << 8) | (img[..., 2] << 16)).astype(np.uint32)


def encode_iframe(lib, rgb, w, h):
    nb = (w // 8) * (h // 8)
    planes = [np.zeros((nb, 64), np.int16) for _ in range(6)]
    lib.ref_encode_iframe(w, h, ptr(rgb), *[ptr(p) for p in planes])
    return planes[:3], planes[3:]  # absolute, differential


def encode_pframe(lib, rgb, w, h, prev_abs):
    nb = (w // 8) * (h // 8)
    prev = [p.copy() for p in prev_abs]
    diff = [np.zeros((nb, 64), np.int16) for _ in range(3)]
    lib.ref_encode_pframe(w, h, ptr(rgb), *[ptr(p) for p in prev], *[ptr(d) for d in diff])
    return prev, diff  # new absolute, differential


def lossless_encode(lib, coefs):
    buf = np.zeros(len(coefs) * 64 * 4 + 64, np.uint8)
    n = lib.lossless_encode(len(coefs), ptr(np.ascontiguousarray(coefs)), ptr(buf))
    pad = (n + 3) // 4 * 4  # frames pad each plane to 4 B (encoder/mjpeg423_encoder.c:188-201)
    return buf[:pad + 4].copy(), int(n)


def lossless_decode_ref(lib, n, stream, dcac, quant, P_frame):
    lib.lossless_decode(n, ptr(stream), ptr(dcac), ptr(quant), int(P_frame))


def write_bmp24(path, rgb):
    """24-bit bottom-up BMP of an HxWx3 uint8 RGB image (input for the reference encoder)."""
    h, w, _ = rgb.shape
    rowb = (w * 3 + 3) // 4 * 4
    data = bytearray()
    for y in range(h - 1, -1, -1):
        data += rgb[y][:, ::-1].tobytes() + b"\0" * (rowb - w * 3)
    with open(path, "wb") as f:
        f.write(struct.pack("<2sIHHI", b"BM", 54 + len(data), 0, 0, 54))
        f.write(struct.pack("<IiiHHIIiiII", 40, w, h, 1, 24, 0, len(data), 2835, 2835, 0, 0))
        f.write(data)


def mpg_fixture(name, w, h, n, max_i, seed):
    rng = np.random.default_rng(seed)
    base = synth_rgb(rng, w, h)
    base = np.stack([(base >> 16) & 255, (base >> 8) & 255, base & 255], -1).astype(np.int32)
    with tempfile.TemporaryDirectory() as td:
        for f in range(n):  # a static scene with a moving square and a slow brightness drift: P-frames win
            rgb = base.copy() + (f % 5)
            x0, y0 = (7 * f) % (w - 24), (3 * f) % (h - 24)
            rgb[y0:y0 + 24, x0:x0 + 24] = [250 - 5 * f, 40 + 3 * f, 90]
            write_bmp24(os.path.join(td, f"in{f:04d}.bmp"), np.clip(rgb, 0, 255).astype(np.uint8))
        mpg = os.path.join(OUT, f"{name}.mpg")
        subprocess.run([REF_APP, "encode", str(n), "0", "1", str(max_i), str(w), str(h),
                        os.path.join(td, "in0000.bmp"), mpg], check=True, capture_output=True)
        subprocess.run([REF_APP, "decode", mpg, os.path.join(td, "dec0000.bmp")], check=True, capture_output=True)
        shas, covered = [], []
        for f in range(n):
            with open(os.path.join(td, f"dec{f:04d}.bmp"), "rb") as fh:
                b = fh.read()
            shas.append(hashlib.sha256(b).hexdigest())
            covered.append(covered_sha256(b, w, h))
            if f == 0:
                with open(os.path.join(OUT, f"{name}_dec0000.bmp"), "wb") as out:
                    out.write(b)
    with open(mpg, "rb") as fh:
        hdr = struct.unpack("<5I", fh.read(20))
    fx = {"width": w, "height": h, "frames": n, "max_I_interval": max_i, "seed": seed,
          "header": list(hdr), "mpg_sha256": hashlib.sha256(open(mpg, "rb").read()).hexdigest()}
    if w % 8 or h % 8:
        # the reference decodes only the w/8 x h/8 whole blocks; the rest of each BMP is its
        # uninitialised rgbblock (mjpeg423_decoder.c:55), so only the coded region is pinned
        fx["coded_region"] = [w // 8 * 8, h // 8 * 8]
        fx["decoded_coded_region_sha256"] = covered
    else:
        fx["decoded_bmp_sha256"] = shas
    return fx


def covered_sha256(bmp, w, h):
    """SHA-256 of the coded region (top-left (w & ~7) x (h & ~7) pixels, top-down rows, BGRA
    bytes) of a 32-bpp bottom-up BMP as the reference's libbmp writes it."""
    off = struct.unpack("<I", bmp[10:14])[0]
    px = np.frombuffer(bmp[off:off + 4 * w * h], np.uint8).reshape(h, w, 4)[::-1]
    return hashlib.sha256(np.ascontiguousarray(px[:h // 8 * 8, :w // 8 * 8]).tobytes()).hexdigest()


def main():
    lib = load_ref()
    os.makedirs(OUT, exist_ok=True)
    yq = np.zeros(64, np.int16)
    cq = np.zeros(64, np.int16)
    zz = np.zeros(64, np.int32)
    lib.ref_tables(ptr(yq), ptr(cq), ptr(zz))
    man = {"generator": "oracle/gen_golden.py", "reference_lib": "oracle/_ref/libmjref.so (built by oracle/Makefile ref)",
           "tables": {"yquant": yq.tolist(), "cquant": cq.tolist(), "zigzag": zz.tolist()}, "fixtures": {}}

    # 1. directed IDCT blocks
    d_in = directed_blocks()
    d_out = ref_idct(lib, d_in)
    np.savez_compressed(os.path.join(OUT, "idct_directed.npz"), inp=d_in, out=d_out)
    man["fixtures"]["idct_directed"] = {"n": len(d_in), "out_fnv1a64": fnv1a64(d_out)}

    # 2. realistic blocks: reference encoder -> lossless_decode dequantization -> idct
    rng = np.random.default_rng(0x4D4A3432)
    w, h = 128, 64  # 128 blocks per plane
    pool = []
    for k in range(11):
        rgb = synth_rgb(rng, w, h, shift=k)
        absq, diff = encode_iframe(lib, rgb, w, h)
        for pi, (plane, quant) in enumerate(zip(diff, (yq, cq, cq))):
            stream, _ = lossless_encode(lib, plane)
            dcac = np.zeros_like(plane)
            lossless_decode_ref(lib, len(plane), stream, dcac, quant, 0)
            pool.append(dcac)
    r_in = np.concatenate(pool)[:4096]
    r_out = ref_idct(lib, r_in)
    np.savez_compressed(os.path.join(OUT, "idct_realistic.npz"), inp=r_in, out=r_out)
    man["fixtures"]["idct_realistic"] = {"n": len(r_in), "seed": 0x4D4A3432, "max_abs_coef": int(np.abs(r_in.astype(np.int32)).max()),
                                         "out_fnv1a64": fnv1a64(r_out)}

    # 3. wrap regime: full-range int16
    rng = np.random.default_rng(7)
    wr_in = rng.integers(-32768, 32768, size=(1024, 64), dtype=np.int16)
    wr_out = ref_idct(lib, wr_in)
    np.savez_compressed(os.path.join(OUT, "idct_wrap.npz"), inp=wr_in, out=wr_out)
    man["fixtures"]["idct_wrap"] = {"n": 1024, "seed": 7, "out_fnv1a64": fnv1a64(wr_out)}

    # 4. CSC: 4096 sampled triples (through a 4:4:4 frame of 64 blocks) + exhaustive hash
    rng = np.random.default_rng(11)
    trip = rng.integers(0, 256, size=(4096, 3), dtype=np.uint8)
    trip[:8] = [[0, 0, 0], [255, 255, 255], [0, 255, 255], [255, 0, 0], [0, 0, 255], [255, 255, 0], [128, 128, 128], [16, 128, 128]]
    planes = [np.ascontiguousarray(trip[:, i].reshape(64, 64)) for i in range(3)]  # 64 blocks, 8 rows of 8 blocks
    rgb = np.zeros(64 * 64, np.uint32)
    lib.ref_csc_frame(64, 64, *[ptr(p) for p in planes], ptr(rgb))
    # pixel of block b, element e sits at raster ((b//8)*8 + e//8, (b%8)*8 + e%8)
    bidx, eidx = np.divmod(np.arange(4096), 64)
    ry, rx = (bidx // 8) * 8 + eidx // 8, (bidx % 8) * 8 + eidx % 8
    bgra = rgb.reshape(64, 64)[ry, rx]
    np.savez_compressed(os.path.join(OUT, "csc_sample.npz"), ycbcr=trip, bgra=bgra)
    man["fixtures"]["csc_sample"] = {"n": 4096, "seed": 11, "exhaustive_fnv1a64": f"{lib.ref_csc_exhaustive_hash():016x}",
                                     "exhaustive_enumeration": "idx=(Y<<16)|(Cb<<8)|Cr ascending, 64 per ycbcr_to_rgb call, BGRA bytes hashed"}

    # 5. 640x480 4:4:4 I + P frame through the full reference pipeline
    w, h = 640, 480
    nb = (w // 8) * (h // 8)
    rng = np.random.default_rng(2024)
    rgb0 = synth_rgb(rng, w, h, shift=0)
    rgb1 = synth_rgb(np.random.default_rng(2024), w, h, shift=3)
    abs0, diff0 = encode_iframe(lib, rgb0, w, h)
    abs1, diff1 = encode_pframe(lib, rgb1, w, h, abs0)
    arrays = {}
    man_dcac = {}
    dcac = [np.zeros((nb, 64), np.int16) for _ in range(3)]
    for fi, (absq, diff, ftype) in enumerate(((abs0, diff0, 0), (abs1, diff1, 1))):
        for pi, (name, quant) in enumerate((("Y", yq), ("Cb", cq), ("Cr", cq))):
            stream, nbytes = lossless_encode(lib, diff[pi])
            lossless_decode_ref(lib, nb, stream, dcac[pi], quant, ftype)  # P-frames accumulate into the same buffer
            arrays[f"f{fi}_{name}_stream"] = stream
            arrays[f"f{fi}_{name}_q"] = absq[pi]
            man_dcac[f"f{fi}_{name}"] = fnv1a64(dcac[pi])
        scratch = np.zeros(3 * nb * 64, np.uint8)
        out = np.zeros(w * h, np.uint32)
        lib.ref_decode_frame_444(w, h, *[ptr(d) for d in dcac], ptr(scratch), ptr(out))
        arrays[f"f{fi}_bgra_rows16"] = out.reshape(h, w)[::16].copy()  # every 16th row; full frame pinned by hash
        man["fixtures"][f"stream_640x480_f{fi}"] = {"type": "IP"[ftype], "bgra_fnv1a64": fnv1a64(out),
                                                    "dcac_fnv1a64": {k: man_dcac[f"f{fi}_{k}"] for k in ("Y", "Cb", "Cr")},
                                                    "stream_bytes": {k: int(arrays[f"f{fi}_{k}_stream"].size) for k in ("Y", "Cb", "Cr")}}
    np.savez_compressed(os.path.join(OUT, "stream_640x480.npz"), **arrays)

    # 6. .mpg streams through the reference's own encoder and decoder (CLI around
    #    mjpeg423_encode / mjpeg423_decode, oracle/ref_app.c)
    for name, (w, h, n, max_i, seed) in {"stream_160x96": (160, 96, 12, 4, 31),
                                         "stream_320x240": (320, 240, 30, 24, 32),
                                         # width/height not multiples of 8 (mjpeg423_encoder.c:21-24)
                                         "stream_100x60": (100, 60, 10, 4, 33)}.items():
        man["fixtures"][name] = mpg_fixture(name, w, h, n, max_i, seed)

    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(man, f, indent=1, sort_keys=True)
    for fn in sorted(os.listdir(OUT)):
        print(f"{fn:28s} {os.path.getsize(os.path.join(OUT, fn)):>10d} B")


if __name__ == "__main__":
    main()
