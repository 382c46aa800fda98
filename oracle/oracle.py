"""ctypes binding of the CPU oracle (oracle/build/liboracle.so) -- TEST INFRASTRUCTURE.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
It is the checker, never the thing shipped or measured as the product.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
REF_PATH = os.path.join(HERE, "_ref", "libmjref.so")
_P = ctypes.c_void_p
_lib = None


class OrcGeom(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("width", "height")] + [("chroma", ctypes.c_int)] + \
               [(n, ctypes.c_uint32) for n in ("mcu_w", "mcu_h", "coded_w", "coded_h", "y_bw", "y_bh", "c_bw",
                                                "c_bh", "y_blocks", "c_blocks")]


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = ctypes.CDLL(LIB_PATH)
        L.orc_csc_exhaustive_hash.restype = ctypes.c_uint64
        L.orc_fnv1a64.restype = ctypes.c_uint64
        L.orc_fnv1a64.argtypes = [ctypes.c_uint64, _P, ctypes.c_size_t]
        L.orc_ycbcr_pixel.restype = ctypes.c_uint32
        L.orc_lossless_decode_ref.restype = ctypes.c_size_t
        L.orc_lossless_decode_q.restype = ctypes.c_size_t
        _lib = L
    return _lib


def ref_lib():
    """The reference's own C compiled in place (oracle/_ref), or None if not built."""
    return ctypes.CDLL(REF_PATH) if os.path.exists(REF_PATH) else None


def _ptr(a):
    return a.ctypes.data_as(_P)


YQUANT = np.array([16, 11, 10, 16, 24, 40, 51, 61, 12, 12, 14, 19, 26, 58, 60, 55, 14, 13, 16, 24, 40, 57, 69, 56,
                   14, 17, 22, 29, 51, 87, 80, 62, 18, 22, 37, 56, 68, 109, 103, 77, 24, 35, 55, 64, 81, 104, 113,
                   92, 49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99], np.int16)
CQUANT = np.array([17, 18, 24, 47] + [99] * 4 + [18, 21, 26, 66] + [99] * 4 + [24, 26, 56] + [99] * 5 +
                  [47, 66] + [99] * 6 + [99] * 32, np.int16)


def geometry(w, h, chroma) -> OrcGeom:
    g = OrcGeom()
    if lib().orc_geometry(ctypes.c_uint32(w), ctypes.c_uint32(h), ctypes.c_int(chroma), ctypes.byref(g)):
        raise ValueError("bad geometry")
    return g


def idct_blocks(blocks) -> np.ndarray:
    b = np.ascontiguousarray(blocks, np.int16).reshape(-1, 64)
    out = np.empty((len(b), 64), np.uint8)
    lib().orc_idct_blocks(ctypes.c_size_t(len(b)), _ptr(b), _ptr(out))
    return out


def dequant(Q, q) -> np.ndarray:
    Qa = np.ascontiguousarray(Q, np.int16).reshape(-1, 64)
    qa = np.ascontiguousarray(q, np.int16)
    out = np.empty_like(Qa)
    lib().orc_dequant_blocks(ctypes.c_size_t(len(Qa)), _ptr(Qa), _ptr(qa), _ptr(out))
    return out


def ycbcr_pixels(y, cb, cr) -> np.ndarray:
    """Vectorised over arrays via per-pixel oracle calls (small inputs only)."""
    f = lib().orc_ycbcr_pixel
    return np.array([f(int(a), int(b), int(c)) for a, b, c in zip(np.ravel(y), np.ravel(cb), np.ravel(cr))],
                    np.uint32)


def decode_frame(Yq, Cbq, Crq, w, h, chroma, yquant=None, cquant=None, dequantized=False) -> np.ndarray:
    out = np.empty((h, w), np.uint32)
    Y, Cb, Cr = (np.ascontiguousarray(a, np.int16) for a in (Yq, Cbq, Crq))
    yq = None if yquant is None else np.ascontiguousarray(yquant, np.int16)
    cq = None if cquant is None else np.ascontiguousarray(cquant, np.int16)
    rc = lib().orc_decode_frame(ctypes.c_uint32(w), ctypes.c_uint32(h), ctypes.c_int(chroma), _ptr(Y), _ptr(Cb),
                                _ptr(Cr), None if yq is None else _ptr(yq), None if cq is None else _ptr(cq),
                                ctypes.c_int(1 if dequantized else 0), _ptr(out), ctypes.c_uint32(w))
    if rc:
        raise ValueError("orc_decode_frame failed")
    return out


def decode_frames_mt(coef, n, w, h, chroma, nthreads=1, dequantized=False) -> np.ndarray:
    out = np.empty((n, h, w), np.uint32)
    c = np.ascontiguousarray(coef, np.int16)
    rc = lib().orc_decode_frames_mt(ctypes.c_uint32(w), ctypes.c_uint32(h), ctypes.c_int(chroma), _ptr(c),
                                    ctypes.c_uint32(n), None, None, ctypes.c_int(1 if dequantized else 0),
                                    _ptr(out), ctypes.c_int(nthreads))
    if rc:
        raise ValueError("orc_decode_frames_mt failed")
    return out


def fnv1a64(a) -> str:
    b = np.ascontiguousarray(a)
    return f"{lib().orc_fnv1a64(0xCBF29CE484222325, _ptr(b), b.nbytes):016x}"


def csc_exhaustive_hash() -> str:
    return f"{lib().orc_csc_exhaustive_hash():016x}"


def lossless_decode_ref(num_blocks, stream, quant, P, prev=None) -> np.ndarray:
    out = np.zeros((num_blocks, 64), np.int16) if prev is None else np.array(prev, np.int16, copy=True)
    s = np.ascontiguousarray(stream, np.uint8)
    q = np.ascontiguousarray(quant, np.int16)
    lib().orc_lossless_decode_ref(ctypes.c_int(num_blocks), _ptr(s), _ptr(out), _ptr(q), ctypes.c_int(int(P)))
    return out


def lossless_decode_q(num_blocks, stream, P, prev=None) -> np.ndarray:
    out = np.zeros((num_blocks, 64), np.int16) if prev is None else np.array(prev, np.int16, copy=True)
    s = np.ascontiguousarray(stream, np.uint8)
    lib().orc_lossless_decode_q(ctypes.c_int(num_blocks), _ptr(s), _ptr(out), ctypes.c_int(int(P)))
    return out


def random_quantized_planes(rng, w, h, chroma, full_range=False, nframes=1):
    """Seeded [frame][Y|Cb|Cr] quantized coefficients shaped like SURVEY §8(d)'s stream."""
    g = geometry(w, h, chroma)
    nb = g.y_blocks + 2 * g.c_blocks
    if full_range:
        return rng.integers(-32768, 32768, size=(nframes, nb, 64), dtype=np.int16)
    coef = np.zeros((nframes, nb, 64), np.int16)
    zz = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20,
                   13, 6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52,
                   45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63])
    qtab = np.concatenate([np.tile(YQUANT, (g.y_blocks, 1)), np.tile(CQUANT, (2 * g.c_blocks, 1))])
    coef[:, :, 0] = rng.integers(0, 2040 // qtab[:, 0] + 1, size=(nframes, nb))
    k = np.arange(1, 64)
    p = 0.6 * np.exp(-k / 8.0)
    nz = rng.random((nframes, nb, 63)) < p
    mag = 1 + rng.geometric(0.35, size=(nframes, nb, 63)) - 1
    sign = np.where(rng.random((nframes, nb, 63)) < 0.5, -1, 1)
    lim = np.maximum(1023 // qtab[:, zz[1:]], 1)
    vals = np.where(nz, sign * np.minimum(mag, lim), 0)
    coef[:, :, zz[1:]] = vals
    return coef
