"""ctypes wrapper of tools/libmpgsynth.so (tools/mpg_synth.cpp): seeded synthetic .mpg
streams for benchmarks and tests.  Not the product and not the oracle."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libmpgsynth.so")
_lib = None


def build():
    src = os.path.join(HERE, "mpg_synth.cpp")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", src, "-o", LIB, "-lpthread"])


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(LIB)
        _lib.mpg_synth_write.restype = ctypes.c_longlong
        _lib.mpg_synth_encode_plane.restype = ctypes.c_long
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def generate(w, h, nframes, gop=24, seed=0x4D4A3432):
    """(absolute planes, coded planes, frame types), planes [frame][Y|Cb|Cr blocks * 64] int16."""
    n = (w // 8) * (h // 8) * 64 * 3
    a = np.empty((nframes, n), np.int16)
    s = np.empty((nframes, n), np.int16)
    t = np.empty(nframes, np.uint8)
    if lib().mpg_synth_generate(ctypes.c_uint32(w), ctypes.c_uint32(h), ctypes.c_uint32(nframes),
                                ctypes.c_uint32(gop), ctypes.c_uint64(seed), _p(a), _p(s), _p(t)) != 0:
        raise ValueError("bad geometry")
    return a, s, t


def write_coef(path, w, h, types, coef):
    types = np.ascontiguousarray(types, np.uint8)
    coef = np.ascontiguousarray(coef, np.int16)
    if lib().mpg_synth_write_coef(str(path).encode(), ctypes.c_uint32(w), ctypes.c_uint32(h),
                                  ctypes.c_uint32(len(types)), _p(types), _p(coef)) != 0:
        raise OSError(f"cannot write {path}")


def write(path, w, h, nframes, gop=24, seed=0x4D4A3432, nthreads=0):
    """Seeded stream straight to a file; returns its size in bytes."""
    n = lib().mpg_synth_write(str(path).encode(), ctypes.c_uint32(w), ctypes.c_uint32(h), ctypes.c_uint32(nframes),
                              ctypes.c_uint32(gop), ctypes.c_uint64(seed), ctypes.c_int(nthreads))
    if n < 0:
        raise OSError(f"cannot write {path}")
    return n


def encode_plane(blocks, P):
    b = np.ascontiguousarray(blocks, np.int16)
    cap = b.size * 4 + 64
    out = np.empty(cap, np.uint8)
    n = lib().mpg_synth_encode_plane(ctypes.c_int(b.size // 64), _p(b), ctypes.c_int(1 if P else 0), _p(out),
                                     ctypes.c_size_t(cap))
    return out[:n].tobytes()
