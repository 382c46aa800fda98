"""Python binding of the MI355X MPEG423 hot-path C ABI (include/mj423gpu.h).

Thin ctypes layer over the in-tree ``libmj423gpu.so``; every call lands in the
HIP kernels.  There is deliberately no fallback: if the library or a GPU is
missing, the calls raise ``Mj423Error`` with the library's own message.

Names mirror the reference's call surface (paths under
core0/software/common/libs/mjpeg423/):
  idct / ycbcr_to_rgb            decoder/mjpeg423_decoder.h:15-16
  decode_frame                   the per-frame body decoder/mjpeg423_decoder.c:109-124
  accelerator API                core0/software/idct_ycbcr_to_rgb_accel.h:13-22
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# MJ423_LIB selects an A/B build of the same library (tools/build_variant.sh); measurements only.
LIB_PATH = os.environ.get("MJ423_LIB") or os.path.join(HERE, "libmj423gpu.so")

CHROMA_444, CHROMA_422, CHROMA_420 = 444, 422, 420
INPUT_QUANTIZED, INPUT_DEQUANTIZED = 0, 1
ERRORS = {0: "OK", -1: "EINVAL", -2: "EHIP", -3: "ENOMEM", -4: "ESTATE"}

_P = ctypes.c_void_p


class Mj423Error(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


class Geometry(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint32), ("height", ctypes.c_uint32), ("chroma", ctypes.c_int32),
                ("mcu_w", ctypes.c_uint32), ("mcu_h", ctypes.c_uint32),
                ("coded_w", ctypes.c_uint32), ("coded_h", ctypes.c_uint32),
                ("y_bw", ctypes.c_uint32), ("y_bh", ctypes.c_uint32),
                ("c_bw", ctypes.c_uint32), ("c_bh", ctypes.c_uint32),
                ("y_blocks", ctypes.c_uint32), ("c_blocks", ctypes.c_uint32),
                ("coef_per_frame", ctypes.c_uint64)]


class FramesDesc(ctypes.Structure):
    _fields_ = [("y", _P), ("cb", _P), ("cr", _P), ("plane_frame_stride", ctypes.c_uint64),
                ("out", _P), ("out_frame_stride", ctypes.c_uint64), ("out_pitch", ctypes.c_uint32),
                ("nframes", ctypes.c_uint32), ("width", ctypes.c_uint32), ("height", ctypes.c_uint32),
                ("chroma", ctypes.c_int32), ("input_form", ctypes.c_int32)]


_lib = None


def lib() -> ctypes.CDLL:
    """Load libmj423gpu.so (built by `make -C mjpeg423-video-decoder-software_amd`)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise Mj423Error(-2, f"{LIB_PATH} not built: run __graft_entry__.build() (no CPU fallback exists)")
        # PyTorch wheels bundle their own libamdhip64 (same SONAME as /opt/rocm's).
        # Loading torch first makes libmj423gpu.so bind to that already-loaded
        # runtime, so torch tensors, streams and this library share ONE HIP runtime
        # in the process; loading ours first would leave torch with a second one.
        try:
            import torch  # noqa: F401
        except ImportError:
            pass
        L = ctypes.CDLL(LIB_PATH)
        L.mj423_last_error.restype = ctypes.c_char_p
        L.mj423_frame_bytes.restype = ctypes.c_uint64
        L.mj423_ctx_stream.restype = _P
        L.mj423_ctx_kernel_ms.restype = ctypes.c_double
        L.mj423_ctx_kernel_frames.restype = ctypes.c_uint32
        L.mj423_ctx_destroy.argtypes = [_P]
        _lib = L
    return _lib


def _check(rc: int):
    if rc != 0:
        raise Mj423Error(rc, lib().mj423_last_error().decode(errors="replace"))


def last_error() -> str:
    return lib().mj423_last_error().decode(errors="replace")


def geometry(w: int, h: int, chroma: int) -> Geometry:
    g = Geometry()
    _check(lib().mj423_geometry(ctypes.c_uint32(w), ctypes.c_uint32(h), ctypes.c_int(chroma), ctypes.byref(g)))
    return g


def frame_bytes(w: int, h: int, chroma: int) -> int:
    """Algorithmic HBM bytes per frame (2 B/coefficient read + 4 B/pixel written)."""
    return int(lib().mj423_frame_bytes(ctypes.c_uint32(w), ctypes.c_uint32(h), ctypes.c_int(chroma)))


# The sources the fused batch and stream kernels are compiled from (csrc/).  Their digest ties a
# committed PMC measurement (profiles/pmc_traffic.json, tools/pmc_summary.py) to the kernel it
# measured: bench.py reports that traffic only while the digest still matches.
KERNEL_SOURCES = ("csrc/mj423_kernels.hip", "csrc/mj423_tile.hpp", "csrc/mj423_idct.hpp", "csrc/mj423_kernels.h")
# ... and the fused .mpg kernel's (the whole-file GPU path's pixel kernel, bench.py --mode file)
FUSED_SOURCES = ("csrc/mj423_fused.hip", "csrc/mj423_tile.hpp", "csrc/mj423_idct.hpp", "csrc/mj423_bits.hpp",
                 "csrc/mj423_entropy.h", "csrc/mj423_kernels.h")


def kernel_source_digest(sources=KERNEL_SOURCES):
    """First 16 hex digits of sha256 over `sources` (default KERNEL_SOURCES), or None where the
    sources are absent."""
    import hashlib
    h = hashlib.sha256()
    try:
        for rel in sources:
            with open(os.path.join(HERE, rel), "rb") as f:
                h.update(rel.encode() + b"\0" + f.read())
    except OSError:
        return None
    return h.hexdigest()[:16]


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(_P)


def _need(a: np.ndarray, dtype, n: int, name: str) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=dtype)
    if a.size < n:
        raise Mj423Error(-1, f"{name}: need {n} elements, got {a.size}")
    return a


class Context:
    """One HIP stream + quant tables + staging buffers (mj423_ctx)."""

    def __init__(self, device: int = -1):
        self._h = _P()
        _check(lib().mj423_ctx_create(ctypes.byref(self._h), ctypes.c_int(device)))

    def close(self):
        if self._h:
            lib().mj423_ctx_destroy(self._h)
            self._h = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self):
        return self._h

    def set_stream(self, hip_stream: int | None):
        _check(lib().mj423_ctx_set_stream(self._h, _P(hip_stream or 0)))

    def stream(self) -> int:
        return lib().mj423_ctx_stream(self._h) or 0

    def set_quant(self, yquant=None, cquant=None):
        y = None if yquant is None else _need(yquant, np.int16, 64, "yquant")
        c = None if cquant is None else _need(cquant, np.int16, 64, "cquant")
        _check(lib().mj423_ctx_set_quant(self._h, None if y is None else _ptr(y), None if c is None else _ptr(c)))

    def get_quant(self):
        y = np.zeros(64, np.int16)
        c = np.zeros(64, np.int16)
        _check(lib().mj423_ctx_get_quant(self._h, _ptr(y), _ptr(c)))
        return y, c

    def synchronize(self):
        _check(lib().mj423_ctx_synchronize(self._h))

    def enable_timing(self, on: bool = True):
        _check(lib().mj423_ctx_enable_timing(self._h, ctypes.c_int(1 if on else 0)))

    def kernel_ms(self) -> float:
        return float(lib().mj423_ctx_kernel_ms(self._h))

    def kernel_frames(self) -> int:
        """Frames decoded by the launch kernel_ms() timed."""
        return int(lib().mj423_ctx_kernel_frames(self._h))

    def kernel_totals(self):
        """(device ms, frames, launches) summed over every timed launch since enable_timing()."""
        ms, fr, n = ctypes.c_double(), ctypes.c_uint64(), ctypes.c_uint32()
        _check(lib().mj423_ctx_kernel_totals(self._h, ctypes.byref(ms), ctypes.byref(fr), ctypes.byref(n)))
        return float(ms.value), int(fr.value), int(n.value)

    def stream_reruns(self) -> int:
        """(GOP segment, tile) jobs the exact stream kernel has re-run for this context (the 4:2:2
        optimistic kernel's escapes; waits for the context's stream)."""
        n = ctypes.c_uint64()
        _check(lib().mj423_ctx_stream_reruns(self._h, ctypes.byref(n)))
        return int(n.value)

    # ---- frame calls (host buffers)
    def decode_frame(self, Yq, Cbq, Crq, w: int, h: int, chroma: int, input_form: int = INPUT_QUANTIZED):
        g = geometry(w, h, chroma)
        Y = _need(Yq, np.int16, 64 * g.y_blocks, "Y")
        Cb = _need(Cbq, np.int16, 64 * g.c_blocks, "Cb")
        Cr = _need(Crq, np.int16, 64 * g.c_blocks, "Cr")
        out = np.empty((h, w), np.uint32)
        _check(lib().mj423_decode_frame_ex(self._h, _ptr(Y), _ptr(Cb), _ptr(Cr), _ptr(out), ctypes.c_uint32(w),
                                           ctypes.c_uint32(h), ctypes.c_int(chroma), ctypes.c_int(input_form)))
        return out

    def decode_frames(self, coef, n: int, w: int, h: int, chroma: int, input_form: int = INPUT_QUANTIZED,
                      out=None):
        """decode_frames() over host buffers; `out` (uint32, n*h*w, C-contiguous) is re-used if given."""
        g = geometry(w, h, chroma)
        c = _need(coef, np.int16, n * g.coef_per_frame, "coef")
        if out is None:
            out = np.empty((n, h, w), np.uint32)
        elif out.dtype != np.uint32 or not out.flags["C_CONTIGUOUS"] or out.size < n * h * w:
            raise Mj423Error(-1, "out must be a C-contiguous uint32 array of n*h*w pixels")
        _check(lib().decode_frames(self._h, ctypes.c_uint32(n), _ptr(c), _ptr(out), ctypes.c_uint32(w),
                                   ctypes.c_uint32(h), ctypes.c_int(chroma), ctypes.c_int(input_form)))
        return out

    def idct_blocks(self, dcac, quant=None):
        d = np.ascontiguousarray(dcac, dtype=np.int16).reshape(-1, 64)
        q = None if quant is None else _need(quant, np.int16, 64, "quant")
        out = np.empty((len(d), 64), np.uint8)
        _check(lib().mj423_idct_blocks(self._h, ctypes.c_size_t(len(d)), _ptr(d), None if q is None else _ptr(q),
                                       _ptr(out)))
        return out

    def ycbcr_to_rgb_444(self, Y, Cb, Cr, w: int, h: int):
        n = w * h
        Yb, Cbb, Crb = (_need(a, np.uint8, n, nm) for a, nm in ((Y, "Y"), (Cb, "Cb"), (Cr, "Cr")))
        out = np.empty((h, w), np.uint32)
        _check(lib().mj423_ycbcr_to_rgb_444(self._h, ctypes.c_uint32(w), ctypes.c_uint32(h), _ptr(Yb), _ptr(Cbb),
                                            _ptr(Crb), _ptr(out)))
        return out

    # ---- device-resident calls (raw device pointers, e.g. torch tensor.data_ptr())
    def decode_frames_device(self, y: int, cb: int, cr: int, plane_frame_stride: int, out: int,
                             out_frame_stride: int, out_pitch: int, nframes: int, w: int, h: int, chroma: int,
                             input_form: int = INPUT_QUANTIZED):
        d = FramesDesc(y, cb, cr, plane_frame_stride, out, out_frame_stride, out_pitch, nframes, w, h, chroma,
                       input_form)
        _check(lib().mj423_decode_frames_device(self._h, ctypes.byref(d)))

    def decode_batch_device(self, coef_ptr: int, out_ptr: int, nframes: int, w: int, h: int, chroma: int,
                            input_form: int = INPUT_QUANTIZED):
        """[frame][Y|Cb|Cr] coefficients -> [frame][h][w] BGRA, both device-resident."""
        g = geometry(w, h, chroma)
        y = coef_ptr
        cb = y + 128 * g.y_blocks
        cr = cb + 128 * g.c_blocks
        self.decode_frames_device(y, cb, cr, g.coef_per_frame, out_ptr, w * h, w, nframes, w, h, chroma, input_form)

    def decode_stream_device(self, coef_ptr: int, out_ptr: int, nframes: int, w: int, h: int, chroma: int,
                             frame_types, state_in: int = 0, state_out: int = 0):
        """[frame][Y|Cb|Cr] coefficients (I: absolute, P: deltas) -> BGRA, P-frames accumulated on chip."""
        g = geometry(w, h, chroma)
        y = coef_ptr
        cb = y + 128 * g.y_blocks
        cr = cb + 128 * g.c_blocks
        d = FramesDesc(y, cb, cr, g.coef_per_frame, out_ptr, w * h, w, nframes, w, h, chroma, INPUT_QUANTIZED)
        t = np.ascontiguousarray(frame_types, np.uint8)
        _check(lib().mj423_decode_stream_device(self._h, ctypes.byref(d), _ptr(t), _P(state_in or 0),
                                                _P(state_out or 0)))

    def synth_frames_device(self, coef_ptr: int, w: int, h: int, chroma: int, nframes: int, frame0: int = 0,
                            seed: int = 0x4D4A3432):
        _check(lib().mj423_synth_frames_device(self._h, _P(coef_ptr), ctypes.c_uint32(w), ctypes.c_uint32(h),
                                               ctypes.c_int(chroma), ctypes.c_uint32(nframes),
                                               ctypes.c_uint64(frame0), ctypes.c_uint64(seed)))


# ---- host front end, container and BMP sink (include/mj423io.h)
class MpgHeader(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("num_frames", "width", "height", "num_iframes", "payload_size")]


class MpgFrame(ctypes.Structure):
    _fields_ = [("index", ctypes.c_uint32), ("frame_type", ctypes.c_uint32), ("frame_size", ctypes.c_uint32),
                ("position", ctypes.c_uint64), ("y", _P), ("cb", _P), ("cr", _P),
                ("y_size", ctypes.c_uint32), ("cb_size", ctypes.c_uint32), ("cr_size", ctypes.c_uint32)]


def lossless_decode(num_blocks: int, bitstream: bytes, dcac: np.ndarray, quant, P: bool) -> None:
    """The reference's dequantizing front end (decoder/lossless_decode.c:60), in place on dcac."""
    if dcac.dtype != np.int16 or not dcac.flags["C_CONTIGUOUS"] or dcac.size < 64 * num_blocks:
        raise Mj423Error(-1, "dcac must be a C-contiguous int16 array of num_blocks*64")
    bs = np.frombuffer(bytes(bitstream) + b"\0" * 8, np.uint8)
    q = _need(quant, np.int16, 64, "quant")
    lib().lossless_decode(ctypes.c_int(num_blocks), _ptr(bs), _ptr(dcac), _ptr(q), ctypes.c_int(1 if P else 0))


def lossless_decode_q(num_blocks: int, bitstream: bytes, P: bool, prev=None) -> np.ndarray:
    """Quantized-domain front end (absolute quantized coefficients)."""
    out = np.zeros((num_blocks, 64), np.int16) if prev is None else np.array(prev, np.int16, copy=True)
    bs = np.frombuffer(bytes(bitstream), np.uint8)
    L = lib()
    L.mj423_lossless_decode_q.restype = ctypes.c_size_t
    used = L.mj423_lossless_decode_q(ctypes.c_int(num_blocks), _ptr(bs) if bs.size else None,
                                     ctypes.c_size_t(bs.size), _ptr(out), ctypes.c_int(1 if P else 0))
    if used == ctypes.c_size_t(-1).value:
        raise Mj423Error(-1, "bitstream ended before all blocks were decoded")
    return out


class Mpg:
    """An .mpg stream (mj423_mpg_*)."""

    def __init__(self, path_or_bytes):
        self._h = _P()
        if isinstance(path_or_bytes, (bytes, bytearray)):
            buf = np.frombuffer(bytes(path_or_bytes), np.uint8)
            _check(lib().mj423_mpg_open_memory(_ptr(buf), ctypes.c_size_t(buf.size), ctypes.byref(self._h)))
        else:
            _check(lib().mj423_mpg_open(str(path_or_bytes).encode(), ctypes.byref(self._h)))
        self.header = MpgHeader()
        _check(lib().mj423_mpg_header(self._h, ctypes.byref(self.header)))

    def close(self):
        if self._h:
            lib().mj423_mpg_close(self._h)
            self._h = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def frame(self, i: int) -> MpgFrame:
        f = MpgFrame()
        _check(lib().mj423_mpg_frame(self._h, ctypes.c_uint32(i), ctypes.byref(f)))
        return f

    def trailer(self):
        n = lib().mj423_mpg_trailer(self._h, None, None, ctypes.c_uint32(0))
        idx = np.zeros(max(n, 1), np.uint32)
        pos = np.zeros(max(n, 1), np.uint32)
        lib().mj423_mpg_trailer(self._h, _ptr(idx), _ptr(pos), ctypes.c_uint32(n))
        return idx[:n], pos[:n]

    def gop_start(self, i: int) -> int:
        g = ctypes.c_uint32()
        _check(lib().mj423_mpg_gop_start(self._h, ctypes.c_uint32(i), ctypes.byref(g)))
        return g.value

    def geometry(self) -> Geometry:
        """mj423_mpg_geometry: the planes of the w/8 x h/8 whole blocks the stream codes."""
        g = Geometry()
        _check(lib().mj423_mpg_geometry(self._h, ctypes.byref(g)))
        return g

    def entropy_decode(self, first: int, count: int, nthreads: int = 0) -> np.ndarray:
        g = self.geometry()
        out = np.empty((count, g.coef_per_frame), np.int16)
        _check(lib().mj423_mpg_entropy_decode(self._h, ctypes.c_uint32(first), ctypes.c_uint32(count), _ptr(out),
                                              ctypes.c_int(nthreads)))
        return out

    def entropy_decode_deltas(self, first: int, count: int, nthreads: int = 0):
        g = self.geometry()
        out = np.empty((count, g.coef_per_frame), np.int16)
        types = np.empty(count, np.uint8)
        _check(lib().mj423_mpg_entropy_decode_deltas(self._h, ctypes.c_uint32(first), ctypes.c_uint32(count),
                                                     _ptr(out), _ptr(types), ctypes.c_int(nthreads)))
        return out, types

    def decode_gpu(self, ctx: "Context", first: int, count: int, out_ptr: int, out_frame_stride: int = 0,
                   window_frames: int = 0) -> None:
        """mj423_mpg_decode_gpu: entropy decode on GPU lanes + stream decode, frames to device memory."""
        stride = out_frame_stride or self.header.width * self.header.height
        _check(lib().mj423_mpg_decode_gpu(ctx.handle, self._h, ctypes.c_uint32(first), ctypes.c_uint32(count),
                                          _P(out_ptr), ctypes.c_uint64(stride), ctypes.c_uint32(window_frames)))

    def decode(self, ctx: "Context", first: int, count: int, nthreads: int = 0) -> np.ndarray:
        w, h = self.header.width, self.header.height
        out = np.empty((count, h, w), np.uint32)
        _check(lib().mj423_decode_mpg(ctx.handle, self._h, ctypes.c_uint32(first), ctypes.c_uint32(count),
                                      _ptr(out), ctypes.c_int(nthreads)))
        return out


class PipelineStats(ctypes.Structure):
    _fields_ = [("frames", ctypes.c_uint64), ("chunks", ctypes.c_uint64), ("wall_s", ctypes.c_double),
                ("frontend_busy_s", ctypes.c_double), ("sink_busy_s", ctypes.c_double),
                ("gpu_span_ms", ctypes.c_double)]


FRAME_SINK = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint32,
                              ctypes.c_uint32)


DEVICE_SINK = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                               ctypes.c_size_t, ctypes.c_void_p)


class DeviceFrames:
    """A chunk of decoded BGRA frames in HBM, exposed through __cuda_array_interface__
    (torch.as_tensor(frames, device="cuda") gives a zero-copy uint32 [count, h, w] view).
    Valid only during the sink call and in order on `stream` (a hipStream_t handle)."""

    def __init__(self, ptr, count, h, w, stride_px, stream):
        self.ptr, self.count, self.h, self.w, self.stream = ptr, count, h, w, stream
        self.__cuda_array_interface__ = {
            "shape": (count, h, w), "typestr": "<u4", "data": (ptr, False), "version": 3,
            "strides": (stride_px * 4, w * 4, 4), "stream": None}


def _device_sink_adapter(sink, err, h, w):
    def _cb(_user, first, count, ptr, stride, stream):
        try:
            return 1 if sink(int(first), DeviceFrames(ptr, int(count), h, w, int(stride), stream)) else 0
        except BaseException as e:  # noqa: BLE001 -- re-raised in the caller's thread
            err.append(e)
            return 1
    return DEVICE_SINK(_cb)


def _sink_adapter(sink, err):
    def _cb(_user, fi, ptr, ww, hh):
        try:
            view = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint32)), shape=(hh, ww))
            return 1 if sink(int(fi), view) else 0
        except BaseException as e:  # noqa: BLE001 -- re-raised in the caller's thread
            err.append(e)
            return 1
    return FRAME_SINK(_cb)


class Pipeline:
    """Reusable streaming decoder (mj423_pipeline_*) for w x h 4:4:4 streams."""

    def __init__(self, ctx: "Context", w: int, h: int, chunk_frames: int = 0, nthreads: int = 0):
        self._h = _P()
        self.ctx = ctx  # keeps the context alive
        _check(lib().mj423_pipeline_create(ctypes.byref(self._h), ctx.handle, ctypes.c_uint32(w), ctypes.c_uint32(h),
                                           ctypes.c_uint32(chunk_frames), ctypes.c_int(nthreads)))

    def decode(self, mpg: Mpg, first: int, count: int, sink) -> PipelineStats:
        err = []
        cb = _sink_adapter(sink, err)
        st = PipelineStats()
        rc = lib().mj423_pipeline_decode(self._h, mpg._h, ctypes.c_uint32(first), ctypes.c_uint32(count), cb, None,
                                         ctypes.byref(st))
        if err:
            raise err[0]
        _check(rc)
        return st

    def decode_device(self, mpg: Mpg, first: int, count: int, sink) -> PipelineStats:
        """Decode to HBM: sink(first_frame, DeviceFrames) per chunk, frames ordered on its stream."""
        err = []
        cb = _device_sink_adapter(sink, err, mpg.header.height, mpg.header.width)
        st = PipelineStats()
        rc = lib().mj423_pipeline_decode_device(self._h, mpg._h, ctypes.c_uint32(first), ctypes.c_uint32(count),
                                                cb, None, ctypes.byref(st))
        if err:
            raise err[0]
        _check(rc)
        return st

    def close(self):
        if self._h:
            lib().mj423_pipeline_destroy(self._h)
            self._h = _P()

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def decode_mpg_pipelined(ctx: "Context", mpg: Mpg, first: int, count: int, sink, chunk_frames: int = 0,
                         nthreads: int = 0) -> PipelineStats:
    """mj423_decode_mpg_pipelined: sink(frame_index, bgra_view[h, w] uint32) per frame, in order,
    on a library thread (the view is only valid during the call; a truthy return stops)."""
    err = []

    cb = _sink_adapter(sink, err)
    st = PipelineStats()
    rc = lib().mj423_decode_mpg_pipelined(ctx.handle, mpg._h, ctypes.c_uint32(first), ctypes.c_uint32(count),
                                          ctypes.c_uint32(chunk_frames), ctypes.c_int(nthreads), cb, None,
                                          ctypes.byref(st))
    if err:
        raise err[0]
    _check(rc)
    return st


def write_bmp(path: str, rgb: np.ndarray) -> None:
    """32-bpp BMP byte-identical to the reference's encode_bmp (libbmp/encode_bmp.c:7)."""
    a = np.ascontiguousarray(rgb, np.uint32)
    h, w = a.shape
    _check(lib().mj423_write_bmp(str(path).encode(), _ptr(a), ctypes.c_uint32(w), ctypes.c_uint32(h)))


def decode_file(path_in: str, base_out: str) -> None:
    """mjpeg423_decode(filename_in, filenamebase_out) (decoder/mjpeg423_decoder.c:20)."""
    _check(lib().mj423_decode_file(str(path_in).encode(), str(base_out).encode()))


# ---- reference per-block symbols (process-default context)
def idct(dcac: np.ndarray) -> np.ndarray:
    """void idct(dct_block_t DCAC, color_block_t block) (decoder/idct.c:22)."""
    d = _need(dcac, np.int16, 64, "DCAC")
    out = np.zeros(64, np.uint8)
    lib().idct(_ptr(d), _ptr(out))
    _check(lib().mj423_dropin_flush())  # the result is read on return: flush the deferred queue
    return out.reshape(8, 8)


def ycbcr_to_rgb(h: int, w: int, w_size: int, Y, Cb, Cr, rgb: np.ndarray) -> None:
    """void ycbcr_to_rgb(h, w, w_size, Y, Cb, Cr, rgbblock) (decoder/ycbcr_to_rgb.c:26); writes into rgb."""
    if rgb.dtype != np.uint32 or not rgb.flags["C_CONTIGUOUS"]:
        raise Mj423Error(-1, "rgb must be a C-contiguous uint32 array")
    Yb, Cbb, Crb = (_need(a, np.uint8, 64, nm) for a, nm in ((Y, "Y"), (Cb, "Cb"), (Cr, "Cr")))
    lib().ycbcr_to_rgb(ctypes.c_int(h), ctypes.c_int(w), ctypes.c_uint32(w_size), _ptr(Yb), _ptr(Cbb), _ptr(Crb),
                       _ptr(rgb))
    _check(lib().mj423_dropin_flush())


# ---- reference accelerator API (c0/idct_ycbcr_to_rgb_accel.h:13-22)
class Accelerator:
    """Process-wide async accelerator; method names are the reference's functions."""

    def __init__(self, w: int = 640, h: int = 480, chroma: int = CHROMA_444):
        _check(lib().mj423_accel_configure(ctypes.c_uint32(w), ctypes.c_uint32(h), ctypes.c_int(chroma)))
        if lib().init_idct_ycbcr_to_rgb_accel() != 1:
            raise Mj423Error(-2, "init_idct_ycbcr_to_rgb_accel failed: " + last_error())
        self._keep = []  # host buffers must outlive the async copies

    def idct_accel_calculate_buffer_y(self, buf: np.ndarray):
        self._keep.append(buf)
        lib().idct_accel_calculate_buffer_y(_ptr(buf), ctypes.c_uint32(buf.nbytes))

    def idct_accel_calculate_buffer_cb(self, buf: np.ndarray):
        self._keep.append(buf)
        lib().idct_accel_calculate_buffer_cb(_ptr(buf), ctypes.c_uint32(buf.nbytes))

    def idct_accel_calculate_buffer_cr(self, buf: np.ndarray):
        self._keep.append(buf)
        lib().idct_accel_calculate_buffer_cr(_ptr(buf), ctypes.c_uint32(buf.nbytes))

    def ycbcr_to_rgb_accel_get_results(self, out: np.ndarray):
        self._keep.append(out)
        lib().ycbcr_to_rgb_accel_get_results(_ptr(out), ctypes.c_uint32(out.nbytes))

    def wait_for_idct_y_finsh(self):
        lib().wait_for_idct_y_finsh()

    def wait_for_ycbcr_to_rgb_finsh(self):
        lib().wait_for_ycbcr_to_rgb_finsh()
        self._keep.clear()

    def ycbcr_to_rgb_accel_calculate_buffer(self, Y, Cr, Cb, out: np.ndarray, hCb_size: int, wCb_size: int,
                                            w_size: int):
        lib().ycbcr_to_rgb_accel_calculate_buffer(_ptr(Y), _ptr(Cr), _ptr(Cb), _ptr(out), ctypes.c_int(hCb_size),
                                                  ctypes.c_int(wCb_size), ctypes.c_int(w_size))

    @staticmethod
    def status() -> int:
        """mj423_accel_status(): first MJ423_E* code since the last call (read-and-clear)."""
        return int(lib().mj423_accel_status())

    @staticmethod
    def shutdown():
        lib().mj423_accel_shutdown()


# ------------------------------------------------------------------ multi-GPU group
MULTI_NO_COMM = 1


def frame_range(rank: int, world: int, total: int) -> tuple[int, int]:
    """mj423_frame_range: contiguous [first, first+count) of `total` frames for `rank`."""
    f, c = ctypes.c_uint64(), ctypes.c_uint64()
    _check(lib().mj423_frame_range(ctypes.c_uint32(rank), ctypes.c_uint32(world), ctypes.c_uint64(total),
                                   ctypes.byref(f), ctypes.byref(c)))
    return int(f.value), int(c.value)


class _BorrowedContext(Context):
    """A Context view of a context some other object owns (a Multi group's rank)."""

    def __init__(self, h, owner):
        self._hb = h
        self._owner = owner  # keeps the group object alive while the view is

    @property
    def _h(self):
        # Multi.close() (or its with-block's end) destroys the rank contexts: a view used after
        # that must fail loudly instead of handing a freed mj423_ctx* to the library.
        if not self._owner._h:
            raise Mj423Error(-4, "the Multi group that owned this context has been closed")
        return self._hb

    def close(self):
        self._hb = _P()  # never destroys: the owner does


class Multi:
    """One process driving N GPUs (mj423_multi, include/mj423gpu.h section 5): a context per
    device, an RCCL communicator per device (ncclCommInitAll), frame-range sharding.
    flags=MULTI_NO_COMM builds it without RCCL (devices may repeat: a sharding rehearsal)."""

    def __init__(self, ndev: int = 0, devices=None, flags: int = 0):
        L = lib()
        L.mj423_multi_ctx.restype = _P
        L.mj423_multi_destroy.argtypes = [_P]
        self._h = _P()
        arr = None
        if devices is not None:
            devices = list(devices)
            ndev = len(devices)
            arr = (ctypes.c_int * ndev)(*devices)
        _check(L.mj423_multi_create(ctypes.byref(self._h), ctypes.c_int(ndev), arr, ctypes.c_int(flags)))

    def close(self):
        if self._h:
            lib().mj423_multi_destroy(self._h)
            self._h = _P()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def size(self) -> int:
        return int(lib().mj423_multi_size(self._h))

    def comm_ranks(self) -> int:
        return int(lib().mj423_multi_comm_ranks(self._h))

    def ctx(self, rank: int) -> "Context":
        """A non-owning Context view of the rank's context."""
        h = lib().mj423_multi_ctx(self._h, ctypes.c_int(rank))
        if not h:
            raise Mj423Error(-1, f"no rank {rank}")
        return _BorrowedContext(_P(h), self)

    def _ctx_handle(self, rank: int):
        return _P(lib().mj423_multi_ctx(self._h, ctypes.c_int(rank)))

    def get_quant(self, rank: int):
        yq, cq = np.empty(64, np.int16), np.empty(64, np.int16)
        _check(lib().mj423_ctx_get_quant(self._ctx_handle(rank), _ptr(yq), _ptr(cq)))
        return yq, cq

    def set_quant(self, yquant=None, cquant=None):
        """Rank 0 takes the tables; ncclBroadcast hands them to every rank."""
        yq = None if yquant is None else _need(yquant, np.int16, 64, "yquant")
        cq = None if cquant is None else _need(cquant, np.int16, 64, "cquant")
        _check(lib().mj423_multi_set_quant(self._h, None if yq is None else _ptr(yq), None if cq is None else _ptr(cq)))

    def decode_frames(self, coef, n: int, w: int, h: int, chroma: int, input_form: int = INPUT_QUANTIZED):
        g = geometry(w, h, chroma)
        c = _need(coef, np.int16, n * g.coef_per_frame, "coef")
        out = np.empty((n, h, w), np.uint32)
        _check(lib().mj423_multi_decode_frames(self._h, ctypes.c_uint64(n), _ptr(c), _ptr(out), ctypes.c_uint32(w),
                                               ctypes.c_uint32(h), ctypes.c_int(chroma), ctypes.c_int(input_form)))
        return out

    def _descs(self, coef_ptrs, out_ptrs, nframes, w, h, chroma, input_form=INPUT_QUANTIZED):
        g = geometry(w, h, chroma)
        n = self.size
        D = (FramesDesc * n)()
        for r in range(n):
            y = int(coef_ptrs[r])
            D[r] = FramesDesc(y, y + 128 * g.y_blocks, y + 128 * (g.y_blocks + g.c_blocks), g.coef_per_frame,
                              int(out_ptrs[r]), w * h, w, int(nframes[r]), w, h, chroma, input_form)
        return D

    def decode_frames_device(self, coef_ptrs, out_ptrs, nframes, w: int, h: int, chroma: int):
        _check(lib().mj423_multi_decode_frames_device(self._h, self._descs(coef_ptrs, out_ptrs, nframes, w, h, chroma)))

    def synth_frames_device(self, coef_ptrs, frame0, nframes, w: int, h: int, chroma: int, seed: int = 0x4D4A3432):
        n = self.size
        P = (_P * n)(*[int(p) for p in coef_ptrs])
        F = (ctypes.c_uint64 * n)(*[int(x) for x in frame0])
        N = (ctypes.c_uint32 * n)(*[int(x) for x in nframes])
        _check(lib().mj423_multi_synth_frames_device(self._h, P, F, N, ctypes.c_uint32(w), ctypes.c_uint32(h),
                                                     ctypes.c_int(chroma), ctypes.c_uint64(seed)))

    def synchronize(self):
        _check(lib().mj423_multi_synchronize(self._h))

    def time_decode(self, coef_ptrs, out_ptrs, nframes, w: int, h: int, chroma: int, steps: int):
        """Start-aligned timed run; returns (max_ms, per_rank_ms, wall_ms) for all steps."""
        n = self.size
        mx, wall = ctypes.c_double(), ctypes.c_double()
        per = (ctypes.c_double * n)()
        _check(lib().mj423_multi_time_decode(self._h, self._descs(coef_ptrs, out_ptrs, nframes, w, h, chroma),
                                             ctypes.c_uint32(steps), ctypes.byref(mx), per, ctypes.byref(wall)))
        return mx.value, list(per), wall.value

    def decode_mpg_gpu(self, mpg: "Mpg", first: int, count: int, out_ptrs, out_frame_stride: int = 0):
        """GOP-aligned ranges over the ranks, each decoded on its device; returns [(first, count)]."""
        n = self.size
        hdr = mpg.header
        stride = out_frame_stride or hdr.width * hdr.height
        P = (_P * n)(*[int(p) if p else None for p in out_ptrs])
        rf, rc = (ctypes.c_uint32 * n)(), (ctypes.c_uint32 * n)()
        _check(lib().mj423_multi_decode_mpg_gpu(self._h, mpg._h, ctypes.c_uint32(first), ctypes.c_uint32(count), P,
                                                ctypes.c_uint64(stride), rf, rc))
        return [(int(rf[r]), int(rc[r])) for r in range(n)]


def mpg_gop_ranges(mpg: "Mpg", first: int, count: int, world: int):
    rf, rc = (ctypes.c_uint32 * world)(), (ctypes.c_uint32 * world)()
    _check(lib().mj423_mpg_gop_ranges(mpg._h, ctypes.c_uint32(first), ctypes.c_uint32(count), ctypes.c_uint32(world),
                                      rf, rc))
    return [(int(rf[r]), int(rc[r])) for r in range(world)]
