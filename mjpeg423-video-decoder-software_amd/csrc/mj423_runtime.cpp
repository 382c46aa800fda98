// mj423_runtime.cpp -- host side of the C ABI declared in include/mj423gpu.h.
//
// Contexts own a HIP stream (or borrow the caller's), the packed quantization
// tables and growable device staging buffers for the host-pointer entry points.
// Everything that computes runs in the HIP kernels of mj423_kernels.hip; there
// is no CPU fallback: without a usable GPU every entry point fails with
// MJ423_EHIP and says why in mj423_last_error().
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <chrono>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mj423gpu.h"
#include "mj423_internal.h"
#include "mj423_kernels.h"

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}
int hipfail(hipError_t e, const char* what) {
    return fail(MJ423_EHIP, std::string(what) + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")");
}
#define HIP_TRY(expr)                                   \
    do {                                                \
        hipError_t e_ = (expr);                         \
        if (e_ != hipSuccess) return hipfail(e_, #expr); \
    } while (0)

// mj/common/tables.c:13-32 (JPEG Annex K.1 / K.2), natural order.
const int16_t kYquant[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                             14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                             18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                             49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
const int16_t kCquant[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                             24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                             99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                             99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
// mj/common/tables.c:35-42: zig-zag position -> natural index
const int32_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

void pack_table(const int16_t q[64], uint32_t out[32]) {
    for (int i = 0; i < 32; i++) out[i] = (uint32_t)(uint16_t)q[2 * i] | ((uint32_t)(uint16_t)q[2 * i + 1] << 16);
}

// Device buffer that only grows.
struct DevBuf {
    void* p = nullptr;
    size_t cap = 0;
    int ensure(size_t bytes) {
        if (bytes <= cap) return 0;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        hipError_t e = hipMalloc(&p, bytes);
        if (e != hipSuccess) {
            p = nullptr;
            return hipfail(e, "hipMalloc");
        }
        cap = bytes;
        return 0;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
};

}  // namespace

struct mj423_ctx {
    int device = 0;
    hipStream_t own = nullptr;
    hipStream_t stream = nullptr;
    int16_t yq[64], cq[64];
    uint32_t qt[2][32];      // packed: [0] luma, [1] chroma
    uint32_t* d_qt = nullptr;  // packed tables on the device (stage kernels)
    DevBuf in, out, scratch;
    // Stream decode, optimistic kernel: one mark per (segment, tile) job, all zero between launches
    // (the exact re-run clears the ones it takes; a larger buffer is zeroed when it is allocated).
    DevBuf jobflag;
    // Stream decode: a copy of state_in when it overlaps state_out and the launch has several GOP
    // segments (segment 0's jobs read state_in while the last segment's jobs write state_out).
    DevBuf state_copy;
    unsigned long long* d_reruns = nullptr;  // jobs the exact kernel re-ran (mj423_ctx_stream_reruns), 64-bit
    // Stream-decode metadata (frame types + segment starts): a ring of upload slots, so a
    // launch never waits for the previous one.  Each slot: pinned host staging (truly async
    // H2D), a device copy, the content it holds (re-used without upload when unchanged) and
    // an event recorded after the last kernel that read it.
    struct MetaSlot {
        std::vector<uint8_t> content;
        uint8_t* pinned = nullptr;
        size_t pinned_cap = 0;
        DevBuf dev;
        hipEvent_t ev = nullptr;
        hipStream_t stream = nullptr;  // stream of the last kernel that read it (nullptr: never used)
    };
    static constexpr int kMetaSlots = 4;
    MetaSlot meta[kMetaSlots];
    int meta_next = 0;
    std::vector<uint8_t> meta_host;  // being built
    bool timing = false;
    // Every bracketed launch since timing was (re)enabled: event pairs reused across resets.
    struct TimedLaunch {
        hipEvent_t a = nullptr, b = nullptr;
        uint32_t frames = 0;
    };
    static constexpr size_t kMaxTimed = 1u << 16;
    std::vector<TimedLaunch> tlog;
    size_t tlog_n = 0;
    bool tlog_full = false;  // more launches than kMaxTimed: totals unavailable
    TimedLaunch overflow;    // once the log is full: the latest launch, for kernel_ms / kernel_frames
    long last = -1;          // the most recent bracketed launch: tlog index, -2 = overflow, -1 = none
    const TimedLaunch* last_launch() const { return last == -2 ? &overflow : last >= 0 ? &tlog[(size_t)last] : nullptr; }
    mj423_fe_cache* fe = nullptr;  // mj423_mpg_decode_gpu's device buffers
};

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int set_quant(mj423_ctx* c, const int16_t* yq, const int16_t* cq) {
    std::memcpy(c->yq, yq ? yq : kYquant, sizeof(c->yq));
    std::memcpy(c->cq, cq ? cq : kCquant, sizeof(c->cq));
    pack_table(c->yq, c->qt[0]);
    pack_table(c->cq, c->qt[1]);
    if (c->d_qt) HIP_TRY(hipMemcpyAsync(c->d_qt, c->qt, sizeof(c->qt), hipMemcpyHostToDevice, c->stream));
    return 0;
}

// Tiles per MCU row and MCUs per tile: balanced tiles of <= TWMAX MCUs.
void tiling(uint32_t mcu_cols, int chroma, bool gop, uint32_t* tpr, uint32_t* tw) {
    const uint32_t twmax = (uint32_t)(gop ? mj423_gop_tile_max_mcus(chroma) : mj423_tile_max_mcus(chroma));
    *tpr = (mcu_cols + twmax - 1) / twmax;
    *tw = (mcu_cols + *tpr - 1) / *tpr;
}

int check_ctx(mj423_ctx* c) { return c ? 0 : fail(MJ423_EINVAL, "null context"); }

// Kernel timing: opens the next log entry (nullptr when timing is off or the log is full)
// and records its start event on the context stream.
int timing_begin(mj423_ctx* c, mj423_ctx::TimedLaunch** t, hipStream_t st = nullptr) {
    *t = nullptr;
    if (!st) st = c->stream;
    if (!c->timing) return 0;
    if (c->tlog_n == mj423_ctx::kMaxTimed) {  // totals are gone, the latest launch is still timed
        c->tlog_full = true;
        if (!c->overflow.a) {
            HIP_TRY(hipEventCreate(&c->overflow.a));
            HIP_TRY(hipEventCreate(&c->overflow.b));
        }
        *t = &c->overflow;
        HIP_TRY(hipEventRecord((*t)->a, st));
        return 0;
    }
    if (c->tlog_n == c->tlog.size()) {
        mj423_ctx::TimedLaunch n;
        HIP_TRY(hipEventCreate(&n.a));
        if (hipError_t e = hipEventCreate(&n.b)) {
            (void)hipEventDestroy(n.a);
            return hipfail(e, "hipEventCreate");
        }
        c->tlog.push_back(n);
    }
    *t = &c->tlog[c->tlog_n];
    HIP_TRY(hipEventRecord((*t)->a, st));
    return 0;
}
int timing_end(mj423_ctx* c, mj423_ctx::TimedLaunch* t, uint32_t frames, hipStream_t st = nullptr) {
    if (!t) return 0;
    HIP_TRY(hipEventRecord(t->b, st ? st : c->stream));
    t->frames = frames;
    if (t != &c->overflow) {
        c->last = (long)c->tlog_n;
        c->tlog_n++;
    } else {
        c->last = -2;
    }
    return 0;
}

// Validates a frames descriptor and fills the kernel parameter block.
int fill_params(mj423_ctx* c, const mj423_frames_desc_t* d, const mj423_geometry_t& g, mj423::DecodeParams* pp,
                bool gop = false) {
    if (!d->y || !d->cb || !d->cr || !d->out) return fail(MJ423_EINVAL, "null plane or output pointer");
    if (d->out_pitch < d->width) return fail(MJ423_EINVAL, "out_pitch < width");
    if (d->input_form != MJ423_INPUT_QUANTIZED && d->input_form != MJ423_INPUT_DEQUANTIZED)
        return fail(MJ423_EINVAL, "unknown input_form");
    if (((uintptr_t)d->y | (uintptr_t)d->cb | (uintptr_t)d->cr) & 15u)
        return fail(MJ423_EINVAL, "coefficient planes must be 16-byte aligned");
    if ((d->plane_frame_stride & 7u) != 0) return fail(MJ423_EINVAL, "plane_frame_stride must be a multiple of 8");
    if (((uintptr_t)d->out & 3u) != 0) return fail(MJ423_EINVAL, "output must be 4-byte aligned");
    mj423::DecodeParams& p = *pp;
    std::memset(&p, 0, sizeof(p));
    p.coef = d->y;
    p.cb_off = (int64_t)(d->cb - d->y);
    p.cr_off = (int64_t)(d->cr - d->y);
    p.plane_fstride = d->plane_frame_stride;
    p.out = reinterpret_cast<uint32_t*>(d->out);
    p.out_fstride = d->out_frame_stride;
    p.out_pitch = d->out_pitch;
    p.aligned16 = (((uintptr_t)d->out & 15u) == 0 && (d->out_pitch & 3u) == 0 &&
                   (d->nframes == 1 || (d->out_frame_stride & 3u) == 0))
                      ? 1u
                      : 0u;
    p.width = d->width;
    p.height = d->height;
    p.y_bw = g.y_bw;
    p.c_bw = g.c_bw;
    p.mcu_cols = g.coded_w / g.mcu_w;
    p.mcu_rows = g.coded_h / g.mcu_h;
    p.mcus_per_frame = p.mcu_cols * p.mcu_rows;
    p.cols_magic = (uint32_t)std::min<uint64_t>((1ull << 32) / p.mcu_cols, 0xffffffffull);  // d = 1: 2^32 - 1
    if (d->chroma == MJ423_CHROMA_420) {  // strips inside one MCU row (an MCU spans two block rows)
        tiling(p.mcu_cols, d->chroma, gop, &p.tiles_per_row, &p.tw);
        p.tiles_per_frame = p.mcu_rows * p.tiles_per_row;
    } else {  // raster runs of tw MCUs, wrapping across rows: every tile full but the frame's last
        p.tw = (uint32_t)(gop ? mj423_gop_tile_max_mcus(d->chroma) : mj423_tile_max_mcus(d->chroma));
        p.tiles_per_row = 0;
        p.tiles_per_frame = (p.mcus_per_frame + p.tw - 1) / p.tw;
    }
    if ((uint64_t)d->nframes * p.tiles_per_frame > 0x7fffffffull) return fail(MJ423_EINVAL, "too many tiles in one call");
    p.ntiles = d->nframes * p.tiles_per_frame;
    if (!gop) p.fgroup = mj423_batch_fgroup(d->chroma, p.tiles_per_frame);
    if (d->input_form == MJ423_INPUT_DEQUANTIZED) {
        const uint32_t one = 0x00010001u;  // unit table: (int16)(Q * 1) == Q
        for (int i = 0; i < 32; i++) p.qt[0][i] = p.qt[1][i] = one;
    } else {
        std::memcpy(p.qt, c->qt, sizeof(p.qt));
    }
    return 0;
}

// Common launcher behind every fused-decode entry point.
int launch_decode(mj423_ctx* c, const mj423_frames_desc_t* d) {
    mj423_geometry_t g;
    if (int rc = mj423_geometry(d->width, d->height, d->chroma, &g)) return rc;
    mj423::DecodeParams p;
    if (int rc = fill_params(c, d, g, &p)) return rc;
    if (d->nframes == 0) return 0;
    DeviceGuard dg(c->device);
    mj423_ctx::TimedLaunch* t;
    if (int rc = timing_begin(c, &t)) return rc;
    hipError_t e = mj423_launch_decode(&p, d->nframes, d->chroma, c->stream);
    if (e != hipSuccess) return hipfail(e, "decode kernel launch");
    return timing_end(c, t, d->nframes);
}

// ------------------------------------------------------------ default context
std::mutex g_default_mu;    // serialises work on the default context
std::mutex g_default_init;  // guards its creation
mj423_ctx* g_default = nullptr;

mj423_ctx* default_ctx() {
    std::lock_guard<std::mutex> lk(g_default_init);
    if (!g_default && mj423_ctx_create(&g_default, -1) != 0) g_default = nullptr;
    return g_default;
}

}  // namespace

int mj423_set_error(int code, const std::string& msg) { return fail(code, msg); }
mj423_ctx* mj423_default_ctx() { return default_ctx(); }
int mj423_ctx_device_id(mj423_ctx* c) { return c ? c->device : -1; }
mj423_fe_cache** mj423_ctx_fe_cache(mj423_ctx* c) { return &c->fe; }
const uint32_t* mj423_ctx_qt_dev(mj423_ctx* c) { return c->d_qt; }
void mj423_ctx_qt_packed(mj423_ctx* c, uint32_t qt[2][32]) { std::memcpy(qt, c->qt, sizeof(c->qt)); }
int mj423_ctx_timing_begin(mj423_ctx* c, void** token, void* stream) {
    mj423_ctx::TimedLaunch* t = nullptr;
    const int rc = timing_begin(c, &t, (hipStream_t)stream);
    *token = t;
    return rc;
}
int mj423_ctx_timing_end(mj423_ctx* c, void* token, uint32_t frames, void* stream) {
    return timing_end(c, static_cast<mj423_ctx::TimedLaunch*>(token), frames, (hipStream_t)stream);
}
std::mutex& mj423_default_mutex() { return g_default_mu; }

// =================================================================== C ABI
extern "C" {

int mj423_version(void) { return 0x000100; }

const char* mj423_last_error(void) { return g_err.c_str(); }

int mj423_geometry(uint32_t width, uint32_t height, int chroma, mj423_geometry_t* g) {
    if (!g) return fail(MJ423_EINVAL, "null geometry");
    uint32_t sx, sy;
    switch (chroma) {
    case MJ423_CHROMA_444: sx = 1; sy = 1; break;
    case MJ423_CHROMA_422: sx = 2; sy = 1; break;
    case MJ423_CHROMA_420: sx = 2; sy = 2; break;
    default: return fail(MJ423_EINVAL, "chroma must be 444, 422 or 420");
    }
    if (width == 0 || height == 0 || width > (1u << 20) || height > (1u << 20))
        return fail(MJ423_EINVAL, "frame size out of range");
    g->width = width;
    g->height = height;
    g->chroma = chroma;
    g->mcu_w = 8 * sx;
    g->mcu_h = 8 * sy;
    g->coded_w = (width + g->mcu_w - 1) / g->mcu_w * g->mcu_w;
    g->coded_h = (height + g->mcu_h - 1) / g->mcu_h * g->mcu_h;
    g->y_bw = g->coded_w / 8;
    g->y_bh = g->coded_h / 8;
    g->c_bw = g->y_bw / sx;
    g->c_bh = g->y_bh / sy;
    g->y_blocks = g->y_bw * g->y_bh;
    g->c_blocks = g->c_bw * g->c_bh;
    g->coef_per_frame = 64ull * ((uint64_t)g->y_blocks + 2ull * g->c_blocks);
    return 0;
}

uint64_t mj423_frame_bytes(uint32_t width, uint32_t height, int chroma) {
    mj423_geometry_t g;
    if (mj423_geometry(width, height, chroma, &g)) return 0;
    return 2ull * g.coef_per_frame + 4ull * width * height;
}

int mj423_ctx_create(mj423_ctx** out, int device) {
    return mj423_guarded([&]() -> int {
        if (!out) return fail(MJ423_EINVAL, "null ctx pointer");
        *out = nullptr;
        int ndev = 0;
        hipError_t e = hipGetDeviceCount(&ndev);
        if (e != hipSuccess || ndev == 0)
            return fail(MJ423_EHIP, "no HIP device available: the MI355X kernels cannot run (no CPU fallback exists)");
        if (device < 0) HIP_TRY(hipGetDevice(&device));
        if (device >= ndev) return fail(MJ423_EINVAL, "device index out of range");
        mj423_ctx* c = new mj423_ctx();
        c->device = device;
        DeviceGuard dg(device);
        if ((e = hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking)) != hipSuccess) {
            delete c;
            return hipfail(e, "hipStreamCreate");
        }
        c->stream = c->own;
        if ((e = hipMalloc(&c->d_qt, sizeof(c->qt))) != hipSuccess) {
            mj423_ctx_destroy(c);
            return hipfail(e, "context resources");
        }
        if (int rc = set_quant(c, nullptr, nullptr)) {
            mj423_ctx_destroy(c);
            return rc;
        }
        *out = c;
        return 0;
    });
}

void mj423_ctx_destroy(mj423_ctx* c) {
    if (!c) return;
    DeviceGuard dg(c->device);
    if (c->stream) (void)hipStreamSynchronize(c->stream);
    c->in.release();
    c->out.release();
    c->scratch.release();
    c->jobflag.release();
    c->state_copy.release();
    if (c->d_reruns) (void)hipFree(c->d_reruns);
    c->d_reruns = nullptr;
    mj423_fe_cache_release(c->fe);
    c->fe = nullptr;
    for (auto& m : c->meta) {
        m.dev.release();
        if (m.pinned) (void)hipHostFree(m.pinned);
        if (m.ev) (void)hipEventDestroy(m.ev);
    }
    if (c->d_qt) (void)hipFree(c->d_qt);
    for (auto& t : c->tlog) {
        (void)hipEventDestroy(t.a);
        (void)hipEventDestroy(t.b);
    }
    if (c->overflow.a) (void)hipEventDestroy(c->overflow.a);
    if (c->overflow.b) (void)hipEventDestroy(c->overflow.b);
    if (c->own) (void)hipStreamDestroy(c->own);
    delete c;
}

int mj423_ctx_set_stream(mj423_ctx* c, void* s) {
    if (int rc = check_ctx(c)) return rc;
    c->stream = s ? (hipStream_t)s : c->own;
    return 0;
}

void* mj423_ctx_stream(mj423_ctx* c) { return c ? (void*)c->stream : nullptr; }

int mj423_ctx_set_quant(mj423_ctx* c, const int16_t yq[64], const int16_t cq[64]) {
    if (int rc = check_ctx(c)) return rc;
    DeviceGuard dg(c->device);
    return set_quant(c, yq, cq);
}

int mj423_ctx_get_quant(mj423_ctx* c, int16_t yq[64], int16_t cq[64]) {
    if (int rc = check_ctx(c)) return rc;
    if (yq) std::memcpy(yq, c->yq, sizeof(c->yq));
    if (cq) std::memcpy(cq, c->cq, sizeof(c->cq));
    return 0;
}

int mj423_ctx_synchronize(mj423_ctx* c) {
    if (int rc = check_ctx(c)) return rc;
    DeviceGuard dg(c->device);
    HIP_TRY(hipStreamSynchronize(c->stream));
    return 0;
}

int mj423_ctx_enable_timing(mj423_ctx* c, int on) {
    if (int rc = check_ctx(c)) return rc;
    c->timing = on != 0;
    c->tlog_n = 0;
    c->tlog_full = false;
    c->last = -1;
    return 0;
}

uint32_t mj423_ctx_kernel_frames(mj423_ctx* c) { return c && c->last_launch() ? c->last_launch()->frames : 0u; }

double mj423_ctx_kernel_ms(mj423_ctx* c) {
    if (!c || !c->last_launch()) return -1.0;
    DeviceGuard dg(c->device);
    const mj423_ctx::TimedLaunch& t = *c->last_launch();
    if (hipEventSynchronize(t.b) != hipSuccess) return -1.0;
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, t.a, t.b) != hipSuccess) return -1.0;
    return (double)ms;
}

int mj423_ctx_kernel_totals(mj423_ctx* c, double* ms, uint64_t* frames, uint32_t* launches) {
    return mj423_guarded([&]() -> int {
        if (int rc = check_ctx(c)) return rc;
        if (!ms || !frames || !launches) return fail(MJ423_EINVAL, "null output pointer");
        *ms = 0.0;
        *frames = 0;
        *launches = 0;
        if (c->tlog_full) return fail(MJ423_EINVAL, "more timed launches than the log holds; re-enable timing sooner");
        DeviceGuard dg(c->device);
        for (size_t i = 0; i < c->tlog_n; i++) {  // launches on one stream finish in order; any may be on another
            const mj423_ctx::TimedLaunch& t = c->tlog[i];
            HIP_TRY(hipEventSynchronize(t.b));
            float x = 0.f;
            HIP_TRY(hipEventElapsedTime(&x, t.a, t.b));
            *ms += x;
            *frames += t.frames;
        }
        *launches = (uint32_t)c->tlog_n;
        return 0;
    });
}

int mj423_ctx_stream_reruns(mj423_ctx* c, uint64_t* jobs) {
    return mj423_guarded([&]() -> int {
        if (int rc = check_ctx(c)) return rc;
        if (!jobs) return fail(MJ423_EINVAL, "null output");
        *jobs = 0;
        if (!c->d_reruns) return 0;
        DeviceGuard dg(c->device);
        HIP_TRY(hipStreamSynchronize(c->stream));
        unsigned long long n = 0;
        HIP_TRY(hipMemcpy(&n, c->d_reruns, sizeof n, hipMemcpyDeviceToHost));
        *jobs = n;
        return 0;
    });
}

// ----------------------------------------------------------- device batches
int mj423_decode_frames_device(mj423_ctx* c, const mj423_frames_desc_t* d) {
    return mj423_guarded([&]() -> int {
        if (int rc = check_ctx(c)) return rc;
        if (!d) return fail(MJ423_EINVAL, "null descriptor");
        return launch_decode(c, d);
    });
}

int mj423_decode_stream_device(mj423_ctx* c, const mj423_frames_desc_t* d, const uint8_t* frame_types,
                               const int16_t* state_in, int16_t* state_out) {
    return mj423_guarded([&]() -> int {
        if (int rc = check_ctx(c)) return rc;
        if (!d || !frame_types) return fail(MJ423_EINVAL, "null descriptor or frame types");
        if (d->input_form != MJ423_INPUT_QUANTIZED) return fail(MJ423_EINVAL, "stream decode takes quantized input");
        mj423_geometry_t g;
        if (int rc = mj423_geometry(d->width, d->height, d->chroma, &g)) return rc;
        if (d->nframes == 0) return 0;
        if (frame_types[0] != 0 && !state_in) return fail(MJ423_EINVAL, "frame 0 is a P-frame: state_in is required");
        if (((uintptr_t)state_in | (uintptr_t)state_out) & 15u) return fail(MJ423_EINVAL, "state buffers must be 16-byte aligned");
        // Segments: frame 0, then every later I-frame.
        std::vector<uint32_t> seg;
        std::vector<uint8_t> types(frame_types, frame_types + d->nframes);
        for (uint32_t f = 0; f < d->nframes; f++) {
            if (types[f] > 1) return fail(MJ423_EINVAL, "frame type must be 0 (I) or 1 (P)");
            if (f == 0 || types[f] == 0) seg.push_back(f);
        }
        seg.push_back(d->nframes);
        const uint32_t nseg = (uint32_t)seg.size() - 1;
        if (nseg > 65535) return fail(MJ423_EINVAL, "more than 65535 GOPs in one call");
        DeviceGuard dg(c->device);
        const size_t toff = ((size_t)d->nframes + 15) / 16 * 16;
        const size_t meta = toff + seg.size() * 4;
        c->meta_host.assign(meta, 0);
        std::memcpy(c->meta_host.data(), types.data(), types.size());
        std::memcpy(c->meta_host.data() + toff, seg.data(), seg.size() * 4);
        mj423_ctx::MetaSlot* ms = nullptr;
        for (auto& m : c->meta)  // unchanged metadata (a bench or a player repeating a GOP pattern): no upload
            if (m.stream && m.content == c->meta_host) {
                ms = &m;
                if (m.stream != c->stream) HIP_TRY(hipStreamWaitEvent(c->stream, m.ev, 0));
                break;
            }
        if (!ms) {
            ms = &c->meta[c->meta_next];
            c->meta_next = (c->meta_next + 1) % mj423_ctx::kMetaSlots;
            if (!ms->ev) HIP_TRY(hipEventCreateWithFlags(&ms->ev, hipEventDisableTiming));
            if (ms->stream) HIP_TRY(hipEventSynchronize(ms->ev));  // its last reader, kMetaSlots launches ago
            if (ms->pinned_cap < meta) {
                if (ms->pinned) (void)hipHostFree(ms->pinned);
                ms->pinned = nullptr;
                ms->pinned_cap = 0;
                HIP_TRY(hipHostMalloc((void**)&ms->pinned, meta, hipHostMallocDefault));
                ms->pinned_cap = meta;
            }
            if (int rc = ms->dev.ensure(meta)) return rc;
            std::memcpy(ms->pinned, c->meta_host.data(), meta);
            ms->content = c->meta_host;
            HIP_TRY(hipMemcpyAsync(ms->dev.p, ms->pinned, meta, hipMemcpyHostToDevice, c->stream));
        }
        const uint8_t* dmeta = (const uint8_t*)ms->dev.p;
        mj423::DecodeParams p;
        if (int rc = fill_params(c, d, g, &p, true)) return rc;
        p.qt_dev = c->d_qt;
        p.ftype = dmeta;
        p.seg_start = (const uint32_t*)(dmeta + toff);
        p.nseg = nseg;
        p.state = state_in;
        p.state_out = state_out;
        if (state_in && state_out && (nseg > 1 || state_in != state_out)) {
            // Segment 0's jobs seed from state_in (and the optimistic kernel's exact re-run seeds from
            // it again) while the last segment's jobs write state_out, in no fixed order: with several
            // segments any overlap, with one segment an overlap that is not the exact alias (a tile's
            // end state then lands on another tile's seed), would let a job read an end state --
            // decode from a copy.  (One segment, state_out == state_in: each job reads its own tile's
            // seed before it writes the same bytes; a flagged job writes none.)
            const size_t sb = (size_t)g.coef_per_frame * 2;
            const uintptr_t a0 = (uintptr_t)state_in, b0 = (uintptr_t)state_out;
            if (a0 < b0 + sb && b0 < a0 + sb) {
                if (int rc = c->state_copy.ensure(sb)) return rc;
                HIP_TRY(hipMemcpyAsync(c->state_copy.p, state_in, sb, hipMemcpyDeviceToDevice, c->stream));
                p.state = (const int16_t*)c->state_copy.p;
            }
        }
        p.st_cb_off = 64ll * g.y_blocks;
        p.st_cr_off = 64ll * (g.y_blocks + g.c_blocks);
        {
            const size_t fb = ((size_t)p.tiles_per_frame * nseg * 4 + 255) / 256 * 256;
            if (fb > c->jobflag.cap) {
                if (int rc = c->jobflag.ensure(fb)) return rc;
                HIP_TRY(hipMemsetAsync(c->jobflag.p, 0, fb, c->stream));
            }
            p.jobflag = (uint32_t*)c->jobflag.p;
            if (!c->d_reruns) {
                HIP_TRY(hipMalloc(&c->d_reruns, sizeof *c->d_reruns));
                HIP_TRY(hipMemsetAsync(c->d_reruns, 0, sizeof *c->d_reruns, c->stream));
            }
            p.reruns = c->d_reruns;
        }
        mj423_ctx::TimedLaunch* t;
        if (int rc = timing_begin(c, &t)) return rc;
        hipError_t e = mj423_launch_decode_gop(&p, nseg, d->chroma, c->stream);
        if (e != hipSuccess) return hipfail(e, "stream decode kernel launch");
        if (int rc = timing_end(c, t, d->nframes)) return rc;
        HIP_TRY(hipEventRecord(ms->ev, c->stream));
        ms->stream = c->stream;
        return 0;
    });
}

int mj423_synth_frames_device(mj423_ctx* c, int16_t* coef, uint32_t w, uint32_t h, int chroma, uint32_t nframes,
                              uint64_t frame0, uint64_t seed) {
    return mj423_guarded([&]() -> int {
        if (int rc = check_ctx(c)) return rc;
        mj423_geometry_t g;
        if (int rc = mj423_geometry(w, h, chroma, &g)) return rc;
        if (!coef || ((uintptr_t)coef & 15u)) return fail(MJ423_EINVAL, "coef must be a 16-byte aligned device pointer");
        mj423::SynthParams p;
        std::memset(&p, 0, sizeof(p));
        p.coef = coef;
        p.frame_stride = g.coef_per_frame;
        p.y_blocks = g.y_blocks;
        p.c_blocks = g.c_blocks;
        p.nframes = nframes;
        p.frame0 = frame0;
        p.seed = seed;
        std::memcpy(p.yq, c->yq, sizeof(p.yq));
        std::memcpy(p.cq, c->cq, sizeof(p.cq));
        std::memcpy(p.zigzag, kZigzag, sizeof(p.zigzag));
        for (int k = 0; k < 64; k++) {
            const double prob = k == 0 ? 0.0 : 0.6 * std::exp(-k / 8.0);
            p.ac_thresh[k] = (uint32_t)std::min(prob * 4294967296.0, 4294967295.0);
        }
        DeviceGuard dg(c->device);
        hipError_t e = mj423_launch_synth(&p, c->stream);
        if (e != hipSuccess) return hipfail(e, "synth kernel launch");
        return 0;
    });
}

// --------------------------------------------------------------- frame call
int decode_frames(mj423_ctx* c, uint32_t n, const int16_t* coef, rgb_pixel_t* out, uint32_t w, uint32_t h,
                  int chroma, int input_form) {
    return mj423_guarded([&]() -> int {
        if (int rc = check_ctx(c)) return rc;
        mj423_geometry_t g;
        if (int rc = mj423_geometry(w, h, chroma, &g)) return rc;
        if (!coef || !out) return fail(MJ423_EINVAL, "null buffer");
        if (n == 0) return 0;
        const size_t in_bytes = (size_t)n * g.coef_per_frame * 2;
        const size_t out_px = (size_t)w * h;
        DeviceGuard dg(c->device);
        if (int rc = c->in.ensure(in_bytes)) return rc;
        if (int rc = c->out.ensure((size_t)n * out_px * 4)) return rc;
        HIP_TRY(hipMemcpyAsync(c->in.p, coef, in_bytes, hipMemcpyHostToDevice, c->stream));
        const int16_t* y = (const int16_t*)c->in.p;
        mj423_frames_desc_t d = {y,
                                 y + 64ull * g.y_blocks,
                                 y + 64ull * (g.y_blocks + g.c_blocks),
                                 g.coef_per_frame,
                                 (rgb_pixel_t*)c->out.p,
                                 out_px,
                                 w,
                                 n,
                                 w,
                                 h,
                                 chroma,
                                 input_form};
        if (int rc = launch_decode(c, &d)) return rc;
        HIP_TRY(hipMemcpyAsync(out, c->out.p, (size_t)n * out_px * 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        return 0;
    });
}

int mj423_decode_frame_ex(mj423_ctx* c, const int16_t* Yq, const int16_t* Cbq, const int16_t* Crq, rgb_pixel_t* out,
                          uint32_t w, uint32_t h, int chroma, int input_form) {
    return mj423_guarded([&]() -> int {
        if (int rc = check_ctx(c)) return rc;
        mj423_geometry_t g;
        if (int rc = mj423_geometry(w, h, chroma, &g)) return rc;
        if (!Yq || !Cbq || !Crq || !out) return fail(MJ423_EINVAL, "null buffer");
        const size_t yb = 128ull * g.y_blocks, cb = 128ull * g.c_blocks;
        const size_t out_bytes = (size_t)w * h * 4;
        DeviceGuard dg(c->device);
        if (int rc = c->in.ensure(yb + 2 * cb)) return rc;
        if (int rc = c->out.ensure(out_bytes)) return rc;
        char* base = (char*)c->in.p;
        HIP_TRY(hipMemcpyAsync(base, Yq, yb, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(base + yb, Cbq, cb, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(base + yb + cb, Crq, cb, hipMemcpyHostToDevice, c->stream));
        mj423_frames_desc_t d = {(const int16_t*)base,
                                 (const int16_t*)(base + yb),
                                 (const int16_t*)(base + yb + cb),
                                 g.coef_per_frame,
                                 (rgb_pixel_t*)c->out.p,
                                 (uint64_t)w * h,
                                 w,
                                 1,
                                 w,
                                 h,
                                 chroma,
                                 input_form};
        if (int rc = launch_decode(c, &d)) return rc;
        HIP_TRY(hipMemcpyAsync(out, c->out.p, out_bytes, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        return 0;
    });
}

int decode_frame(mj423_ctx* c, const int16_t* Yq, const int16_t* Cbq, const int16_t* Crq, rgb_pixel_t* out,
                 uint32_t w, uint32_t h, int chroma) {
    return mj423_decode_frame_ex(c, Yq, Cbq, Crq, out, w, h, chroma, MJ423_INPUT_QUANTIZED);
}

// ------------------------------------------------------------- stage calls
int mj423_idct_blocks(mj423_ctx* c, size_t n, const int16_t* DCAC, const int16_t* quant, uint8_t* blocks) {
    return mj423_guarded([&]() -> int {
        if (int rc = check_ctx(c)) return rc;
        if (!DCAC || !blocks) return fail(MJ423_EINVAL, "null buffer");
        if (n == 0) return 0;
        if (n > 0xffffffffull) return fail(MJ423_EINVAL, "too many blocks");
        DeviceGuard dg(c->device);
        if (int rc = c->in.ensure(n * 128)) return rc;
        if (int rc = c->out.ensure(n * 64)) return rc;
        const uint32_t* qt = nullptr;
        if (quant) {
            if (int rc = c->scratch.ensure(128)) return rc;
            uint32_t packed[32];
            pack_table(quant, packed);
            HIP_TRY(hipMemcpyAsync(c->scratch.p, packed, 128, hipMemcpyHostToDevice, c->stream));
            qt = (const uint32_t*)c->scratch.p;
        }
        HIP_TRY(hipMemcpyAsync(c->in.p, DCAC, n * 128, hipMemcpyHostToDevice, c->stream));
        hipError_t e = mj423_launch_idct_blocks((const int16_t*)c->in.p, (uint8_t*)c->out.p, (uint32_t)n, qt, c->stream);
        if (e != hipSuccess) return hipfail(e, "idct kernel launch");
        HIP_TRY(hipMemcpyAsync(blocks, c->out.p, n * 64, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        return 0;
    });
}

int mj423_ycbcr_to_rgb_444(mj423_ctx* c, uint32_t w_size, uint32_t h_size, const uint8_t* Y, const uint8_t* Cb,
                           const uint8_t* Cr, rgb_pixel_t* rgb) {
    return mj423_guarded([&]() -> int {
        if (int rc = check_ctx(c)) return rc;
        if (!Y || !Cb || !Cr || !rgb) return fail(MJ423_EINVAL, "null buffer");
        if (w_size == 0 || h_size == 0 || (w_size & 7u) || (h_size & 7u))
            return fail(MJ423_EINVAL, "4:4:4 block-raster frame needs width and height multiples of 8");
        const size_t plane = (size_t)w_size * h_size;
        DeviceGuard dg(c->device);
        if (int rc = c->in.ensure(3 * plane)) return rc;
        if (int rc = c->out.ensure(plane * 4)) return rc;
        uint8_t* b = (uint8_t*)c->in.p;
        HIP_TRY(hipMemcpyAsync(b, Y, plane, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(b + plane, Cb, plane, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(b + 2 * plane, Cr, plane, hipMemcpyHostToDevice, c->stream));
        hipError_t e = mj423_launch_csc444(b, b + plane, b + 2 * plane, (uint32_t*)c->out.p, w_size, h_size, w_size,
                                           c->stream);
        if (e != hipSuccess) return hipfail(e, "csc kernel launch");
        HIP_TRY(hipMemcpyAsync(rgb, c->out.p, plane * 4, hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        return 0;
    });
}

}  // extern "C"
