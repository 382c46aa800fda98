// mj423_internal.h -- helpers shared by the library's host translation units (not exported API).
#pragma once
#include <exception>
#include <mutex>
#include <new>
#include <string>

#include "../../include/mj423gpu.h"

// Records msg as this thread's mj423_last_error() and returns code.
int mj423_set_error(int code, const std::string& msg);

// Runs an entry point's body so that no C++ exception crosses the C ABI: allocation
// failures become MJ423_ENOMEM, anything else MJ423_EINVAL, with the message recorded.
template <class F>
int mj423_guarded(F&& body) noexcept {
    try {
        return body();
    } catch (const std::bad_alloc&) {
        return mj423_set_error(MJ423_ENOMEM, "out of host memory");
    } catch (const std::exception& e) {
        return mj423_set_error(MJ423_EINVAL, std::string("internal error: ") + e.what());
    } catch (...) {
        return mj423_set_error(MJ423_EINVAL, "internal error");
    }
}
// The process-default context behind the reference's context-free symbols
// (idct, ycbcr_to_rgb, mjpeg423_decode); created on first use, nullptr if no GPU.
mj423_ctx* mj423_default_ctx();
// The HIP device a context was created on (-1 for null).
int mj423_ctx_device_id(mj423_ctx* ctx);
// Serialises users of the default context.
std::mutex& mj423_default_mutex();
// Host threads the library's pools use by default: the CPUs this process may run on (affinity
// mask), capped by a cgroup v2 `cpu.max` quota; not std::thread::hardware_concurrency(), which
// counts the whole machine (256 on the MI355X hosts, of which a job may own 16).
int mj423_host_threads();
// Decodes this thread's deferred idct() / ycbcr_to_rgb() calls (mj423_dropin.cpp); the
// library's encode_bmp() and lossless_decode() call it before they touch any buffer.
void mj423_dropin_flush_point();

struct mj423_mpg;
// Planes of a w x h .mpg stream: the w/8 x h/8 whole blocks the reference codes
// (mjpeg423_decoder.c:45-48), i.e. mj423_geometry(w & ~7, h & ~7, 444); zero blocks (and
// coef_per_frame 0) when w or h is below 8.  Pure host arithmetic.
int mj423_coded_geometry_444(uint32_t w, uint32_t h, mj423_geometry_t* g);
// The defined fill outside a frame's coded region: pixels (x, y) with x >= cw or y >= ch of
// nframes frames (frame i at out + i * frame_stride, rows `pitch` pixels apart, w x h displayed)
// set to zero on `stream` (a hipStream_t).  No-op when cw == w and ch == h.  hipError_t as int.
int mj423_launch_fill_margin(rgb_pixel_t* out, uint64_t frame_stride, uint32_t pitch, uint32_t cw, uint32_t ch,
                             uint32_t w, uint32_t h, uint32_t nframes, void* stream);
// One (frame, plane) task of mj423_mpg_entropy_decode_deltas: plane `plane` of frame f
// into frame_coef ([Y | Cb | Cr] of that frame); plane 0 also stores the frame type.
// 0 on success, -1 if the bitstream ran out.
int mj423_delta_plane_task(const mj423_mpg* m, uint32_t f, int plane, int16_t* frame_coef, uint8_t* frame_type);
// Sparse form of the same task (walk_sparse in mj423_io.cpp): per-block counts, entries
// (natural index << 16 | uint16 value; I absolute, P deltas) and per-256-block entry
// offsets; `ent` must hold 64 * blocks-per-plane entries.  Returns the entry count, -1
// if the bitstream ran out.
long mj423_sparse_plane_task(const mj423_mpg* m, uint32_t f, int plane, uint8_t* counts, uint32_t* seg_off,
                             uint32_t* ent, uint8_t* frame_type);

// mj423_pipeline_create for one known decode, frames [first, first + frames) of `m`
// (mj423_pipeline.cpp): with chunk_frames 0 the ring is sized to the call (chunks of
// ceil(frames / 6), at most the default) instead of to a long stream, the transfer
// buffers to what those frames' bitstreams can expand to instead of dense planes, and
// `sink_threads` > 1 calls the host sink for a chunk's frames concurrently and in no
// particular order (sinks with independent outputs, e.g. one BMP file per frame).
// m == nullptr: no sizing hint (mj423_pipeline_create).
struct mj423_pipeline;
int mj423_pipeline_create_for(mj423_pipeline** out, mj423_ctx* ctx, uint32_t w, uint32_t h, uint32_t chunk_frames,
                              int nthreads, const mj423_mpg* m, uint32_t first, uint32_t frames, int sink_threads);

// Device buffers of the whole-GPU .mpg decoder (mj423_gpu_frontend.cpp), kept by the
// context across calls and released by mj423_ctx_destroy.
struct mj423_fe_cache;
mj423_fe_cache** mj423_ctx_fe_cache(mj423_ctx* ctx);
void mj423_fe_cache_release(mj423_fe_cache* c);
// The context's packed quant tables (mj423_ctx_set_quant): on the device, and a host copy.
const uint32_t* mj423_ctx_qt_dev(mj423_ctx* ctx);
void mj423_ctx_qt_packed(mj423_ctx* ctx, uint32_t qt[2][32]);
// Brackets a launch on the context's stream with its timing events (mj423_ctx_enable_timing;
// mj423_ctx_kernel_totals sums them): begin before the launch, end after it.
int mj423_ctx_timing_begin(mj423_ctx* ctx, void** token, void* stream = nullptr);  // stream: default the context's
int mj423_ctx_timing_end(mj423_ctx* ctx, void* token, uint32_t frames, void* stream = nullptr);
// A page-locked copy of the file's bytes for asynchronous uploads: made on the first call (one
// hipHostMalloc + memcpy, thread-safe), freed by mj423_mpg_close; byte i of the file is at [i].
// nullptr if the driver refused (uploads then go from pageable memory, synchronously staged).
const uint8_t* mj423_mpg_pinned(const mj423_mpg* m);
