// mj423_pipeline.cpp -- streaming .mpg decoder (include/mj423io.h,
// mj423_decode_mpg_pipelined): the reference's per-frame loop
// (mjpeg423_decoder.c:88-141: read frame, lossless_decode x3, IDCT + CSC, write BMP)
// restructured as a four-stage pipeline over chunks of frames so that every stage
// runs at the same time on its own resource:
//
//   front end (host threads)  ->  H2D (copy stream)  ->  stream-decode kernel
//   (compute stream)  ->  D2H (copy stream)  ->  sink (caller's callback thread)
//
// Chunks travel through a ring of slots (pinned host + device buffers).  The front end
// emits per-frame deltas (every (frame, plane) bitstream independent); the GPU keeps
// the accumulated P-frame coefficients on chip within a chunk and hands them to the
// next chunk through a device state buffer (state_out -> state_in), so a GOP may span
// chunk boundaries with no host-side accumulation.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mj423io.h"
#include "mj423_internal.h"

namespace {

using clk = std::chrono::steady_clock;
double secs(clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); }

struct Slot {
    int16_t* h_coef = nullptr;  // pinned: front end output
    uint8_t* types = nullptr;   // host: frame types of the chunk
    rgb_pixel_t* h_out = nullptr;  // pinned: D2H target
    void* d_coef = nullptr;
    void* d_out = nullptr;
    hipEvent_t uploaded = nullptr, decoded = nullptr, downloaded = nullptr;
    uint32_t first = 0, count = 0;
    // ring protocol: FREE -> FILLED (front end) -> SUBMITTED (GPU) -> FREE (sink)
    enum { FREE, FILLED, SUBMITTED } state = FREE;
    int64_t seq = -1;  // chunk number held
};

// First error wins; carries its message across threads (mj423_last_error is thread-local).
struct ErrBox {
    std::mutex mu;
    int code = 0;
    std::string msg;
    std::atomic<bool> set{false};
    void put(int c, const char* m) {
        std::lock_guard<std::mutex> lk(mu);
        if (code == 0) {
            code = c;
            msg = m ? m : "";
            set.store(true);
        }
    }
};

}  // namespace

extern "C" int mj423_decode_mpg_pipelined(mj423_ctx* ctx, const mj423_mpg* m, uint32_t first, uint32_t count,
                                          uint32_t chunk_frames, int nthreads, mj423_frame_sink_fn sink, void* user,
                                          mj423_pipeline_stats_t* stats) {
    if (!ctx || !m || !sink) return mj423_set_error(MJ423_EINVAL, "pipeline: null argument");
    mj423_mpg_header_t hdr;
    if (int rc = mj423_mpg_header(m, &hdr)) return rc;
    if ((uint64_t)first + count > hdr.num_frames) return mj423_set_error(MJ423_EINVAL, "pipeline: frame range out of range");
    if (stats) std::memset(stats, 0, sizeof(*stats));
    if (count == 0) return 0;
    const uint32_t w = hdr.width, h = hdr.height;
    mj423_geometry_t g;
    if (int rc = mj423_geometry(w, h, MJ423_CHROMA_444, &g)) return rc;
    const size_t frame_bytes = (size_t)g.coef_per_frame * 2 + (size_t)w * h * 4;
    const uint32_t cap = (uint32_t)std::max<size_t>(1, (256ull << 20) / frame_bytes);
    const uint32_t chunk = std::max<uint32_t>(1, std::min({chunk_frames ? chunk_frames : std::min(24u, cap), count}));
    const uint32_t nchunks = (count + chunk - 1) / chunk;
    const int kSlots = 3;
    const size_t coef_pf = g.coef_per_frame, px_pf = (size_t)w * h;
    const size_t coef_bytes = (size_t)chunk * coef_pf * 2, out_bytes = (size_t)chunk * px_pf * 4;
    const clk::time_point t_start = clk::now();

    const int dev = mj423_ctx_device_id(ctx);
    int prev_dev = -1;
    (void)hipGetDevice(&prev_dev);
    if (hipSetDevice(dev) != hipSuccess) return mj423_set_error(MJ423_EHIP, "pipeline: hipSetDevice failed");
    hipStream_t s_comp = (hipStream_t)mj423_ctx_stream(ctx);
    hipStream_t s_in = nullptr, s_out = nullptr;
    Slot slots[kSlots];
    void* d_state[2] = {nullptr, nullptr};
    int rc = 0;
    auto hipok = [&](hipError_t e, const char* what) {
        if (e != hipSuccess && rc == 0)
            rc = mj423_set_error(MJ423_EHIP, std::string("pipeline: ") + what + ": " + hipGetErrorString(e));
        return e == hipSuccess;
    };
    bool ok = hipok(hipStreamCreateWithFlags(&s_in, hipStreamNonBlocking), "stream") &&
              hipok(hipStreamCreateWithFlags(&s_out, hipStreamNonBlocking), "stream") &&
              hipok(hipMalloc(&d_state[0], coef_pf * 2), "hipMalloc") &&
              hipok(hipMalloc(&d_state[1], coef_pf * 2), "hipMalloc");
    for (int i = 0; ok && i < kSlots; i++) {
        Slot& sl = slots[i];
        ok = hipok(hipHostMalloc((void**)&sl.h_coef, coef_bytes, hipHostMallocDefault), "hipHostMalloc") &&
             hipok(hipHostMalloc((void**)&sl.h_out, out_bytes, hipHostMallocDefault), "hipHostMalloc") &&
             hipok(hipMalloc(&sl.d_coef, coef_bytes), "hipMalloc") && hipok(hipMalloc(&sl.d_out, out_bytes), "hipMalloc") &&
             hipok(hipEventCreateWithFlags(&sl.uploaded, hipEventDisableTiming), "event") &&
             hipok(hipEventCreateWithFlags(&sl.decoded, hipEventDisableTiming), "event") &&
             hipok(hipEventCreateWithFlags(&sl.downloaded, hipEventDisableTiming), "event");
        if (ok) sl.types = new uint8_t[chunk];
    }
    // Seeking into a GOP: the absolute coefficients of frame first-1 seed the GPU state.
    uint8_t t0 = 0;
    if (ok) {
        mj423_mpg_frame_t fr;
        ok = mj423_mpg_frame(m, first, &fr) == 0 || (rc = MJ423_EINVAL, false);
        t0 = ok ? (uint8_t)fr.frame_type : 0;
    }
    if (ok && t0 != 0) {
        std::vector<int16_t> st(coef_pf);
        if ((rc = mj423_mpg_entropy_decode(m, first - 1, 1, st.data(), nthreads)) != 0)
            ok = false;
        else
            ok = hipok(hipMemcpy(d_state[1], st.data(), coef_pf * 2, hipMemcpyHostToDevice), "state upload");
    }

    std::mutex mu;
    std::condition_variable cv;
    ErrBox err;
    double fe_busy = 0.0, sink_busy = 0.0;
    std::atomic<bool> stop{false};

    // ---- front end: fills FREE slots with chunk c (slot c % kSlots), in order
    auto front = [&]() {
        for (uint32_t c = 0; c < nchunks && !stop.load(); c++) {
            Slot& sl = slots[c % kSlots];
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop.load() || sl.state == Slot::FREE; });
                if (stop.load()) return;
            }
            sl.first = first + c * chunk;
            sl.count = std::min(chunk, first + count - sl.first);
            const clk::time_point a = clk::now();
            if (mj423_mpg_entropy_decode_deltas(m, sl.first, sl.count, sl.h_coef, sl.types, nthreads) != 0) {
                err.put(MJ423_EINVAL, mj423_last_error());
                stop.store(true);
                cv.notify_all();
                return;
            }
            fe_busy += secs(a, clk::now());
            std::lock_guard<std::mutex> lk(mu);
            sl.seq = c;
            sl.state = Slot::FILLED;
            cv.notify_all();
        }
    };
    // ---- sink: waits for chunk c's download, hands frames to the caller in order
    auto back = [&]() {
        for (uint32_t c = 0; c < nchunks && !stop.load(); c++) {
            Slot& sl = slots[c % kSlots];
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop.load() || (sl.state == Slot::SUBMITTED && sl.seq == (int64_t)c); });
                if (stop.load()) return;
            }
            if (hipEventSynchronize(sl.downloaded) != hipSuccess) {
                err.put(MJ423_EHIP, "pipeline: GPU stage failed");
                stop.store(true);
                cv.notify_all();
                return;
            }
            const clk::time_point a = clk::now();
            for (uint32_t i = 0; i < sl.count; i++) {
                if (sink(user, sl.first + i, sl.h_out + (size_t)i * px_pf, w, h) != 0) {
                    err.put(MJ423_EINVAL, "pipeline: frame sink reported an error");
                    stop.store(true);
                    cv.notify_all();
                    return;
                }
            }
            sink_busy += secs(a, clk::now());
            std::lock_guard<std::mutex> lk(mu);
            sl.state = Slot::FREE;
            sl.seq = -1;
            cv.notify_all();
        }
    };

    float gpu_ms = 0.f;
    hipEvent_t g0 = nullptr, g1 = nullptr;
    if (ok) ok = hipok(hipEventCreate(&g0), "event") && hipok(hipEventCreate(&g1), "event");
    if (ok) {
        std::thread tf(front), tb(back);
        (void)hipSetDevice(dev);  // this thread submits the GPU stages
        bool first_kernel = true;
        for (uint32_t c = 0; c < nchunks; c++) {
            Slot& sl = slots[c % kSlots];
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop.load() || (sl.state == Slot::FILLED && sl.seq == (int64_t)c); });
                if (stop.load()) break;
            }
            const size_t nb = (size_t)sl.count * coef_pf * 2;
            // H2D on the copy-in stream; the kernel waits for it; D2H waits for the kernel.
            bool k = hipok(hipMemcpyAsync(sl.d_coef, sl.h_coef, nb, hipMemcpyHostToDevice, s_in), "H2D") &&
                     hipok(hipEventRecord(sl.uploaded, s_in), "event") &&
                     hipok(hipStreamWaitEvent(s_comp, sl.uploaded, 0), "wait");
            if (k && first_kernel) k = hipok(hipEventRecord(g0, s_comp), "event");
            if (k) {
                const int16_t* y = (const int16_t*)sl.d_coef;
                mj423_frames_desc_t d = {y, y + 64ull * g.y_blocks, y + 64ull * (g.y_blocks + g.c_blocks), coef_pf,
                                         (rgb_pixel_t*)sl.d_out, px_pf, w, sl.count, w, h, MJ423_CHROMA_444,
                                         MJ423_INPUT_QUANTIZED};
                // state: chunk c reads d_state[(c+1)%2] (written by chunk c-1, or the seek seed) and writes d_state[c%2]
                const int16_t* st_in = sl.types[0] != 0 ? (const int16_t*)d_state[(c + 1) % 2] : nullptr;
                if (int r = mj423_decode_stream_device(ctx, &d, sl.types, st_in, (int16_t*)d_state[c % 2])) {
                    rc = r;
                    k = false;
                }
            }
            first_kernel = false;
            k = k && hipok(hipEventRecord(sl.decoded, s_comp), "event") && hipok(hipEventRecord(g1, s_comp), "event") &&
                hipok(hipStreamWaitEvent(s_out, sl.decoded, 0), "wait") &&
                hipok(hipMemcpyAsync(sl.h_out, sl.d_out, (size_t)sl.count * px_pf * 4, hipMemcpyDeviceToHost, s_out),
                      "D2H") &&
                hipok(hipEventRecord(sl.downloaded, s_out), "event");
            std::lock_guard<std::mutex> lk(mu);
            if (!k) {
                stop.store(true);
                cv.notify_all();
                break;
            }
            sl.state = Slot::SUBMITTED;
            cv.notify_all();
        }
        tf.join();
        tb.join();
        if (rc == 0 && err.set.load()) rc = mj423_set_error(err.code, err.msg);
        (void)hipStreamSynchronize(s_in);
        (void)hipStreamSynchronize(s_comp);
        (void)hipStreamSynchronize(s_out);
        if (rc == 0 && hipEventElapsedTime(&gpu_ms, g0, g1) != hipSuccess) gpu_ms = 0.f;
    }
    if (g0) (void)hipEventDestroy(g0);
    if (g1) (void)hipEventDestroy(g1);
    for (Slot& sl : slots) {
        if (sl.h_coef) (void)hipHostFree(sl.h_coef);
        if (sl.h_out) (void)hipHostFree(sl.h_out);
        if (sl.d_coef) (void)hipFree(sl.d_coef);
        if (sl.d_out) (void)hipFree(sl.d_out);
        if (sl.uploaded) (void)hipEventDestroy(sl.uploaded);
        if (sl.decoded) (void)hipEventDestroy(sl.decoded);
        if (sl.downloaded) (void)hipEventDestroy(sl.downloaded);
        delete[] sl.types;
    }
    if (d_state[0]) (void)hipFree(d_state[0]);
    if (d_state[1]) (void)hipFree(d_state[1]);
    if (s_in) (void)hipStreamDestroy(s_in);
    if (s_out) (void)hipStreamDestroy(s_out);
    if (prev_dev >= 0) (void)hipSetDevice(prev_dev);
    if (stats && rc == 0) {
        stats->frames = count;
        stats->chunks = nchunks;
        stats->wall_s = secs(t_start, clk::now());
        stats->frontend_busy_s = fe_busy;
        stats->sink_busy_s = sink_busy;
        stats->gpu_span_ms = gpu_ms;
    }
    return rc;
}
