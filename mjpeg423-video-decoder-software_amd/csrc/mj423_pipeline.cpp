// mj423_pipeline.cpp -- streaming .mpg decoder (include/mj423io.h, mj423_pipeline_*):
// the reference's per-frame loop (mjpeg423_decoder.c:88-141: read frame,
// lossless_decode x3, IDCT + CSC, write BMP) restructured as a pipeline over chunks of
// frames so that every stage runs at the same time on its own resource:
//
//   front end (host thread pool)  ->  H2D (copy stream)  ->  stream-decode kernel
//   (context stream)  ->  D2H (copy stream)  ->  sink (caller's callback, own thread)
//
// Chunks travel through a ring of slots (pinned host + device buffers) allocated once
// per pipeline object.  What crosses PCIe is the SPARSE form of each (frame, plane):
// per-block counts + one 4-byte entry per coefficient the bitstream sets (a plane falls
// back to its dense int16 form when that is smaller); expand_kernel rebuilds the dense
// planes in HBM.  For typical content this is ~10x fewer bytes than dense planes, and
// the front end writes only what it decodes.  The front end emits per-frame deltas (every (frame, plane)
// bitstream independent, so all of a chunk's planes decode in parallel); the GPU keeps
// the accumulated P-frame coefficients on chip within a chunk and hands them to the
// next chunk through a device state buffer (state_out -> state_in), so a GOP may span
// chunk boundaries with no host-side accumulation.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mj423io.h"
#include "mj423_internal.h"
#include "mj423_kernels.h"

namespace {

using clk = std::chrono::steady_clock;
double secs(clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); }

// Fixed pool: run(n, fn) calls fn(i) for i in [0, n) on the workers and the caller.
class Pool {
  public:
    explicit Pool(int nthreads) {
        for (int i = 1; i < nthreads; i++) workers_.emplace_back([this] { loop(); });
    }
    ~Pool() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            quit_ = true;
        }
        cv_.notify_all();
        for (auto& t : workers_) t.join();
    }
    void run(size_t n, const std::function<void(size_t)>& fn) {
        {
            std::lock_guard<std::mutex> lk(mu_);
            fn_ = &fn;
            n_ = n;
            next_.store(0);
            active_ = (int)workers_.size();
            gen_++;
        }
        cv_.notify_all();
        drain();
        std::unique_lock<std::mutex> lk(mu_);
        done_.wait(lk, [&] { return active_ == 0; });
        fn_ = nullptr;
    }

  private:
    void drain() {
        for (size_t i; (i = next_.fetch_add(1)) < n_;) (*fn_)(i);
    }
    void loop() {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [&] { return quit_ || gen_ != seen; });
                if (quit_) return;
                seen = gen_;
            }
            drain();
            std::lock_guard<std::mutex> lk(mu_);
            if (--active_ == 0) done_.notify_all();
        }
    }
    std::vector<std::thread> workers_;
    std::mutex mu_;
    std::condition_variable cv_, done_;
    const std::function<void(size_t)>* fn_ = nullptr;
    size_t n_ = 0;
    std::atomic<size_t> next_{0};
    int active_ = 0;
    uint64_t gen_ = 0;
    bool quit_ = false;
};

struct Slot {
    uint8_t* h_xfer = nullptr;     // pinned: front-end output (transfer layout, mj423_kernels.h ExpandParams)
    void* d_xfer = nullptr;
    uint64_t xfer_cap = 0;         // bytes of h_xfer and d_xfer
    uint64_t words = 0;            // entry words used in this chunk
    uint8_t* types = nullptr;      // host: frame types of the chunk
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
    void put(int c, const std::string& m) {
        std::lock_guard<std::mutex> lk(mu);
        if (code == 0) {
            code = c;
            msg = m;
            set.store(true);
        }
    }
};

struct DeviceScope {
    int prev = -1;
    explicit DeviceScope(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        (void)hipSetDevice(dev);
    }
    ~DeviceScope() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

constexpr int kSlots = 3;

}  // namespace

struct mj423_pipeline {
    mj423_ctx* ctx = nullptr;
    int dev = 0;
    uint32_t w = 0, h = 0, chunk = 0;
    int nthreads = 1;
    mj423_geometry_t g{};
    size_t coef_pf = 0, px_pf = 0;
    hipStream_t s_in = nullptr, s_out = nullptr;
    Slot slots[kSlots];
    void* d_state[2] = {nullptr, nullptr};
    hipEvent_t g0 = nullptr, g1 = nullptr;
    // transfer layout for a full chunk (ntask = 3 * chunk)
    uint32_t nblk = 0, nseg = 0;
    uint64_t off_mode = 0, off_seg = 0, off_counts = 0, entries_off = 0, xfer_max = 0;
    Pool* pool = nullptr;
    Pool* sink_pool = nullptr;  // unordered host sink (mj423_pipeline_create_for), else null
    std::vector<int16_t> seed_host;  // seek: absolute coefficients of the frame before `first`

    ~mj423_pipeline() {
        DeviceScope ds(dev);
        if (s_in) (void)hipStreamSynchronize(s_in);
        if (s_out) (void)hipStreamSynchronize(s_out);
        if (ctx) (void)mj423_ctx_synchronize(ctx);
        for (Slot& sl : slots) {
            if (sl.h_xfer) (void)hipHostFree(sl.h_xfer);
            if (sl.d_xfer) (void)hipFree(sl.d_xfer);
            if (sl.h_out) (void)hipHostFree(sl.h_out);
            if (sl.d_coef) (void)hipFree(sl.d_coef);
            if (sl.d_out) (void)hipFree(sl.d_out);
            if (sl.uploaded) (void)hipEventDestroy(sl.uploaded);
            if (sl.decoded) (void)hipEventDestroy(sl.decoded);
            if (sl.downloaded) (void)hipEventDestroy(sl.downloaded);
            delete[] sl.types;
        }
        for (void* p : d_state)
            if (p) (void)hipFree(p);
        if (g0) (void)hipEventDestroy(g0);
        if (g1) (void)hipEventDestroy(g1);
        if (s_in) (void)hipStreamDestroy(s_in);
        if (s_out) (void)hipStreamDestroy(s_out);
        delete pool;
        delete sink_pool;
    }
};

namespace {
// Transfer bytes frames [f0, f0 + n) can need, from their bitstream sizes: per (frame, plane)
// the dense plane, or fewer words when the bitstream is short -- the walk emits at most one DC
// entry per block and each AC entry costs the stream >= 9 bits (RUN(4) SIZE(4) and >= 1
// amplitude bit, mj423_walk.hpp), and an accepted walk reads no bits past the plane's end
// (mj423_sparse_plane_task); +3 words of entry alignment per task.
uint64_t chunk_xfer_bytes(const mj423_pipeline* p, const mj423_mpg* m, uint32_t f0, uint32_t n) {
    const uint64_t dense = (uint64_t)p->nblk * 32;
    uint64_t words = 0;
    for (uint32_t i = 0; i < n; i++) {
        mj423_mpg_frame_t fr;
        if (mj423_mpg_frame(m, f0 + i, &fr) != 0) return p->xfer_max;
        for (uint64_t nb : {(uint64_t)fr.y_size, (uint64_t)fr.cb_size, (uint64_t)fr.cr_size})
            words += std::min<uint64_t>(dense, p->nblk + nb * 8 / 9) + 3;
    }
    return std::min(p->xfer_max, p->entries_off + words * 4);
}
}  // namespace

int mj423_pipeline_create_for(mj423_pipeline** out, mj423_ctx* ctx, uint32_t w, uint32_t h, uint32_t chunk_frames,
                              int nthreads, const mj423_mpg* m, uint32_t first, uint32_t frames, int sink_threads) {
    return mj423_guarded([&]() -> int {
        if (!out || !ctx) return mj423_set_error(MJ423_EINVAL, "pipeline: null argument");
        *out = nullptr;
        if (w == 0 || h == 0 || w > (1u << 20) || h > (1u << 20))
            return mj423_set_error(MJ423_EINVAL, "pipeline: frame size out of range");
        if (m && frames) {  // the sizing hint walks these frames: check the range first
            mj423_mpg_header_t hdr;
            if (int rc = mj423_mpg_header(m, &hdr)) return rc;
            if ((uint64_t)first + frames > hdr.num_frames)
                return mj423_set_error(MJ423_EINVAL, "pipeline: frame range out of range");
        }
        // the planes hold the w/8 x h/8 whole blocks; frames are w x h with a zero margin
        mj423_geometry_t g;
        if (int rc = mj423_coded_geometry_444(w, h, &g)) return rc;
        mj423_pipeline* p = new mj423_pipeline();
        p->ctx = ctx;
        p->dev = mj423_ctx_device_id(ctx);
        p->w = w;
        p->h = h;
        p->g = g;
        p->coef_pf = g.coef_per_frame;
        p->px_pf = (size_t)w * h;
        const size_t frame_bytes = p->coef_pf * 2 + p->px_pf * 4;
        // Default chunk: 48 frames (two GOPs at the reference's maximum I-interval of 24,
        // c0/common/config.h:54), at most 1 GiB of device coefficients + pixels per slot.  A chunk
        // is one stream-kernel launch of (tiles per frame) x (GOP segments in the chunk)
        // workgroups; a 12-frame chunk inside one GOP gave 1080p 4:4:4 510 workgroups, half of
        // one round of resident workgroups (4 per CU), so the launches ran at 0.43 of the HBM
        // roofline.  Two GOPs per chunk fill a round.
        // The default also fits the device memory free right now: the kSlots ring holds a chunk's
        // planes, pixels and transfer buffer per slot (plus pinned host copies), so several pipelines
        // or ranks sharing one GPU take at most a quarter of what is free each, in whole frames.
        DeviceScope ds(p->dev);
        size_t cap_bytes = 1024ull << 20;
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess && free_b > 0)
            cap_bytes = std::min(cap_bytes, free_b / 4 / kSlots / 2);  // /2: the transfer buffer ~ the planes
        const uint32_t cap = (uint32_t)std::max<size_t>(1, cap_bytes / frame_bytes);
        p->chunk = chunk_frames ? chunk_frames : std::min(48u, cap);
        // A one-shot decode of a short file: chunks of a sixth of the call, so the stages still
        // overlap and the ring holds half the call at most -- pinned host memory costs ~0.27 s per
        // GiB to allocate and free, and the default ring for 1080p took 0.9 s to create and
        // destroy, 60x the decode of 48 frames; the GPU's share of such a call is a few ms
        // whatever its fill (profiles/r04/e2e/).
        if (!chunk_frames && frames)
            p->chunk = std::min(p->chunk, std::max(1u, (frames + 2 * kSlots - 1) / (2 * kSlots)));
        p->nthreads = nthreads > 0 ? nthreads : mj423_host_threads();
        int rc = 0;
        auto ok = [&](hipError_t e, const char* what) {
            if (e != hipSuccess && rc == 0)
                rc = mj423_set_error(MJ423_EHIP, std::string("pipeline: ") + what + ": " + hipGetErrorString(e));
            return e == hipSuccess;
        };
        const size_t coef_bytes = (size_t)p->chunk * p->coef_pf * 2, out_bytes = (size_t)p->chunk * p->px_pf * 4;
        const uint64_t ntask = 3ull * p->chunk;
        p->nblk = g.y_blocks;  // 4:4:4: every plane alike
        p->nseg = (p->nblk + 255) / 256;
        p->off_mode = ntask * 4;
        p->off_seg = p->off_mode + ntask * 4;
        p->off_counts = p->off_seg + ntask * (p->nseg + 1) * 4;
        p->entries_off = (p->off_counts + ntask * p->nblk + 15) / 16 * 16;
        p->xfer_max = p->entries_off + coef_bytes + ntask * 16;  // entries never exceed the dense planes (+ alignment)
        // The transfer ring: for a known decode, what its chunks can need; else an eighth of the
        // dense bound (typical streams set far fewer coefficients, see the file comment).  The
        // decode grows a slot whose next chunk could need more (a stall of one chunk, once).
        uint64_t xfer_cap = std::min(p->xfer_max, p->entries_off + coef_bytes / 8 + ntask * 16);
        if (m && frames) {
            xfer_cap = 0;
            const uint64_t stop = (uint64_t)first + frames;  // (validated above; 64-bit: no wrap near 2^32)
            for (uint64_t f = first; f < stop; f += p->chunk)
                xfer_cap = std::max(xfer_cap, chunk_xfer_bytes(p, m, (uint32_t)f, (uint32_t)std::min<uint64_t>(p->chunk, stop - f)));
        }
        // (no block: nothing crosses PCIe and nothing is decoded, the buffers stay minimal)
        const size_t coef_alloc = std::max<size_t>(16, coef_bytes), state_alloc = std::max<size_t>(16, p->coef_pf * 2);
        xfer_cap = std::max<uint64_t>(16, xfer_cap);
        bool good = ok(hipStreamCreateWithFlags(&p->s_in, hipStreamNonBlocking), "stream") &&
                    ok(hipStreamCreateWithFlags(&p->s_out, hipStreamNonBlocking), "stream") &&
                    ok(hipMalloc(&p->d_state[0], state_alloc), "hipMalloc") &&
                    ok(hipMalloc(&p->d_state[1], state_alloc), "hipMalloc") && ok(hipEventCreate(&p->g0), "event") &&
                    ok(hipEventCreate(&p->g1), "event");
        for (int i = 0; good && i < kSlots; i++) {
            Slot& sl = p->slots[i];
            sl.xfer_cap = xfer_cap;
            good = ok(hipHostMalloc((void**)&sl.h_xfer, xfer_cap, hipHostMallocDefault), "hipHostMalloc") &&
                   ok(hipMalloc(&sl.d_xfer, xfer_cap), "hipMalloc") &&
                   ok(hipHostMalloc((void**)&sl.h_out, out_bytes, hipHostMallocDefault), "hipHostMalloc") &&
                   ok(hipMalloc(&sl.d_coef, coef_alloc), "hipMalloc") && ok(hipMalloc(&sl.d_out, out_bytes), "hipMalloc") &&
                   ok(hipEventCreateWithFlags(&sl.uploaded, hipEventDisableTiming), "event") &&
                   ok(hipEventCreateWithFlags(&sl.decoded, hipEventDisableTiming), "event") &&
                   ok(hipEventCreateWithFlags(&sl.downloaded, hipEventDisableTiming), "event");
            if (good) sl.types = new uint8_t[p->chunk];
        }
        if (!good) {
            delete p;
            return rc;
        }
        p->pool = new Pool(p->nthreads);
        if (sink_threads > 1) p->sink_pool = new Pool(sink_threads);
        *out = p;
        return 0;
    });
}

extern "C" int mj423_pipeline_create(mj423_pipeline** out, mj423_ctx* ctx, uint32_t w, uint32_t h,
                                     uint32_t chunk_frames, int nthreads) {
    return mj423_pipeline_create_for(out, ctx, w, h, chunk_frames, nthreads, nullptr, 0, 0, 1);
}

extern "C" void mj423_pipeline_destroy(mj423_pipeline* p) { delete p; }

namespace {
// Host sink (frames downloaded into pinned memory, `sink` per frame) or device sink
// (`dsink` per chunk with the frames still in HBM, no D2H).
int pipeline_run(mj423_pipeline* p, const mj423_mpg* m, uint32_t first, uint32_t count, mj423_frame_sink_fn sink,
                 mj423_device_sink_fn dsink, void* user, mj423_pipeline_stats_t* stats) {
    return mj423_guarded([&]() -> int {
        if (!p || !m || (!sink && !dsink)) return mj423_set_error(MJ423_EINVAL, "pipeline: null argument");
        mj423_mpg_header_t hdr;
        if (int rc = mj423_mpg_header(m, &hdr)) return rc;
        if (hdr.width != p->w || hdr.height != p->h)
            return mj423_set_error(MJ423_EINVAL, "pipeline: stream size differs from the pipeline's");
        if ((uint64_t)first + count > hdr.num_frames) return mj423_set_error(MJ423_EINVAL, "pipeline: frame range out of range");
        if (stats) std::memset(stats, 0, sizeof(*stats));
        if (count == 0) return 0;
        const clk::time_point t_start = clk::now();
        const uint32_t chunk = std::min(p->chunk, count);
        const uint32_t nchunks = (count + chunk - 1) / chunk;
        const size_t coef_pf = p->coef_pf, px_pf = p->px_pf;
        const mj423_geometry_t& g = p->g;
        DeviceScope ds(p->dev);
        hipStream_t s_comp = (hipStream_t)mj423_ctx_stream(p->ctx);
        int rc = 0;
        auto hipok = [&](hipError_t e, const char* what) {
            if (e != hipSuccess && rc == 0)
                rc = mj423_set_error(MJ423_EHIP, std::string("pipeline: ") + what + ": " + hipGetErrorString(e));
            return e == hipSuccess;
        };
        // Seeking into a GOP: the absolute coefficients of frame first-1 seed the GPU state
        // (d_state[1] is chunk 0's state_in).
        mj423_mpg_frame_t fr0;
        if (int r = mj423_mpg_frame(m, first, &fr0)) return r;
        if (fr0.frame_type != 0 && coef_pf) {
            p->seed_host.resize(coef_pf);
            if (int r = mj423_mpg_entropy_decode(m, first - 1, 1, p->seed_host.data(), p->nthreads)) return r;
            if (!hipok(hipMemcpyAsync(p->d_state[1], p->seed_host.data(), coef_pf * 2, hipMemcpyHostToDevice, s_comp),
                       "state upload") ||
                !hipok(hipStreamSynchronize(s_comp), "state upload"))
                return rc;
        }
        for (Slot& sl : p->slots) {
            sl.state = Slot::FREE;
            sl.seq = -1;
        }
        std::mutex mu;
        std::condition_variable cv;
        ErrBox err;
        double fe_busy = 0.0, sink_busy = 0.0;
        std::atomic<bool> stop{false};
        auto halt = [&](int code, const std::string& msg) {
            err.put(code, msg);
            std::lock_guard<std::mutex> lk(mu);
            stop.store(true);
            cv.notify_all();
        };

        // ---- front end: fills FREE slots with chunk c (slot c % kSlots), in order
        auto front = [&]() {
            (void)hipSetDevice(p->dev);
            for (uint32_t c = 0; c < nchunks && !stop.load(); c++) {
                Slot& sl = p->slots[c % kSlots];
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return stop.load() || sl.state == Slot::FREE; });
                    if (stop.load()) return;
                }
                sl.first = first + c * chunk;
                sl.count = std::min(chunk, first + count - sl.first);
                const uint64_t need = chunk_xfer_bytes(p, m, sl.first, sl.count);
                if (need > sl.xfer_cap) {  // this chunk could expand past the slot's buffers: regrow them
                    // once the GPU has expanded the slot's previous chunk (never-recorded event: no-op)
                    if (hipEventSynchronize(sl.decoded) != hipSuccess) return halt(MJ423_EHIP, "pipeline: GPU stage failed");
                    (void)hipHostFree(sl.h_xfer);
                    (void)hipFree(sl.d_xfer);
                    sl.h_xfer = nullptr;
                    sl.d_xfer = nullptr;
                    sl.xfer_cap = 0;
                    const uint64_t cap = std::min(p->xfer_max, need + need / 4);
                    if (hipHostMalloc((void**)&sl.h_xfer, cap, hipHostMallocDefault) != hipSuccess ||
                        hipMalloc(&sl.d_xfer, cap) != hipSuccess)
                        return halt(MJ423_ENOMEM, "pipeline: transfer buffer allocation failed");
                    sl.xfer_cap = cap;
                }
                const clk::time_point a = clk::now();
                std::atomic<int> bad{0};
                std::atomic<uint64_t> words{0};
                uint32_t* base = reinterpret_cast<uint32_t*>(sl.h_xfer);
                uint32_t* mode = reinterpret_cast<uint32_t*>(sl.h_xfer + p->off_mode);
                uint32_t* ent0 = reinterpret_cast<uint32_t*>(sl.h_xfer + p->entries_off);
                if (p->nblk == 0)  // no whole block: only the frame types
                    for (uint32_t i = 0; i < sl.count; i++) {
                        mj423_mpg_frame_t fr;
                        (void)mj423_mpg_frame(m, sl.first + i, &fr);
                        sl.types[i] = (uint8_t)fr.frame_type;
                    }
                p->pool->run(p->nblk ? (size_t)sl.count * 3 : 0, [&](size_t t) {
                    thread_local std::vector<uint32_t> tl;
                    if (tl.size() < (size_t)p->nblk * 64) tl.resize((size_t)p->nblk * 64);
                    const uint32_t i = (uint32_t)(t / 3);
                    const int plane = (int)(t % 3);
                    uint8_t* counts = sl.h_xfer + p->off_counts + t * p->nblk;
                    uint32_t* seg = reinterpret_cast<uint32_t*>(sl.h_xfer + p->off_seg) + t * (p->nseg + 1);
                    const long n = mj423_sparse_plane_task(m, sl.first + i, plane, counts, seg, tl.data(), sl.types + i);
                    if (n < 0) {
                        bad.store(1);
                        return;
                    }
                    const uint64_t dense_words = (uint64_t)p->nblk * 32;
                    if ((uint64_t)n < dense_words) {  // sparse: counts + entries
                        const uint64_t at = words.fetch_add(((uint64_t)n + 3) & ~3ull);
                        std::memcpy(ent0 + at, tl.data(), (size_t)n * 4);
                        base[t] = (uint32_t)at;
                        mode[t] = 0;
                    } else {  // denser than the plane itself: ship the int16 plane
                        const uint64_t at = words.fetch_add(dense_words);
                        int16_t* dst = reinterpret_cast<int16_t*>(ent0 + at);
                        mj423_mpg_frame_t fr;
                        (void)mj423_mpg_frame(m, sl.first + i, &fr);
                        const uint8_t* bs = plane == 0 ? fr.y : plane == 1 ? fr.cb : fr.cr;
                        const size_t nbs = plane == 0 ? fr.y_size : plane == 1 ? fr.cb_size : fr.cr_size;
                        if (fr.frame_type != 0) std::memset(dst, 0, dense_words * 4);
                        if (mj423_lossless_decode_q((int)p->nblk, bs, nbs, dst, fr.frame_type != 0) == (size_t)-1)
                            bad.store(1);
                        base[t] = (uint32_t)at;
                        mode[t] = 1;
                    }
                });
                sl.words = words.load();
                fe_busy += secs(a, clk::now());
                if (bad.load()) return halt(MJ423_EINVAL, "mpg: a bitstream ended before all of its blocks were decoded");
                std::lock_guard<std::mutex> lk(mu);
                sl.seq = c;
                sl.state = Slot::FILLED;
                cv.notify_all();
            }
        };
        // ---- sink: waits for chunk c's download, hands its frames to the caller in order
        auto back = [&]() {
            (void)hipSetDevice(p->dev);
            for (uint32_t c = 0; c < nchunks && !stop.load(); c++) {
                Slot& sl = p->slots[c % kSlots];
                {
                    std::unique_lock<std::mutex> lk(mu);
                    cv.wait(lk, [&] { return stop.load() || (sl.state == Slot::SUBMITTED && sl.seq == (int64_t)c); });
                    if (stop.load()) return;
                }
                if (dsink) {
                    // the pinned staging must be read by the DMA before the front end refills
                    // it; the device buffers are protected by stream order (see the submit loop)
                    if (hipEventSynchronize(sl.uploaded) != hipSuccess) return halt(MJ423_EHIP, "pipeline: GPU stage failed");
                    const clk::time_point a = clk::now();
                    if (dsink(user, sl.first, sl.count, (const rgb_pixel_t*)sl.d_out, px_pf, (void*)s_comp) != 0)
                        return halt(MJ423_EINVAL, "pipeline: frame sink reported an error");
                    sink_busy += secs(a, clk::now());
                } else {
                    if (hipEventSynchronize(sl.downloaded) != hipSuccess) return halt(MJ423_EHIP, "pipeline: GPU stage failed");
                    const clk::time_point a = clk::now();
                    if (p->sink_pool) {  // unordered: the chunk's frames on the sink pool
                        std::atomic<int> failed{0};
                        p->sink_pool->run(sl.count, [&](size_t i) {
                            if (!failed.load() &&
                                sink(user, sl.first + (uint32_t)i, sl.h_out + i * px_pf, p->w, p->h) != 0)
                                failed.store(1);
                        });
                        if (failed.load()) return halt(MJ423_EINVAL, "pipeline: frame sink reported an error");
                    } else {
                        for (uint32_t i = 0; i < sl.count; i++)
                            if (sink(user, sl.first + i, sl.h_out + (size_t)i * px_pf, p->w, p->h) != 0)
                                return halt(MJ423_EINVAL, "pipeline: frame sink reported an error");
                    }
                    sink_busy += secs(a, clk::now());
                }
                std::lock_guard<std::mutex> lk(mu);
                sl.state = Slot::FREE;
                sl.seq = -1;
                cv.notify_all();
            }
        };

        std::thread tf(front), tb(back);
        bool first_kernel = true;
        for (uint32_t c = 0; c < nchunks; c++) {  // this thread submits the GPU stages
            Slot& sl = p->slots[c % kSlots];
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop.load() || (sl.state == Slot::FILLED && sl.seq == (int64_t)c); });
                if (stop.load()) break;
            }
            // H2D of the sparse transfer on the copy-in stream; expansion + decode wait for it;
            // D2H waits for the decode.
            const size_t nb = p->entries_off + sl.words * 4;
            // d_xfer is free once this slot's previous chunk has been expanded (a device sink
            // frees slots before the GPU is done with them); a never-recorded event is a no-op
            bool k = hipok(hipStreamWaitEvent(p->s_in, sl.decoded, 0), "wait") &&
                     (p->nblk == 0 || hipok(hipMemcpyAsync(sl.d_xfer, sl.h_xfer, nb, hipMemcpyHostToDevice, p->s_in), "H2D")) &&
                     hipok(hipEventRecord(sl.uploaded, p->s_in), "event") &&
                     hipok(hipStreamWaitEvent(s_comp, sl.uploaded, 0), "wait");
            if (k && first_kernel) k = hipok(hipEventRecord(p->g0, s_comp), "event");
            first_kernel = false;
            if (k && p->nblk) {
                mj423::ExpandParams ep{};
                ep.xfer = (const uint8_t*)sl.d_xfer;
                ep.off_mode = p->off_mode;
                ep.off_seg = p->off_seg;
                ep.off_counts = p->off_counts;
                ep.entries_off = p->entries_off;
                ep.ntask = sl.count * 3;
                ep.nblk = p->nblk;
                ep.nseg = p->nseg;
                ep.out = (int16_t*)sl.d_coef;
                ep.coef_pf = coef_pf;
                k = hipok(mj423_launch_expand(&ep, s_comp), "expand kernel");
            }
            if (k && p->nblk) {  // the coded region at pitch w (the margin is filled below)
                const int16_t* y = (const int16_t*)sl.d_coef;
                mj423_frames_desc_t d = {y, y + 64ull * g.y_blocks, y + 64ull * (g.y_blocks + g.c_blocks), coef_pf,
                                         (rgb_pixel_t*)sl.d_out, px_pf, p->w, sl.count, g.width, g.height, MJ423_CHROMA_444,
                                         MJ423_INPUT_QUANTIZED};
                // state: chunk c reads d_state[(c+1)%2] (chunk c-1's end state, or the seek seed)
                // and writes d_state[c%2]
                const int16_t* st_in = sl.types[0] != 0 ? (const int16_t*)p->d_state[(c + 1) % 2] : nullptr;
                if (int r = mj423_decode_stream_device(p->ctx, &d, sl.types, st_in, (int16_t*)p->d_state[c % 2])) {
                    rc = r;
                    k = false;
                }
            }
            if (k)  // the defined fill outside the coded region (mj423_margin.hip); no-op for whole blocks
                k = hipok((hipError_t)mj423_launch_fill_margin((rgb_pixel_t*)sl.d_out, px_pf, p->w, g.width, g.height, p->w,
                                                               p->h, sl.count, s_comp),
                          "margin fill");
            k = k && hipok(hipEventRecord(sl.decoded, s_comp), "event") && hipok(hipEventRecord(p->g1, s_comp), "event");
            if (k && !dsink)
                k = hipok(hipStreamWaitEvent(p->s_out, sl.decoded, 0), "wait") &&
                    hipok(hipMemcpyAsync(sl.h_out, sl.d_out, (size_t)sl.count * px_pf * 4, hipMemcpyDeviceToHost,
                                         p->s_out),
                          "D2H") &&
                    hipok(hipEventRecord(sl.downloaded, p->s_out), "event");
            if (!k) {
                halt(rc ? rc : MJ423_EHIP, mj423_last_error());
                break;
            }
            std::lock_guard<std::mutex> lk(mu);
            sl.state = Slot::SUBMITTED;
            cv.notify_all();
        }
        tf.join();
        tb.join();
        (void)hipStreamSynchronize(p->s_in);
        (void)hipStreamSynchronize(s_comp);
        (void)hipStreamSynchronize(p->s_out);
        if (err.set.load()) return mj423_set_error(err.code, err.msg);
        if (rc) return rc;
        if (stats) {
            float gpu_ms = 0.f;
            if (hipEventElapsedTime(&gpu_ms, p->g0, p->g1) != hipSuccess) gpu_ms = 0.f;
            stats->frames = count;
            stats->chunks = nchunks;
            stats->wall_s = secs(t_start, clk::now());
            stats->frontend_busy_s = fe_busy;
            stats->sink_busy_s = sink_busy;
            stats->gpu_span_ms = gpu_ms;
        }
        return 0;
    });
}

}  // namespace

extern "C" int mj423_pipeline_decode(mj423_pipeline* p, const mj423_mpg* m, uint32_t first, uint32_t count,
                                     mj423_frame_sink_fn sink, void* user, mj423_pipeline_stats_t* stats) {
    if (!sink) return mj423_set_error(MJ423_EINVAL, "pipeline: null sink");
    return pipeline_run(p, m, first, count, sink, nullptr, user, stats);
}

extern "C" int mj423_pipeline_decode_device(mj423_pipeline* p, const mj423_mpg* m, uint32_t first, uint32_t count,
                                            mj423_device_sink_fn sink, void* user, mj423_pipeline_stats_t* stats) {
    if (!sink) return mj423_set_error(MJ423_EINVAL, "pipeline: null sink");
    return pipeline_run(p, m, first, count, nullptr, sink, user, stats);
}

extern "C" int mj423_decode_mpg_pipelined(mj423_ctx* ctx, const mj423_mpg* m, uint32_t first, uint32_t count,
                                          uint32_t chunk_frames, int nthreads, mj423_frame_sink_fn sink, void* user,
                                          mj423_pipeline_stats_t* stats) {
    return mj423_guarded([&]() -> int {
        if (!ctx || !m || !sink) return mj423_set_error(MJ423_EINVAL, "pipeline: null argument");
        mj423_mpg_header_t hdr;
        if (int rc = mj423_mpg_header(m, &hdr)) return rc;
        mj423_pipeline* p = nullptr;
        if (int rc = mj423_pipeline_create_for(&p, ctx, hdr.width, hdr.height, chunk_frames, nthreads, m, first, count, 1))
            return rc;
        const int rc = mj423_pipeline_decode(p, m, first, count, sink, user, stats);
        mj423_pipeline_destroy(p);
        return rc;
    });
}
