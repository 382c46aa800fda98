// mj423_dropin.cpp -- the reference's per-block symbols, idct() and ycbcr_to_rgb()
// (mj/decoder/mjpeg423_decoder.h:15-16; idct.c:22, ycbcr_to_rgb.c:26), served by the GPU.
//
// One 8x8 block per call (mjpeg423_decoder.c:114-124) is a latency problem, not a
// bandwidth one, so there are two ways to serve a call:
//
//  * deferred: both symbols only record the call -- idct() copies its 128 coefficient bytes
//    into this thread's page-locked queue, ycbcr_to_rgb() resolves its three block pointers
//    to the queued idct() calls that write them (or copies the block when no queued call
//    does) -- and a FLUSH decodes everything queued in two launches (idct_blocks_kernel,
//    dropin_csc_kernel), then writes every colour block and BGRA pixel to the callers'
//    buffers in call order.  Flush points: encode_bmp() and lossless_decode() of this
//    library (the reference's frame loop calls one of them before it reads anything:
//    mjpeg423_decoder.c:110-132), mj423_dropin_flush(), mj423_dropin_defer(0) and a full queue.
//    Calls still queued when the thread ends are dropped and the drop is reported
//    (mj423_dropin_status() = MJ423_ESTATE, a line on stderr): by then the caller's output buffers
//    may be gone, so nothing is written into them after the caller's code has finished.
//    MJ423_DROPIN_EXIT_FLUSH=1 writes them at thread exit instead (buffers that outlive the thread);
//
//  * immediate: each call is one launch of dropin_block_kernel on page-locked, device-mapped
//    staging; the host spins on a completion word the kernel stores (~8-10 us per call, every
//    result in the caller's buffer when the call returns, as the reference's C does).
//
// Mode (MJ423_DROPIN_DEFER / mj423_dropin_defer): 0 immediate, 1 always deferred, 2 adaptive
// (the default): a thread's calls are immediate until that thread reaches one of the
// library's own flush points (lossless_decode() / encode_bmp()), which proves its frame loop
// ends in one, and deferred from then on.  So a caller that swaps in only idct.c and
// ycbcr_to_rgb.c and keeps the reference's lossless_decode and libbmp gets the reference's
// synchronous semantics, and the reference's frame loop linked against the library's
// lossless_decode or encode_bmp gets one batch per frame.
//
// The queue is per thread (no lock per call; the reference is single-threaded per core);
// the flush takes the default context's lock.  Page-locked staging comes from a process-wide
// pool and goes back to it when a thread ends.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/mj423gpu.h"
#include "../../include/mj423io.h"
#include "mj423_internal.h"
#include "mj423_kernels.h"

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

// ------------------------------------------------------------------ status
std::mutex g_status_mu;
int g_status = MJ423_OK;  // sticky first failure (mj423_dropin_status)
std::string g_status_msg;

int drop_fail(int code, const std::string& msg) {
    mj423_set_error(code, "per-block symbols: " + msg);
    std::lock_guard<std::mutex> lk(g_status_mu);
    if (g_status == MJ423_OK) {
        g_status = code;
        g_status_msg = "per-block symbols: " + msg;
    }
    return code;
}

std::atomic<int> g_defer{-1};  // -1: not yet read from MJ423_DROPIN_DEFER; 0 / 1 / 2 (see the file comment)
thread_local bool tl_armed = false;  // this thread has reached a library flush point (adaptive mode)
std::atomic<bool> g_noticed{false};

int defer_mode() {
    int d = g_defer.load(std::memory_order_relaxed);
    if (d < 0) {
        const char* v = getenv("MJ423_DROPIN_DEFER");
        const int want = v && *v ? std::min(2, std::max(0, atoi(v))) : 2;  // unset: adaptive
        g_defer.compare_exchange_strong(d, want);
        d = g_defer.load(std::memory_order_relaxed);
    }
    return d;
}

bool deferring() {
    const int d = defer_mode();
    return d == 1 || (d == 2 && tl_armed);
}

// Adaptive mode engages on a thread: say once per process what that means.
void arm_thread() {
    if (tl_armed) return;
    tl_armed = true;
    const char* v = getenv("MJ423_DROPIN_DEFER");
    if (defer_mode() == 2 && !(v && *v) && !g_noticed.exchange(true))
        fputs("libmj423gpu: this thread reached the library's lossless_decode()/encode_bmp(): its later "
              "idct()/ycbcr_to_rgb() calls are deferred, their outputs written at its next such call or "
              "mj423_dropin_flush() (the reference decoder's frame loop reaches one before it reads them).  "
              "MJ423_DROPIN_DEFER=0 keeps every call synchronous (one GPU launch per call).\n",
              stderr);
}

// ------------------------------------------------- page-locked staging pool
struct Pinned {
    uint8_t* p = nullptr;
    size_t cap = 0;
};
std::mutex g_pool_mu;
std::vector<Pinned> g_pool;  // free page-locked buffers (never returned to the driver)

int pool_get(size_t bytes, Pinned* out) {
    {
        std::lock_guard<std::mutex> lk(g_pool_mu);
        size_t best = g_pool.size();
        for (size_t i = 0; i < g_pool.size(); i++)
            if (g_pool[i].cap >= bytes && (best == g_pool.size() || g_pool[i].cap < g_pool[best].cap)) best = i;
        if (best < g_pool.size()) {
            *out = g_pool[best];
            g_pool.erase(g_pool.begin() + (long)best);
            return 0;
        }
    }
    void* p = nullptr;
    hipError_t e = hipHostMalloc(&p, bytes, hipHostMallocDefault);
    if (e != hipSuccess) return drop_fail(MJ423_ENOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
    out->p = (uint8_t*)p;
    out->cap = bytes;
    return 0;
}
void pool_put(Pinned& b) {
    if (!b.p) return;
    std::lock_guard<std::mutex> lk(g_pool_mu);
    g_pool.push_back(b);
    b = Pinned{};
}
// Grows b to hold `need` bytes, keeping its first `used` bytes.
int pool_grow(Pinned& b, size_t need, size_t used) {
    if (need <= b.cap) return 0;
    Pinned n;
    if (int rc = pool_get(std::max(need, std::max<size_t>(2 * b.cap, 64 * 1024)), &n)) return rc;
    if (used) std::memcpy(n.p, b.p, used);
    pool_put(b);
    b = n;
    return 0;
}

// -------------------------------------------------------- deferred queue
constexpr uint32_t kLit = 0x80000000u;        // slot flag: a copied (literal) colour block
constexpr uint32_t kMaxBlocks = 1u << 20;     // queued idct() calls before a forced flush (128 MiB)
constexpr size_t kMaxRuns = 256;              // destination runs searched per lookup
constexpr size_t kMaxRegions = 16;            // distinct (rgb, w_size) outputs per flush

struct Queue {
    Queue() {
        // Thread-local objects are destroyed in the reverse order of their construction, and the
        // thread-exit flush below calls HIP (whose per-thread state is thread_local too) and may
        // record an error (mj423_last_error's text is thread_local): touch both first, so both
        // are constructed before this queue and destroyed after it.
        int d = 0;
        (void)hipGetDevice(&d);
        (void)mj423_last_error();
    }
    Pinned coef;  // 128 B of coefficients per queued idct() call
    uint32_t n = 0;
    struct Run {                // consecutive calls writing consecutive blocks (the reference's plane loops)
        uint8_t* base;
        uint32_t slot0, count;
    };
    std::vector<Run> runs;
    Pinned lit;  // 64-B colour blocks copied by ycbcr_to_rgb() (no queued idct() writes them)
    uint32_t nlit = 0;
    struct Call {
        uint32_t sy, scb, scr, region;
        int32_t h, w;
    };
    std::vector<Call> calls;
    struct Region {  // one caller frame: all calls share (rgb, w_size) and an 8x8 grid phase
        rgb_pixel_t* rgb;
        uint32_t w_size;
        int32_t ah, aw;          // anchor (first call): every call is at (ah + 8i, aw + 8j)
        int32_t h0, h1, w0, w1;  // bounding box of the calls, pixels
    };
    std::vector<Region> regions;
    uint32_t cur_region = 0;
    ~Queue();  // thread exit: pending calls dropped and reported (or written, MJ423_DROPIN_EXIT_FLUSH=1), staging back to the pool
    bool empty() const { return n == 0 && calls.empty(); }
    void clear() {
        n = 0;
        nlit = 0;
        runs.clear();
        calls.clear();
        regions.clear();
        cur_region = 0;
    }
};
thread_local Queue tq;

// Process-wide flush resources (under the default context's lock).
struct Flush {
    void* d_in = nullptr;
    size_t d_in_cap = 0;
    void* d_col = nullptr;
    size_t d_col_cap = 0;
    void* d_rgb = nullptr;
    size_t d_rgb_cap = 0;
    void* d_calls = nullptr;
    size_t d_calls_cap = 0;
    Pinned calls_h, col_h, rgb_h;
};
Flush g_fl;

int dev_ensure(void** p, size_t* cap, size_t bytes) {
    if (bytes <= *cap) return 0;
    const size_t want = std::max(bytes, std::max<size_t>(2 * *cap, 1u << 20));
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    hipError_t e = hipMalloc(p, want);
    if (e != hipSuccess) {
        *p = nullptr;
        return drop_fail(MJ423_ENOMEM, std::string("hipMalloc: ") + hipGetErrorString(e));
    }
    *cap = want;
    return 0;
}

#define DROP_HIP(expr, what)                                                                    \
    do {                                                                                        \
        hipError_t e_ = (expr);                                                                 \
        if (e_ != hipSuccess) return drop_fail(MJ423_EHIP, std::string(what) + ": " + hipGetErrorString(e_)); \
    } while (0)

// Decodes this thread's queue and writes every result to the callers' buffers.  The queue
// is empty afterwards, whether it succeeded or not (a failure is recorded, nothing is
// half-written).
int flush_queue(Queue& q) {
    if (q.empty()) return 0;
    struct Clear {
        Queue& q;
        ~Clear() { q.clear(); }
    } clear_on_exit{q};
    mj423_ctx* c = mj423_default_ctx();
    if (!c) return drop_fail(MJ423_EHIP, "no HIP device (the library has no CPU fallback); queued calls dropped");
    std::lock_guard<std::mutex> lk(mj423_default_mutex());
    DeviceGuard dg(mj423_ctx_device_id(c));
    hipStream_t s = (hipStream_t)mj423_ctx_stream(c);
    const uint32_t n = q.n, nl = q.nlit;

    // Output layout: each region's bounding box, row pitch = its width, back to back in d_rgb;
    // within a region the LAST call per 8x8 cell wins (the order the reference would write).
    std::vector<size_t> roff(q.regions.size() + 1, 0);
    std::vector<std::vector<int32_t>> win(q.regions.size());
    for (size_t r = 0; r < q.regions.size(); r++) {
        const Queue::Region& R = q.regions[r];
        const size_t gh = (size_t)(R.h1 - R.h0) / 8, gw = (size_t)(R.w1 - R.w0) / 8;
        win[r].assign(gh * gw, -1);
        roff[r + 1] = roff[r] + gh * gw * 64;
    }
    for (size_t i = 0; i < q.calls.size(); i++) {
        const Queue::Call& k = q.calls[i];
        const Queue::Region& R = q.regions[k.region];
        const size_t gw = (size_t)(R.w1 - R.w0) / 8;
        win[k.region][(size_t)((k.h - R.h0) / 8) * gw + (size_t)((k.w - R.w0) / 8)] = (int32_t)i;
    }
    size_t m = 0;
    for (auto& v : win)
        for (int32_t i : v) m += i >= 0;
    const size_t rec_b = m * sizeof(mj423::DropinCsc);
    if (int rc = pool_grow(g_fl.calls_h, rec_b, 0)) return rc;
    auto* rec = reinterpret_cast<mj423::DropinCsc*>(g_fl.calls_h.p);
    auto slot = [&](uint32_t v) { return v & kLit ? n + (v & ~kLit) : v; };
    size_t j = 0;
    for (size_t r = 0; r < q.regions.size(); r++) {
        const Queue::Region& R = q.regions[r];
        const uint32_t rp = (uint32_t)(R.w1 - R.w0);
        for (int32_t i : win[r]) {
            if (i < 0) continue;
            const Queue::Call& k = q.calls[(size_t)i];
            rec[j++] = mj423::DropinCsc{slot(k.sy), slot(k.scb), slot(k.scr), rp,
                                        roff[r] + (uint64_t)(k.h - R.h0) * rp + (uint64_t)(k.w - R.w0), 0};
        }
    }
    const size_t px = roff.back();
    if (int rc = dev_ensure(&g_fl.d_in, &g_fl.d_in_cap, (size_t)n * 128 + 16)) return rc;
    if (int rc = dev_ensure(&g_fl.d_col, &g_fl.d_col_cap, (size_t)(n + nl) * 64 + 16)) return rc;
    if (int rc = dev_ensure(&g_fl.d_rgb, &g_fl.d_rgb_cap, px * 4 + 16)) return rc;
    if (int rc = dev_ensure(&g_fl.d_calls, &g_fl.d_calls_cap, rec_b + 16)) return rc;
    if (int rc = pool_grow(g_fl.col_h, (size_t)n * 64, 0)) return rc;
    if (int rc = pool_grow(g_fl.rgb_h, px * 4, 0)) return rc;
    if (n) DROP_HIP(hipMemcpyAsync(g_fl.d_in, q.coef.p, (size_t)n * 128, hipMemcpyHostToDevice, s), "coefficient upload");
    if (nl)
        DROP_HIP(hipMemcpyAsync((uint8_t*)g_fl.d_col + (size_t)n * 64, q.lit.p, (size_t)nl * 64, hipMemcpyHostToDevice, s),
                 "block upload");
    if (m) DROP_HIP(hipMemcpyAsync(g_fl.d_calls, rec, rec_b, hipMemcpyHostToDevice, s), "call table upload");
    DROP_HIP(mj423_launch_idct_blocks((const int16_t*)g_fl.d_in, (uint8_t*)g_fl.d_col, n, nullptr, s), "idct launch");
    DROP_HIP(mj423_launch_dropin_csc((const uint8_t*)g_fl.d_col, (const mj423::DropinCsc*)g_fl.d_calls, (uint32_t)m,
                                     (uint32_t*)g_fl.d_rgb, s),
             "ycbcr_to_rgb launch");
    if (n) DROP_HIP(hipMemcpyAsync(g_fl.col_h.p, g_fl.d_col, (size_t)n * 64, hipMemcpyDeviceToHost, s), "block download");
    if (px) DROP_HIP(hipMemcpyAsync(g_fl.rgb_h.p, g_fl.d_rgb, px * 4, hipMemcpyDeviceToHost, s), "pixel download");
    DROP_HIP(hipStreamSynchronize(s), "deferred batch");

    // Colour blocks, in call order (a block written twice ends with the later result).
    for (const Queue::Run& r : q.runs) std::memcpy(r.base, g_fl.col_h.p + (size_t)r.slot0 * 64, (size_t)r.count * 64);
    // Pixels: whole rows where a region's grid is fully covered, else cell by cell.
    const uint32_t* src = reinterpret_cast<const uint32_t*>(g_fl.rgb_h.p);
    for (size_t r = 0; r < q.regions.size(); r++) {
        const Queue::Region& R = q.regions[r];
        const size_t gw = (size_t)(R.w1 - R.w0) / 8, rp = (size_t)(R.w1 - R.w0);
        const bool full = std::find(win[r].begin(), win[r].end(), -1) == win[r].end();
        const uint32_t* b = src + roff[r];
        if (full) {
            for (int32_t y = R.h0; y < R.h1; y++)
                std::memcpy(R.rgb + (ptrdiff_t)y * R.w_size + R.w0, b + (size_t)(y - R.h0) * rp, rp * 4);
            continue;
        }
        for (size_t cell = 0; cell < win[r].size(); cell++) {
            if (win[r][cell] < 0) continue;
            const int32_t h = R.h0 + (int32_t)(cell / gw) * 8, w = R.w0 + (int32_t)(cell % gw) * 8;
            for (int32_t y = 0; y < 8; y++)
                std::memcpy(R.rgb + (ptrdiff_t)(h + y) * R.w_size + w, b + (size_t)(h + y - R.h0) * rp + (size_t)(w - R.w0),
                            32);
        }
    }
    return 0;
}

Queue::~Queue() {
    // A thread that ends with queued calls reached no flush point after them.  Its output buffers
    // may already be freed (a caller's frame buffer often dies with the thread's last stack frame or
    // just before the thread returns), so the calls are dropped, never written after the fact, and the
    // drop is reported -- unless MJ423_DROPIN_EXIT_FLUSH=1 says the buffers outlive the thread.
    if (!empty()) {
        const char* v = getenv("MJ423_DROPIN_EXIT_FLUSH");
        if (v && atoi(v) == 1) {
            (void)flush_queue(*this);  // a failure is recorded in mj423_dropin_status() like any flush's
        } else {
            const std::string msg = std::to_string(n) + " idct() and " + std::to_string(calls.size()) +
                                    " ycbcr_to_rgb() calls still queued at thread exit were dropped (no flush point "
                                    "after them: call mj423_dropin_flush() before the thread ends, or set "
                                    "MJ423_DROPIN_EXIT_FLUSH=1 if their output buffers outlive the thread)";
            fprintf(stderr, "libmj423gpu: %s\n", msg.c_str());
            (void)drop_fail(MJ423_ESTATE, msg);
            clear();
        }
    }
    pool_put(coef);
    pool_put(lit);
}

// True if the 64 bytes at p overlap a queued destination block without being exactly one
// (their bytes are not known until a flush).  Every run is checked, not only the latest one
// containing p: a later run that starts inside p's block overwrites part of it, so the slot
// resolve() would pick is not the whole story.  (The reference's plane loops make about
// three runs per frame.)
bool straddles(const Queue& q, const uint8_t* p) {
    const uintptr_t a = (uintptr_t)p;
    for (const Queue::Run& r : q.runs) {
        const uintptr_t b = (uintptr_t)r.base, e = b + (uintptr_t)r.count * 64;
        if (a + 64 <= b || a >= e) continue;  // disjoint
        if ((a - b) % 64 != 0) return true;   // (mod 2^64, then mod 64: the true offset's residue)
    }
    return false;
}

// Slot of the queued idct() call that last wrote `p` (the latest run first), or kLit|i
// after copying the block when none did; -1 after a failure.
int64_t resolve(Queue& q, const uint8_t* p) {
    for (size_t i = q.runs.size(); i-- > 0;) {
        const Queue::Run& r = q.runs[i];
        const uintptr_t d = (uintptr_t)p - (uintptr_t)r.base;
        if (d < (uintptr_t)r.count * 64) return r.slot0 + (uint32_t)(d / 64);  // d % 64 == 0: straddles() ran
    }
    if (pool_grow(q.lit, ((size_t)q.nlit + 1) * 64, (size_t)q.nlit * 64)) return -1;
    std::memcpy(q.lit.p + (size_t)q.nlit * 64, p, 64);
    return (int64_t)(kLit | q.nlit++);
}

// True if the 8x8 block this ycbcr_to_rgb() call writes shares bytes with the pixel span of a
// queued region other than `self` (a region's span: its bounding box's first to last pixel,
// rows included, so the test is conservative -- a false positive only costs a flush).
bool overlaps_other_region(const Queue& q, uint32_t self, int h, int w, uint32_t w_size, const rgb_pixel_t* rgb) {
    const uintptr_t a0 = (uintptr_t)(rgb + (ptrdiff_t)h * w_size + w);
    const uintptr_t a1 = (uintptr_t)(rgb + (ptrdiff_t)(h + 7) * w_size + w + 8);
    for (uint32_t i = 0; i < q.regions.size(); i++) {
        if (i == self) continue;
        const Queue::Region& R = q.regions[i];
        const uintptr_t b0 = (uintptr_t)(R.rgb + (ptrdiff_t)R.h0 * R.w_size + R.w0);
        const uintptr_t b1 = (uintptr_t)(R.rgb + (ptrdiff_t)(R.h1 - 1) * R.w_size + R.w1);
        if (a0 < b1 && b0 < a1) return true;
    }
    return false;
}

// ----------------------------------------------------- immediate mode
struct Immediate {
    uint8_t* in_h = nullptr;  // one block triple / DCAC block + its result, host-mapped
    uint8_t* in_d = nullptr;
    uint32_t* done_h = nullptr;  // completion word
    uint32_t* done_d = nullptr;
    uint32_t seq = 0;
};
Immediate g_imm;  // under the default context's lock

int map_alloc(void** host, void** dev, size_t bytes) {
    hipError_t e = hipHostMalloc(host, bytes, hipHostMallocMapped | hipHostMallocCoherent);  // read/written by kernels
    if (e != hipSuccess) return drop_fail(MJ423_ENOMEM, std::string("hipHostMalloc: ") + hipGetErrorString(e));
    e = hipHostGetDevicePointer(dev, *host, 0);
    if (e != hipSuccess) return drop_fail(MJ423_EHIP, std::string("hipHostGetDevicePointer: ") + hipGetErrorString(e));
    return 0;
}

// One block through dropin_block_kernel (op 0 idct, 1 ycbcr_to_rgb) on g_imm.in_h; waits by
// spinning on the completion word (a stream synchronisation costs ~10 us, more than the
// launch).  After ~50 ms without the word the stream is synchronised instead, which reports
// a failed kernel.  Caller holds the default context's lock.
int run_one(mj423_ctx* c, int op) {
    if (!g_imm.in_h && map_alloc((void**)&g_imm.in_h, (void**)&g_imm.in_d, 512)) return MJ423_ENOMEM;
    if (!g_imm.done_h && map_alloc((void**)&g_imm.done_h, (void**)&g_imm.done_d, 64)) return MJ423_ENOMEM;
    hipStream_t s = (hipStream_t)mj423_ctx_stream(c);
    const uint32_t seq = ++g_imm.seq;
    const uint8_t* in = g_imm.in_d;
    uint8_t* out = g_imm.in_d + 192;  // idct: 128 B in, 64 B out; ycbcr: 3 x 64 B in, 256 B out
    hipError_t e = mj423_launch_dropin_block(op, in, out, g_imm.done_d, seq, s);
    if (e != hipSuccess) return drop_fail(MJ423_EHIP, std::string("block kernel launch: ") + hipGetErrorString(e));
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t i = 0; __atomic_load_n(g_imm.done_h, __ATOMIC_ACQUIRE) != seq; i++) {
        if ((i & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(50)) {
            e = hipStreamSynchronize(s);
            if (e != hipSuccess) return drop_fail(MJ423_EHIP, std::string("block kernel: ") + hipGetErrorString(e));
            if (__atomic_load_n(g_imm.done_h, __ATOMIC_ACQUIRE) != seq)
                return drop_fail(MJ423_EHIP, "block kernel finished without signalling completion");
            break;
        }
    }
    return 0;
}

void ycbcr_immediate(int h, int w, uint32_t w_size, const uint8_t* Y, const uint8_t* Cb, const uint8_t* Cr,
                     rgb_pixel_t* rgb) {
    mj423_ctx* c = mj423_default_ctx();
    if (!c) return (void)drop_fail(MJ423_EHIP, "no HIP device (the library has no CPU fallback)");
    std::lock_guard<std::mutex> lk(mj423_default_mutex());
    DeviceGuard dg(mj423_ctx_device_id(c));
    if (!g_imm.in_h && map_alloc((void**)&g_imm.in_h, (void**)&g_imm.in_d, 512)) return;
    std::memcpy(g_imm.in_h, Y, 64);
    std::memcpy(g_imm.in_h + 64, Cb, 64);
    std::memcpy(g_imm.in_h + 128, Cr, 64);
    if (run_one(c, 1)) return;
    const rgb_pixel_t* px = (const rgb_pixel_t*)(g_imm.in_h + 192);
    for (int y = 0; y < 8; y++)
        std::memcpy(rgb + (ptrdiff_t)(h + y) * w_size + w, px + 8 * y, 8 * sizeof(rgb_pixel_t));
}

}  // namespace

// Flush point for the library's own encode_bmp() / lossless_decode() (mj423_io.cpp).
void mj423_dropin_flush_point() {
    arm_thread();
    if (!tq.empty()) (void)flush_queue(tq);
}

extern "C" {

void idct(dct_block_t DCAC, color_block_t block) {
    if (!DCAC || !block) return (void)drop_fail(MJ423_EINVAL, "null buffer");
    if (deferring()) {
        Queue& q = tq;
        // the first call of a batch checks for the device, so a machine without one fails here
        // (outputs untouched) rather than at the flush
        if (q.empty() && !mj423_default_ctx())
            return (void)drop_fail(MJ423_EHIP, "no HIP device (the library has no CPU fallback)");
        if (q.n == kMaxBlocks && flush_queue(q)) return;
        if (pool_grow(q.coef, ((size_t)q.n + 1) * 128, (size_t)q.n * 128)) return;
        std::memcpy(q.coef.p + (size_t)q.n * 128, &DCAC[0][0], 128);
        uint8_t* d = &block[0][0];
        if (!q.runs.empty() && q.runs.back().base + (size_t)q.runs.back().count * 64 == d)
            q.runs.back().count++;
        else
            q.runs.push_back(Queue::Run{d, q.n, 1});
        q.n++;
        if (q.runs.size() > kMaxRuns) (void)flush_queue(q);  // keeps every lookup short
        return;
    }
    if (!tq.empty() && flush_queue(tq)) return;  // deferral was switched off by another thread
    mj423_ctx* c = mj423_default_ctx();
    if (!c) return (void)drop_fail(MJ423_EHIP, "no HIP device (the library has no CPU fallback)");
    std::lock_guard<std::mutex> lk(mj423_default_mutex());
    DeviceGuard dg(mj423_ctx_device_id(c));
    if (!g_imm.in_h && map_alloc((void**)&g_imm.in_h, (void**)&g_imm.in_d, 512)) return;
    std::memcpy(g_imm.in_h, &DCAC[0][0], 128);
    if (run_one(c, 0)) return;
    std::memcpy(&block[0][0], g_imm.in_h + 192, 64);
}

void ycbcr_to_rgb(int h, int w, uint32_t w_size, pcolor_block_t Y, pcolor_block_t Cb, pcolor_block_t Cr,
                  rgb_pixel_t* rgbblock) {
    if (!Y || !Cb || !Cr || !rgbblock) return (void)drop_fail(MJ423_EINVAL, "null buffer");
    const uint8_t *y = &Y[0][0], *cb = &Cb[0][0], *cr = &Cr[0][0];
    Queue& q = tq;
    if (!deferring()) {
        if (!q.empty() && flush_queue(q)) return;
        return ycbcr_immediate(h, w, w_size, y, cb, cr, rgbblock);
    }
    if (q.empty() && !mj423_default_ctx())
        return (void)drop_fail(MJ423_EHIP, "no HIP device (the library has no CPU fallback)");
    if (straddles(q, y) || straddles(q, cb) || straddles(q, cr)) {
        if (flush_queue(q)) return;  // the blocks it reads are in the callers' buffers now
    }
    uint32_t r = q.cur_region;
    if (r >= q.regions.size() || q.regions[r].rgb != rgbblock || q.regions[r].w_size != w_size) {
        for (r = 0; r < q.regions.size(); r++)
            if (q.regions[r].rgb == rgbblock && q.regions[r].w_size == w_size) break;
        if (r == q.regions.size() && q.regions.size() == kMaxRegions) {
            if (flush_queue(q)) return;
            r = 0;
        }
    }
    if (r < q.regions.size()) {
        const Queue::Region& R = q.regions[r];
        const int64_t bh = (int64_t)std::max(R.h1, h + 8) - std::min(R.h0, h);
        const int64_t bw = (int64_t)std::max(R.w1, w + 8) - std::min(R.w0, w);
        if (((h - R.ah) & 7) || ((w - R.aw) & 7)) {
            // off the region's 8x8 grid (the reference's calls never are): keep the call order
            // by decoding everything queued, then this block on its own
            if (flush_queue(q)) return;
            return ycbcr_immediate(h, w, w_size, y, cb, cr, rgbblock);
        }
        if (bh * bw > ((int64_t)1 << 28)) {  // a bounding box beyond 1 GiB of pixels: decode what is queued first
            if (flush_queue(q)) return;
            r = 0;
        }
    }
    if (overlaps_other_region(q, r, h, w, w_size, rgbblock)) {
        // pixels of another queued region share these bytes (the same buffer under another
        // w_size, or frames inside one allocation): the flush writes region by region, so
        // keep the call order by decoding what is queued first
        if (flush_queue(q)) return;
        r = 0;
    }
    const int64_t sy = resolve(q, y), scb = sy < 0 ? -1 : resolve(q, cb), scr = scb < 0 ? -1 : resolve(q, cr);
    if (scr < 0) return;
    if (r >= q.regions.size()) {
        r = (uint32_t)q.regions.size();
        q.regions.push_back(Queue::Region{rgbblock, w_size, h, w, h, h + 8, w, w + 8});
    }
    q.cur_region = r;
    Queue::Region& R = q.regions[r];
    R.h0 = std::min(R.h0, h);
    R.h1 = std::max(R.h1, h + 8);
    R.w0 = std::min(R.w0, w);
    R.w1 = std::max(R.w1, w + 8);
    q.calls.push_back(Queue::Call{(uint32_t)sy, (uint32_t)scb, (uint32_t)scr, r, h, w});
}

int mj423_dropin_defer(int on) {
    const int prev = defer_mode();
    g_defer.store(on <= 0 ? 0 : on >= 2 ? 2 : 1, std::memory_order_relaxed);
    if (!deferring() && !tq.empty()) {
        int st = flush_queue(tq);
        if (st) return st;
    }
    return prev;
}

int mj423_dropin_flush(void) { return tq.empty() ? MJ423_OK : flush_queue(tq); }

int mj423_dropin_status(void) {
    std::lock_guard<std::mutex> lk(g_status_mu);
    const int st = g_status;
    if (st != MJ423_OK) mj423_set_error(st, g_status_msg);
    g_status = MJ423_OK;
    g_status_msg.clear();
    return st;
}

}  // extern "C"
