// mj423_gpu_frontend.cpp -- whole-GPU .mpg decode (include/mj423io.h, mj423_mpg_decode_gpu):
// the frames' bitstreams go to HBM once; the entropy front end decodes every (frame, plane)
// stream into per-frame delta planes -- by default many lanes per stream, each on a
// 64-byte subsequence found by self-synchronisation (mj423_entropy.hip); MJ423_GPU_FE=wave
// selects the one-wave-per-stream entropy_kernel -- and decode_gop_kernel accumulates the
// P-frames on chip and runs dequant + IDCT + CSC.  No coefficient crosses PCIe and no host
// thread decodes bits.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <string>
#include <vector>

#include "../../include/mj423io.h"
#include "mj423_entropy.h"
#include "mj423_internal.h"
#include "mj423_kernels.h"

// Device buffers kept by the context across calls (a whole-file decode allocates ~12 MB
// per 1080p frame; hipMalloc + hipFree of them cost ~2.5 ms per call).  Grow-only.
struct mj423_fe_cache {
    struct Buf {
        void* p = nullptr;
        size_t cap = 0;
        hipError_t ensure(size_t n) {
            if (n <= cap) return hipSuccess;
            release();
            const hipError_t e = hipMalloc(&p, n);
            if (e != hipSuccess) {
                p = nullptr;
                return e;
            }
            cap = n;
            return hipSuccess;
        }
        void release() {
            if (p) (void)hipFree(p);
            p = nullptr;
            cap = 0;
        }
    };
    Buf bytes, coef[2], tasks, status, state[2], sub0, start, exit_, nb, dcs, zrun, zlast, flags, tchg, wcnt, qbits, lane_task, bpos, tiles, meta,
        mc_list, mc_x, mc_map, mc_rec, mc_st, mc_sfx, mc_ck;
    // Host-mapped staging for the per-call tables (tasks, subsequence starts, seek seed) and
    // the status read-back, moved by a copy kernel on the context stream.  Traced passes
    // (profiles/r02/frontend): a hipMemcpyAsync of the 17 KB task table blocked the host for
    // 7.4 ms from pageable memory and 8.6 ms from page-locked memory, once in ~100 passes,
    // while the copy stream was uploading the windows' bytes -- the occasional 10 ms pass.
    void* host = nullptr;
    void* host_d = nullptr;  // its device-side address
    size_t host_cap = 0;
    hipError_t host_ensure(size_t n) {
        if (n <= host_cap) return hipSuccess;
        // grown with slack (x1.5, >= 1 MiB, whole pages): calls of growing sizes -- a seek adds the
        // seed frame -- re-allocate (free + map) page-locked memory rarely
        n = std::max<size_t>(std::max<size_t>(n + n / 2, host_cap + host_cap / 2), (size_t)1 << 20);
        n = (n + 4095) & ~(size_t)4095;
        if (host) (void)hipHostFree(host);
        host = host_d = nullptr;
        host_cap = 0;
        // coherent (fine-grained): the copy kernels read the host's fresh tables and write the
        // status straight to host memory -- no GPU-cached copy of a previous call's contents
        hipError_t e = hipHostMalloc(&host, n, hipHostMallocMapped | hipHostMallocCoherent);
        if (e == hipSuccess) e = hipHostGetDevicePointer(&host_d, host, 0);
        if (e != hipSuccess) {
            if (host) (void)hipHostFree(host);
            host = host_d = nullptr;
            return e;
        }
        host_cap = n;
        return hipSuccess;
    }
    hipStream_t copy = nullptr;     // window uploads of page-locked file bytes
    hipStream_t ent = nullptr;      // entropy kernels (the stream kernel runs on the context's stream)
    std::vector<hipEvent_t> ev;     // one per window: its bytes have arrived
    std::vector<hipEvent_t> ev_ent, ev_dec;  // per window: its planes are written / consumed
    hipEvent_t ev_setup = nullptr;  // the call's uploads on the context stream are done
    uint64_t budget = 0;            // default window budget (bytes), from the first call's free HBM
};

void mj423_fe_cache_release(mj423_fe_cache* c) {
    if (!c) return;
    if (c->copy) (void)hipStreamSynchronize(c->copy);
    if (c->ent) (void)hipStreamSynchronize(c->ent);
    for (auto* b : {&c->bytes, &c->coef[0], &c->coef[1], &c->tasks, &c->status, &c->state[0], &c->state[1], &c->sub0, &c->start,
                    &c->exit_, &c->nb, &c->dcs, &c->zrun, &c->zlast, &c->flags, &c->tchg, &c->wcnt, &c->qbits, &c->lane_task, &c->bpos, &c->tiles, &c->meta,
                    &c->mc_list, &c->mc_x, &c->mc_map, &c->mc_rec, &c->mc_st, &c->mc_sfx, &c->mc_ck})
        b->release();
    for (auto* v : {&c->ev, &c->ev_ent, &c->ev_dec})
        for (hipEvent_t e : *v) (void)hipEventDestroy(e);
    if (c->ev_setup) (void)hipEventDestroy(c->ev_setup);
    if (c->host) (void)hipHostFree(c->host);
    if (c->copy) (void)hipStreamDestroy(c->copy);
    if (c->ent) (void)hipStreamDestroy(c->ent);
    delete c;
}

namespace {
constexpr int kRetrySmaller = 1;

inline uint64_t sat_sub(uint64_t a, uint64_t b) { return a > b ? a - b : 0; }  // internal: the window buffers did not fit, budget re-measured

// Two forms after the same many-lanes synchronisation (mj423_entropy.hip):
//  * fused (default): an index pass records where every block starts, and mpg_fused_kernel
//    (mj423_fused.hip) entropy-decodes, accumulates, transforms and converts each tile's blocks
//    in one pass -- no dense coefficient plane is written or read;
//  * dense (MJ423_GPU_FE_FUSED=0 or MJ423_GPU_FE=wave): the emit pass writes dense int16 delta
//    planes per window and decode_gop_kernel reads them back (mj423_decode_stream_device).
int decode_gpu_once(mj423_ctx* ctx, const mj423_mpg* m, uint32_t first, uint32_t count, rgb_pixel_t* d_out,
                    uint64_t out_frame_stride, uint32_t window_frames, bool may_retry, bool dense) {
    // MJ423_FE_HOSTTIME=1 (diagnostic): host microseconds from entry to the first upload issued, to the
    // last launch issued, and to the return, one stderr line per call
    static const bool host_time = std::getenv("MJ423_FE_HOSTTIME") != nullptr;
    const auto t_entry = std::chrono::steady_clock::now();
    double t_upload = -1, t_launched = -1;
    auto us_since = [&]() { return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_entry).count(); };
    struct HostTimeReport {
        const bool& on;
        std::function<double()> now;
        double &up, &la;
        ~HostTimeReport() {
            if (on) std::fprintf(stderr, "mj423 hosttime: upload issued %.1f us, launches issued %.1f us, return %.1f us\n", up, la, now());
        }
    } report{host_time, us_since, t_upload, t_launched};
    {
        if (!ctx || !m || (!d_out && count)) return mj423_set_error(MJ423_EINVAL, "decode_gpu: null argument");
        mj423_mpg_header_t hdr;
        if (int rc = mj423_mpg_header(m, &hdr)) return rc;
        if ((uint64_t)first + count > hdr.num_frames) return mj423_set_error(MJ423_EINVAL, "decode_gpu: frame range out of range");
        if (count == 0) return 0;
        const uint32_t w = hdr.width, h = hdr.height;
        if (out_frame_stride < (uint64_t)w * h) return mj423_set_error(MJ423_EINVAL, "decode_gpu: out_frame_stride < w*h");
        // the planes hold the w/8 x h/8 whole blocks; frames are w x h with a zero margin
        mj423_geometry_t g;
        if (int rc = mj423_mpg_geometry(m, &g)) return rc;
        const uint64_t coef_pf = g.coef_per_frame;
        const uint32_t nblk = g.y_blocks;
        if (nblk == 0) {  // no whole block: every frame is the fill
            hipStream_t s0 = (hipStream_t)mj423_ctx_stream(ctx);
            int prev = -1;
            (void)hipGetDevice(&prev);
            if (hipSetDevice(mj423_ctx_device_id(ctx)) != hipSuccess) return mj423_set_error(MJ423_EHIP, "decode_gpu: hipSetDevice failed");
            hipError_t e = (hipError_t)mj423_launch_fill_margin(d_out, out_frame_stride, w, 0, 0, w, h, count, s0);
            if (e == hipSuccess) e = hipStreamSynchronize(s0);
            if (prev >= 0) (void)hipSetDevice(prev);
            return e == hipSuccess ? 0 : mj423_set_error(MJ423_EHIP, std::string("decode_gpu: margin fill: ") + hipGetErrorString(e));
        }
        if (nblk >= (1u << 26))  // the kernel forms plane positions 64 * block + index in 32 bits
            return mj423_set_error(MJ423_EINVAL, "decode_gpu: more than 2^26 blocks per plane");
        // Default window: as many frames as half the free HBM holds in dense delta planes (at
        // most 64 GiB).  A launch lasts as long as its longest stream (an I-frame plane), so
        // the more frames share it, the faster the batch: 1080p 4:4:4 is ~12 MB per frame,
        // so a whole file of a few thousand frames decodes in one window.
        mj423_fe_cache*& cache = *mj423_ctx_fe_cache(ctx);
        if (!cache) cache = new mj423_fe_cache();
        mj423_fe_cache& C = *cache;
        uint64_t budget = 4ull << 30;
        if (!window_frames && C.budget) {
            budget = C.budget;
        } else if (!window_frames) {  // the context's own cached staging counts as free; asked once per
            // context (hipMemGetInfo on every call showed as occasional ~7 ms stalls)
            size_t free_b = 0, total_b = 0;
            int cur = -1;
            (void)hipGetDevice(&cur);
            if (hipSetDevice(mj423_ctx_device_id(ctx)) == hipSuccess && hipMemGetInfo(&free_b, &total_b) == hipSuccess)
                budget = std::max<uint64_t>(budget, std::min<uint64_t>((free_b + C.coef[0].cap + C.coef[1].cap) / 2, 64ull << 30));
            if (cur >= 0) (void)hipSetDevice(cur);
            C.budget = budget;
        }
        const char* fe = std::getenv("MJ423_GPU_FE");
        const bool par = !(fe && std::strcmp(fe, "wave") == 0);
        const char* fz = std::getenv("MJ423_GPU_FE_FUSED");
        const bool fused = par && !dense && !(fz && std::atoi(fz) == 0);
        // the fused path stages no planes: windows only pace the upload (or follow window_frames)
        const uint32_t win = window_frames ? window_frames
                             : fused      ? 0xffffffffu
                                          : (uint32_t)std::max<uint64_t>(1, budget / (coef_pf * 4));  // two buffers
        // walks read their subsequence from a window staged in LDS (MJ423_GPU_FE_LDSWIN=0: from global memory; A/B)
        const bool lds_window = !(std::getenv("MJ423_GPU_FE_LDSWIN") && std::atoi(std::getenv("MJ423_GPU_FE_LDSWIN")) == 0);
        const bool dbg = std::getenv("MJ423_ENTPAR_DEBUG") != nullptr;
        // streams still changing after the last iteration: multi-class resolution (mj423_entropy.hip
        // entmc_*) before the serial fallback (MJ423_GPU_FE_MC=0: fallback only; A/B)
        const bool mc = !(std::getenv("MJ423_GPU_FE_MC") && std::atoi(std::getenv("MJ423_GPU_FE_MC")) == 0);
        // Page-locked file bytes upload asynchronously on a copy stream, window by window, so
        // window k decodes while window k+1 is still crossing PCIe (state crosses windows on
        // the GPU).
        // Unequal windows (weights 2 : 3 : 4 by default): only the small first window's upload
        // is exposed; each later window's upload overlaps earlier windows' decode, and its
        // entropy kernels (stream C.ent) overlap the previous window's stream kernel (the
        // context stream).  Interleaved A/B (round 1-2), 240 frames of 1080p 4:4:4, round 1: 1:2:2
        // 157 Gpix/s (three runs of three), 1:2:3 157-158, 1:3 151-152, 2:3:3 and four windows
        // slower; round 2, after the faster synchronisation walk, three interleaved rounds:
        // 1:3:3 160-161, 1:2:3 147-160, 1:2:2 145-159, 2:3:3 155, 1:1:2 153, 1:2:2:2 144-151.
        // Round 5, fused path (index pass + fused kernel), one process per schedule, two rounds
        // (tools/win_ab.sh): 1:2:3 2.65 ms, 1:3:5 2.67, 1:2:4 2.68, 2:4:5 2.68-2.71, 2:3:4 2.74,
        // 1:3:3 2.79-2.80, 1:2:3:4 2.80, 1:2:2:2 2.88-2.92, 1:1:2:3 2.90.
        // Round 6, after the fused kernel lost ~10 % of its time (the GPU work, not PCIe, bounds the pass:
        // profiles/r06/fused/windows_sweep{1,2}.log, two boxes, two rounds each): 2:3:4 2.243-2.258 ms,
        // 1:2:3:4 2.253-2.270, 3:4:5 2.263-2.274, 2:3:4:5 2.285-2.295, 1:2:3 2.328-2.335, 1:3:5 2.40,
        // 1:2:4 2.41, 1:3:9 2.57.
        std::vector<uint32_t> weights = {2, 3, 4};
        if (const char* pw = std::getenv("MJ423_GPU_FE_WINDOWS")) {  // A/B override (tools): "N" equal or "a,b,c"
            weights.clear();
            if (std::strchr(pw, ',')) {
                for (const char* q = pw; *q; q = std::strchr(q, ',') ? std::strchr(q, ',') + 1 : q + std::strlen(q))
                    weights.push_back((uint32_t)std::max(1, std::atoi(q)));
            } else {
                weights.assign((size_t)std::max(1, std::atoi(pw)), 1u);
            }
        }
        uint32_t wsum = 0;
        for (uint32_t x : weights) wsum += x;
        // windowed uploads from the file's page-locked copy (every window >= 1 frame)
        const uint8_t* pinned_file = par && weights.size() > 1 && count >= wsum ? mj423_mpg_pinned(m) : nullptr;
        const bool pinned = pinned_file != nullptr;
        std::vector<uint32_t> wb = {0};  // window k = frames [wb[k], wb[k+1])
        const uint32_t wmax = *std::max_element(weights.begin(), weights.end());
        if (pinned && (uint64_t)count * wmax / wsum + 1 <= win) {
            uint32_t acc = 0;
            for (uint32_t x : weights) {
                acc += x;
                wb.push_back((uint32_t)((uint64_t)count * acc / wsum));
            }
        } else {
            const uint32_t step = std::min(win, count);
            for (uint32_t f = step; f < count; f += step) wb.push_back(f);
            wb.push_back(count);
        }
        const uint32_t nwin = (uint32_t)wb.size() - 1;
        uint32_t wf = 0;  // largest window (sizes the coefficient buffer)
        for (uint32_t k = 0; k < nwin; k++) wf = std::max(wf, wb[k + 1] - wb[k]);
        std::vector<uint32_t> win_of(count);
        for (uint32_t k = 0; k < nwin; k++)
            for (uint32_t i = wb[k]; i < wb[k + 1]; i++) win_of[i] = k;

        // frame table and the byte range [b0, b1) holding frames first .. first+count-1
        std::vector<mj423_mpg_frame_t> fr(count);
        for (uint32_t i = 0; i < count; i++)
            if (int rc = mj423_mpg_frame(m, first + i, &fr[i])) return rc;
        const uint64_t b0 = fr[0].position, b1 = fr[count - 1].position + fr[count - 1].frame_size;
        const uint8_t* host0 = pinned ? pinned_file + b0 : fr[0].y - 16;  // the file's bytes at b0

        const int dev = mj423_ctx_device_id(ctx);
        int prev = -1;
        (void)hipGetDevice(&prev);
        struct Restore {
            int d;
            ~Restore() {
                if (d >= 0) (void)hipSetDevice(d);
            }
        } restore{prev};
        if (hipSetDevice(dev) != hipSuccess) return mj423_set_error(MJ423_EHIP, "decode_gpu: hipSetDevice failed");
        hipStream_t s = (hipStream_t)mj423_ctx_stream(ctx);
        auto hipok = [&](hipError_t e, const char* what) {
            return e == hipSuccess ? 0 : mj423_set_error(MJ423_EHIP, std::string("decode_gpu: ") + what + ": " + hipGetErrorString(e));
        };
        auto& d_bytes = C.bytes;
        auto& d_tasks = C.tasks;
        auto& d_status = C.status;
        auto* d_state = C.state;
        const uint64_t nbytes = b1 - b0;
        if (int rc = hipok(hipStreamSynchronize(s), "synchronize")) return rc;  // earlier users of the cached buffers
        // From the first queued copy on, every return -- an error too -- first waits for the call's three
        // streams: the copy engine may still be reading the file's page-locked bytes and the kernels
        // writing the caller's frames, both of which the caller may free once we return.
        struct Drain {
            hipStream_t st[3] = {nullptr, nullptr, nullptr};
            ~Drain() {
                for (hipStream_t x : st)
                    if (x) (void)hipStreamSynchronize(x);
            }
        } drain;
        drain.st[0] = s;
        if (int rc = hipok(d_bytes.ensure(nbytes + 64), "hipMalloc")) return rc;
        // window k's planes in coef[k % 2]: window k+1's entropy kernels (stream C.ent) overlap
        // window k's stream kernel (the context stream)
        for (uint32_t i = 0; i < (fused ? 0u : std::min(nwin, 2u)); i++)
            if (C.coef[i].ensure((size_t)wf * coef_pf * 2) != hipSuccess) {
                if (may_retry && !window_frames) {
                    // the budget cached from an earlier call's free HBM is stale (others have
                    // allocated since): drop the window buffers, measure again, size again
                    (void)hipGetLastError();
                    C.coef[0].release();
                    C.coef[1].release();
                    C.budget = 0;
                    return kRetrySmaller;
                }
                return hipok(hipErrorOutOfMemory, "hipMalloc of the window planes");
            }
        if (int rc = hipok(d_tasks.ensure(((size_t)count * 3 * sizeof(mj423::EntropyTask) + 15) & ~(size_t)15), "hipMalloc"))
            return rc;
        if (int rc = hipok(d_status.ensure(((size_t)count * 3 * 4 + 15) & ~(size_t)15), "hipMalloc")) return rc;
        for (int i = 0; i < 2; i++)
            if (int rc = hipok(d_state[i].ensure(coef_pf * 2), "hipMalloc")) return rc;
        if (pinned) {  // every window's bytes on the copy stream now; window k waits for its event
            if (!C.copy && hipok(hipStreamCreateWithFlags(&C.copy, hipStreamNonBlocking), "stream")) return MJ423_EHIP;
            drain.st[1] = C.copy;
            while (C.ev.size() < nwin) {
                hipEvent_t e;
                if (int rc = hipok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event")) return rc;
                C.ev.push_back(e);
            }
            if (int rc = hipok(hipEventRecord(C.ev[0], s), "event")) return rc;  // after the sync above: buffers free
            if (int rc = hipok(hipStreamWaitEvent(C.copy, C.ev[0], 0), "event")) return rc;
            for (uint32_t k = 0; k < nwin; k++) {
                const uint32_t f0 = wb[k], f1 = wb[k + 1] - 1;
                const uint64_t lo = fr[f0].position - b0, hi = fr[f1].position + fr[f1].frame_size - b0;
                if (int rc = hipok(hipMemcpyAsync((uint8_t*)d_bytes.p + lo, host0 + lo, hi - lo, hipMemcpyHostToDevice, C.copy),
                                   "upload"))
                    return rc;
                if (int rc = hipok(hipEventRecord(C.ev[k], C.copy), "event")) return rc;
            }
        } else if (int rc = hipok(hipMemcpyAsync(d_bytes.p, host0, nbytes, hipMemcpyHostToDevice, s), "upload")) {
            return rc;
        }
        if (host_time) t_upload = us_since();
        // tasks: every (frame, plane) of the range, frame index relative to its window
        std::vector<mj423::EntropyTask> tasks((size_t)count * 3);
        std::vector<uint8_t> types(count);
        for (uint32_t i = 0; i < count; i++) {
            types[i] = (uint8_t)fr[i].frame_type;
            const uint64_t y0 = fr[i].position + 16 - b0;
            const uint64_t off[3] = {y0, y0 + fr[i].y_size, y0 + fr[i].y_size + fr[i].cb_size};
            const uint32_t len[3] = {fr[i].y_size, fr[i].cb_size, fr[i].cr_size};
            if (std::max({len[0], len[1], len[2]}) >= (1u << 28))  // the kernel counts bits in 32 bits
                return mj423_set_error(MJ423_EINVAL, "decode_gpu: a plane bitstream of 256 MiB or more");
            for (int pl = 0; pl < 3; pl++) tasks[(size_t)i * 3 + pl] = {off[pl], len[pl], i - wb[win_of[i]], (uint32_t)pl, types[i]};
        }
        // page-locked staging for this call's small uploads and the status read-back: [tasks |
        // sub0 | seed | status] (the synchronisation above retired the previous call's copies)
        const size_t tasks_b = tasks.size() * sizeof(tasks[0]);
        const size_t sub0_off = (tasks_b + 255) & ~(size_t)255, sub0_b = (tasks.size() + 1) * 4;
        const size_t seed_off = (sub0_off + sub0_b + 255) & ~(size_t)255, seed_b = types[0] != 0 ? coef_pf * 2 : 0;
        const size_t status_off = (seed_off + seed_b + 255) & ~(size_t)255, status_b = tasks.size() * 4;
        // fused path: the frames' types and every window's GOP segments (device metadata of the fused
        // kernel)
        // synchronisation iterations per window (see below; MJ423_GPU_FE_ITERS = 2 ... 12 for A/B)
        // 10 by default: content here settles by iteration 4 (a wrong parse rarely survives more than
        // two or three subsequences), and every iteration after the last change is a ~6-8 us launch
        constexpr uint32_t kMaxIters = 12;
        uint32_t kIters = 10;
        if (const char* pi = std::getenv("MJ423_GPU_FE_ITERS")) kIters = (uint32_t)std::min(12, std::max(2, std::atoi(pi)));
        constexpr uint32_t kFl = kMaxIters + 1;  // words per window: iteration flags (+ one unused)
        std::vector<uint32_t> segs, seg_at(nwin + 1, 0), nsegs(nwin, 0);
        for (uint32_t k = 0; k < nwin; k++) {
            seg_at[k] = (uint32_t)segs.size();
            for (uint32_t i = wb[k]; i < wb[k + 1]; i++)
                if (i == wb[k] || types[i] == 0) segs.push_back(i - wb[k]);
            nsegs[k] = (uint32_t)segs.size() - seg_at[k];
            if (nsegs[k] > 65535) return mj423_set_error(MJ423_EINVAL, "decode_gpu: more than 65535 GOPs in one window");
            segs.push_back(wb[k + 1] - wb[k]);
        }
        const size_t meta_types_b = ((size_t)count + 15) & ~(size_t)15, meta_b = meta_types_b + segs.size() * 4;
        const size_t meta_off = (status_off + status_b + 255) & ~(size_t)255;
        if (int rc = hipok(C.host_ensure(meta_off + ((meta_b + 15) & ~(size_t)15)), "hipHostMalloc")) return rc;  // the copy moves whole 16-B units
        uint8_t* hst = (uint8_t*)C.host;
        uint8_t* hst_d = (uint8_t*)C.host_d;
        std::memcpy(hst, tasks.data(), tasks_b);
        if (int rc = hipok(mj423_launch_copy16(hst_d, d_tasks.p, tasks_b, s), "upload")) return rc;
        // Many-lanes-per-stream front end: subsequences of every task (>= 1 each) and per-lane
        // state arrays for the whole range.  Self-synchronisation usually settles in 2-5
        // iterations; kIters are always launched (an iteration after the one that changed
        // nothing returns at once), and a stream still changing in the last one -- a periodic
        // bit pattern that never falls into phase, e.g. dense blocks ending only at index 63 --
        // is skipped by the emit pass and decoded by the one-wave kernel, all decided on the
        // device: no host round trip per window.
        std::vector<uint32_t> sub0(tasks.size() + 1, 0);
        auto &d_sub0 = C.sub0, &d_start = C.start, &d_exit = C.exit_, &d_nb = C.nb, &d_dcs = C.dcs, &d_zrun = C.zrun,
             &d_flags = C.flags, &d_tchg = C.tchg;
        if (par) {
            uint64_t acc = 0;
            for (size_t i = 0; i < tasks.size(); i++) {
                sub0[i] = (uint32_t)acc;
                acc += std::max<uint64_t>(1, (tasks[i].nbytes + mj423::kSubBytes - 1) / mj423::kSubBytes);
            }
            if (acc >= (1ull << 31)) return mj423_set_error(MJ423_EINVAL, "decode_gpu: too many stream bytes in one call");
            sub0[tasks.size()] = (uint32_t)acc;
            if (int rc = hipok(d_sub0.ensure((sub0.size() * 4 + 15) & ~(size_t)15), "hipMalloc")) return rc;
            if (int rc = hipok(d_start.ensure(acc * 8), "hipMalloc")) return rc;
            if (int rc = hipok(d_exit.ensure(acc * 8), "hipMalloc")) return rc;
            if (int rc = hipok(d_nb.ensure(acc * 4), "hipMalloc")) return rc;
            if (int rc = hipok(d_dcs.ensure(acc * 4), "hipMalloc")) return rc;
            if (int rc = hipok(d_zrun.ensure(acc * 4), "hipMalloc")) return rc;
            if (int rc = hipok(C.zlast.ensure(acc * 4), "hipMalloc")) return rc;
            if (int rc = hipok(C.lane_task.ensure(acc * 4), "hipMalloc")) return rc;
            const size_t qb = ((acc + 31) / 32) * 2 * 4;  // two lane bitmaps
            if (int rc = hipok(C.qbits.ensure(qb), "hipMalloc")) return rc;
            if (int rc = hipok(hipMemsetAsync(C.qbits.p, 0, qb, s), "memset")) return rc;
            if (int rc = hipok(d_flags.ensure(((size_t)nwin * kFl * 4 + 15) & ~(size_t)15), "hipMalloc")) return rc;
            if (int rc = hipok(d_tchg.ensure(tasks.size() * 4), "hipMalloc")) return rc;
            if (int rc = hipok(C.wcnt.ensure(tasks.size() * 16 * 4), "hipMalloc")) return rc;
            if (mc) {  // multi-class arrays, per lane of the largest window
                uint64_t wl = 0;
                for (uint32_t k = 0; k < nwin; k++) wl = std::max<uint64_t>(wl, sub0[(size_t)wb[k + 1] * 3] - sub0[(size_t)wb[k] * 3]);
                if (int rc = hipok(C.mc_list.ensure(std::max<uint64_t>(wl, 1) * 4), "hipMalloc")) return rc;
                if (int rc = hipok(C.mc_x.ensure(std::max<uint64_t>(wl, 1) * 16 * 8), "hipMalloc")) return rc;
                if (int rc = hipok(C.mc_map.ensure(std::max<uint64_t>(wl, 1) * 8), "hipMalloc")) return rc;
                if (int rc = hipok(C.mc_rec.ensure(std::max<uint64_t>(wl, 1) * 16 * 4), "hipMalloc")) return rc;
                if (int rc = hipok(C.mc_st.ensure(std::max<uint64_t>(wl, 1) * 16 * 8), "hipMalloc")) return rc;
                if (int rc = hipok(C.mc_sfx.ensure(std::max<uint64_t>(wl, 1) * 16 * 4), "hipMalloc")) return rc;
                if (int rc = hipok(C.mc_ck.ensure(std::max<uint64_t>(wl, 1) * 4), "hipMalloc")) return rc;
            }
            std::memcpy(hst + sub0_off, sub0.data(), sub0_b);
            if (int rc = hipok(mj423_launch_copy16(hst_d + sub0_off, d_sub0.p, sub0_b, s), "upload")) return rc;
            if (int rc = hipok(hipMemsetAsync(d_flags.p, 0, (size_t)nwin * kFl * 4, s), "memset")) return rc;
        }
        const uint32_t tiles_pp = (nblk + mj423::kFuseTw - 1) / mj423::kFuseTw;
        if (fused) {
            if (int rc = hipok(C.bpos.ensure((size_t)count * 3 * (nblk + 1) * 4), "hipMalloc")) return rc;
            if (int rc = hipok(C.tiles.ensure((size_t)count * 3 * tiles_pp * 8), "hipMalloc")) return rc;
            if (int rc = hipok(C.meta.ensure((meta_b + 15) & ~(size_t)15), "hipMalloc")) return rc;
            std::memcpy(hst + meta_off, types.data(), count);
            std::memcpy(hst + meta_off + meta_types_b, segs.data(), segs.size() * 4);
            if (int rc = hipok(mj423_launch_copy16(hst_d + meta_off, C.meta.p, meta_b, s), "upload")) return rc;
        }
        // seeking into a GOP: absolute coefficients of frame first-1 seed the accumulation
        if (types[0] != 0) {
            int16_t* seed = (int16_t*)(hst + seed_off);
            if (int rc = mj423_mpg_entropy_decode(m, first - 1, 1, seed, 0)) return rc;
            if (int rc = hipok(mj423_launch_copy16(hst_d + seed_off, d_state[1].p, seed_b, s), "upload")) return rc;
        }
        if (!C.ent && hipok(hipStreamCreateWithFlags(&C.ent, hipStreamNonBlocking), "stream")) return MJ423_EHIP;
        if (!C.ev_setup && hipok(hipEventCreateWithFlags(&C.ev_setup, hipEventDisableTiming), "event")) return MJ423_EHIP;
        for (auto* v : {&C.ev_ent, &C.ev_dec})
            while (v->size() < nwin) {
                hipEvent_t e;
                if (int rc = hipok(hipEventCreateWithFlags(&e, hipEventDisableTiming), "event")) return rc;
                v->push_back(e);
            }
        const hipStream_t es = C.ent;
        drain.st[2] = es;
        if (int rc = hipok(hipEventRecord(C.ev_setup, s), "event")) return rc;  // tasks, sub0, flags, seed, bytes
        if (int rc = hipok(hipStreamWaitEvent(es, C.ev_setup, 0), "event")) return rc;
        const bool index_es = std::getenv("MJ423_GPU_FE_INDEX_ES") && std::atoi(std::getenv("MJ423_GPU_FE_INDEX_ES")) == 1;
        for (uint32_t k = 0; k < nwin; k++) {
            const uint32_t w0 = wb[k], n = wb[k + 1] - wb[k];
            // what each of this window's pointers may index, from the allocations (mj423_check.hpp: read by
            // bounds-check builds only)
            mj423::BufLimits lim_common{};
            lim_common.bytes_dw = d_bytes.cap / 4;
            lim_common.tasks = sat_sub(d_tasks.cap / sizeof(mj423::EntropyTask), (uint64_t)w0 * 3);
            lim_common.sub0 = sat_sub(d_sub0.cap / 4, (uint64_t)w0 * 3);
            lim_common.lanes = std::min({d_start.cap / 8, d_exit.cap / 8, d_nb.cap / 4, d_dcs.cap / 4, d_zrun.cap / 4,
                                         C.zlast.cap / 4, C.lane_task.cap / 4});
            lim_common.qbits = C.qbits.cap / 4;
            lim_common.tchg = std::min(sat_sub(d_tchg.cap / 4, (uint64_t)w0 * 3), sat_sub(C.wcnt.cap / 64, (uint64_t)w0 * 3));
            lim_common.status = sat_sub(d_status.cap / 4, (uint64_t)w0 * 3);
            lim_common.bpos = sat_sub(C.bpos.cap / 4, (uint64_t)w0 * 3 * (nblk + 1));
            lim_common.tiles = sat_sub(C.tiles.cap / 8, (uint64_t)w0 * 3 * tiles_pp);
            auto& d_coef = C.coef[k % 2];
            mj423::EntParParams ipp{};
            bool index_on_s = false;
            if (pinned)
                if (int rc = hipok(hipStreamWaitEvent(es, C.ev[k], 0), "event")) return rc;
            if (k >= 2)  // window k-2's stream kernel has read this buffer
                if (int rc = hipok(hipStreamWaitEvent(es, C.ev_dec[k - 2], 0), "event")) return rc;
            mj423::EntropyParams ep{};
            ep.bytes = (const uint8_t*)d_bytes.p;
            ep.bytes_len = nbytes;
            ep.tasks = (const mj423::EntropyTask*)d_tasks.p + (size_t)w0 * 3;
            ep.ntasks = n * 3;
            ep.nblk = nblk;
            ep.out = (int16_t*)d_coef.p;
            ep.coef_pf = coef_pf;
            ep.status = (uint32_t*)d_status.p + (size_t)w0 * 3;
            if (!par) {  // entropy_kernel writes only the coefficients a stream sets
                if (int rc = hipok(hipMemsetAsync(d_coef.p, 0, (size_t)n * coef_pf * 2, es), "memset")) return rc;
                if (int rc = hipok(mj423_launch_entropy(&ep, es), "entropy kernel")) return rc;
            } else {
                mj423::EntParParams& pp = ipp;
                pp = mj423::EntParParams{};
                pp.bytes = ep.bytes;
                pp.bytes_len = ep.bytes_len;
                pp.tasks = ep.tasks;
                pp.ntasks = ep.ntasks;
                pp.sub0 = (const uint32_t*)d_sub0.p + (size_t)w0 * 3;
                pp.g0 = sub0[(size_t)w0 * 3];
                pp.nsub = sub0[(size_t)(w0 + n) * 3];
                pp.nblk = nblk;
                pp.start = (uint64_t*)d_start.p;
                pp.exit_ = (uint64_t*)d_exit.p;
                pp.nb = (uint32_t*)d_nb.p;
                pp.dcs = (uint32_t*)d_dcs.p;
                pp.zrun = (uint32_t*)d_zrun.p;
                pp.zlast = (uint32_t*)C.zlast.p;
                pp.lane_task = (uint32_t*)C.lane_task.p;
                pp.qbits = (uint32_t*)C.qbits.p;
                pp.qwords = (sub0[tasks.size()] + 31) / 32;  // every lane of the call
                pp.flags = (uint32_t*)d_flags.p + (size_t)k * kFl;
                pp.tchg = (uint32_t*)d_tchg.p + (size_t)w0 * 3;
                pp.wcnt = (uint32_t*)C.wcnt.p + (size_t)w0 * 3 * 16;
                pp.unsettled = kIters;  // tchg == kIters: changed in the last iteration
                pp.lds_window = lds_window ? 1u : 0u;
                pp.out = ep.out;
                pp.coef_pf = coef_pf;
                pp.status = ep.status;
                pp.bpos = (uint32_t*)C.bpos.p + (size_t)w0 * 3 * (nblk + 1);
                pp.tiles = (uint2*)C.tiles.p + (size_t)w0 * 3 * tiles_pp;
                pp.tiles_pp = tiles_pp;
                if (mc) {
                    pp.mc_list = (uint32_t*)C.mc_list.p;
                    pp.mc_count = pp.flags + kMaxIters;  // the window's spare flags word (zeroed with them)
                    pp.mc_x = (uint64_t*)C.mc_x.p;
                    pp.mc_map = (uint64_t*)C.mc_map.p;
                    pp.mc_rec = (uint32_t*)C.mc_rec.p;
                    pp.mc_st = (uint64_t*)C.mc_st.p;
                    pp.mc_sfx = (uint32_t*)C.mc_sfx.p;
                    pp.mc_ck = (uint32_t*)C.mc_ck.p;
                }
                pp.lim = lim_common;
                pp.lim.flags = sat_sub(d_flags.cap / 4, (uint64_t)k * kFl);
                pp.lim.mc = std::min({C.mc_list.cap / 4, C.mc_x.cap / 128, C.mc_map.cap / 8, C.mc_rec.cap / 64, C.mc_st.cap / 128,
                                      C.mc_sfx.cap / 64, C.mc_ck.cap / 4});
                if (int rc = hipok(mj423_launch_entpar(&pp, kIters, es), "entropy sync")) return rc;
                if (fused) {  // index only: on the fused kernels' stream (below), or here (A/B)
                    if (index_es) {
                        if (int rc = hipok(mj423_launch_entpar_index(&pp, es), "entropy index")) return rc;
                    } else {
                        index_on_s = true;
                    }
                } else {
                    if (int rc = hipok(mj423_launch_entpar_finish(&pp, es), "entropy emit")) return rc;
                    mj423::EntropyParams fp = ep;  // fallback: only streams still changing do any work
                    fp.tchg = pp.tchg;
                    fp.unsettled = kIters;
                    if (int rc = hipok(mj423_launch_entropy(&fp, es), "entropy kernel")) return rc;
                }
                if (dbg) {
                    std::vector<uint32_t> fl(kIters), tc((size_t)n * 3);
                    (void)hipStreamSynchronize(es);
                    (void)hipMemcpy(fl.data(), pp.flags, kIters * 4, hipMemcpyDeviceToHost);
                    (void)hipMemcpy(tc.data(), pp.tchg, tc.size() * 4, hipMemcpyDeviceToHost);
                    uint32_t used = 0, unsettled = 0;
                    while (used < kIters && fl[used]) used++;
                    for (uint32_t v : tc) unsettled += v == kIters;
                    std::fprintf(stderr, "entpar: window %u/%u: %u lanes, %u changing iterations, %u stream(s) to the fallback%s\n",
                                 k, nwin, pp.nsub - pp.g0, used, unsettled, pinned ? ", pinned upload" : "");
                    std::fprintf(stderr, "entpar: window %u flags:", k);  // walks per iteration in -DMJ423_SYNC_COUNT builds
                    for (uint32_t v : fl) std::fprintf(stderr, " %u", v);
                    std::fprintf(stderr, "\n");
                }
            }
            if (int rc = hipok(hipEventRecord(C.ev_ent[k], es), "event")) return rc;
            if (int rc = hipok(hipStreamWaitEvent(s, C.ev_ent[k], 0), "event")) return rc;
            // The index pass (scan, index walk, serial walk of unsettled streams) runs on the context
            // stream ahead of the window's fused kernel: the entropy stream goes on to the next
            // window's synchronisation meanwhile (MJ423_GPU_FE_INDEX_ES=1: on the entropy stream, A/B)
            if (index_on_s)
                if (int rc = hipok(mj423_launch_entpar_index(&ipp, s), "entropy index")) return rc;
            // window k reads d_state[(k+1)%2] (window k-1's end state, or the seek seed), writes d_state[k%2]
            if (fused) {
                mj423::FusedParams fpar{};
                mj423::DecodeParams& dp = fpar.d;
                rgb_pixel_t* out0 = d_out + (size_t)w0 * out_frame_stride;
                dp.cb_off = 64ll * nblk;  // plane offsets of the [Y | Cb | Cr] state buffers (coef unused)
                dp.cr_off = 128ll * nblk;
                dp.out = reinterpret_cast<uint32_t*>(out0);
                dp.out_fstride = out_frame_stride;
                dp.out_pitch = w;
                dp.aligned16 = (((uintptr_t)out0 & 15u) == 0 && (w & 3u) == 0 && (n == 1 || (out_frame_stride & 3u) == 0)) ? 1u : 0u;
                dp.width = g.width;  // the coded region; the margin is filled below
                dp.height = g.height;
                dp.y_bw = dp.c_bw = dp.mcu_cols = g.y_bw;
                dp.mcu_rows = g.y_bh;
                dp.mcus_per_frame = nblk;
                dp.cols_magic = (uint32_t)std::min<uint64_t>((1ull << 32) / g.y_bw, 0xffffffffull);
                dp.tw = mj423::kFuseTw;
                dp.tiles_per_frame = tiles_pp;
                dp.ntiles = n * tiles_pp;
                mj423_ctx_qt_packed(ctx, dp.qt);
                dp.qt_dev = mj423_ctx_qt_dev(ctx);
                dp.ftype = (const uint8_t*)C.meta.p + w0;
                dp.seg_start = reinterpret_cast<const uint32_t*>((const uint8_t*)C.meta.p + meta_types_b) + seg_at[k];
                dp.nseg = nsegs[k];
                dp.state = types[w0] != 0 ? (const int16_t*)d_state[(k + 1) % 2].p : nullptr;
                dp.state_out = (int16_t*)d_state[k % 2].p;
                dp.st_cb_off = 64ll * nblk;
                dp.st_cr_off = 128ll * nblk;
                fpar.bytes = (const uint8_t*)d_bytes.p;
                fpar.bytes_len = nbytes;
                fpar.tasks = (const mj423::EntropyTask*)d_tasks.p + (size_t)w0 * 3;
                fpar.bpos = (const uint32_t*)C.bpos.p + (size_t)w0 * 3 * (nblk + 1);
                fpar.tiles = (const uint2*)C.tiles.p + (size_t)w0 * 3 * tiles_pp;
                fpar.nblk = nblk;
                fpar.tiles_pp = tiles_pp;
                fpar.state_quantized = k == 0 ? 1u : 0u;  // window 0: the host's seek seed; later: window k-1's end state
                fpar.lim = lim_common;
                fpar.lim.ftype = (uint64_t)count - w0;
                fpar.lim.seg_start = segs.size() - seg_at[k];
                fpar.lim.state = std::min(d_state[0].cap, d_state[1].cap) / 2;
                fpar.lim.out = (uint64_t)(count - w0) * out_frame_stride;
                void* tok = nullptr;
                if (int rc = mj423_ctx_timing_begin(ctx, &tok)) return rc;
                if (int rc = hipok(mj423_launch_mpg_fused(&fpar, s), "fused decode kernel")) return rc;
                if (int rc = mj423_ctx_timing_end(ctx, tok, n)) return rc;
                if (int rc = hipok(hipEventRecord(C.ev_dec[k], s), "event")) return rc;
                continue;
            }
            const int16_t* y = (const int16_t*)d_coef.p;
            mj423_frames_desc_t d = {y, y + 64ull * g.y_blocks, y + 64ull * (g.y_blocks + g.c_blocks), coef_pf,
                                     d_out + (size_t)w0 * out_frame_stride, out_frame_stride, w, n, g.width, g.height,
                                     MJ423_CHROMA_444, MJ423_INPUT_QUANTIZED};
            const int16_t* st_in = types[w0] != 0 ? (const int16_t*)d_state[(k + 1) % 2].p : nullptr;
            if (int rc = mj423_decode_stream_device(ctx, &d, types.data() + w0, st_in, (int16_t*)d_state[k % 2].p))
                return rc;
            if (int rc = hipok(hipEventRecord(C.ev_dec[k], s), "event")) return rc;
        }
        // the defined fill outside the coded region (mj423_margin.hip; no-op for whole blocks)
        if (int rc = hipok((hipError_t)mj423_launch_fill_margin(d_out, out_frame_stride, w, g.width, g.height, w, h, count, s),
                           "margin fill"))
            return rc;
        if (host_time) t_launched = us_since();
        const uint32_t* status = (const uint32_t*)(hst + status_off);
        // the status read back by a DMA copy, not by a kernel's stores into host memory: a kernel's
        // writes to host memory complete before they land, so a fault on them can surface only at
        // a later call
        if (int rc = hipok(hipMemcpyAsync(hst + status_off, d_status.p, status_b, hipMemcpyDeviceToHost, s), "status"))
            return rc;
        if (int rc = hipok(hipStreamSynchronize(s), "synchronize")) return rc;
        // (every stream this call used is idle by now -- s waited for them -- but a fault on one of
        // them may be reported late: check here, so that it is attributed to this call)
        if (int rc = hipok(hipStreamSynchronize(es), "synchronize entropy stream")) return rc;
        if (C.copy)
            if (int rc = hipok(hipStreamSynchronize(C.copy), "synchronize copy stream")) return rc;
        drain = Drain{};  // (every stream synchronised above)
        if (int rc = hipok(hipGetLastError(), "kernel")) return rc;
        for (size_t i = 0; i < tasks.size(); i++)
            if (status[i])
                return mj423_set_error(MJ423_EINVAL, "mpg: frame " + std::to_string(first + i / 3) + " plane " +
                                                         std::to_string(i % 3) +
                                                         (status[i] == 1 ? ": bitstream ended before all of its blocks were decoded"
                                                                         : ": runaway bitstream"));
        return 0;
    }
}
}  // namespace

extern "C" int mj423_mpg_decode_gpu(mj423_ctx* ctx, const mj423_mpg* m, uint32_t first, uint32_t count,
                                    rgb_pixel_t* d_out, uint64_t out_frame_stride, uint32_t window_frames) {
    return mj423_guarded([&]() -> int {
        int rc = decode_gpu_once(ctx, m, first, count, d_out, out_frame_stride, window_frames, true, false);
        if (rc != kRetrySmaller) return rc;
        return decode_gpu_once(ctx, m, first, count, d_out, out_frame_stride, window_frames, false, true);
    });
}
