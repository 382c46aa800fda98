// mj423_multi.cpp -- one process driving N GPUs: frame-range sharding + an RCCL broadcast
// of the quantization tables (include/mj423gpu.h section 5, include/mj423io.h).
//
// What it replaces: the reference spreads one frame over two Nios II cores that hand
// planes back and forth over a mailbox (c0/playback.c:80-134, core1/software/main.c:227-335).
// On MI355X frames are independent once their coefficients are absolute, so a
// job is cut into contiguous frame ranges, one per device, with nothing exchanged on the data
// path.  The decoder's only global state -- {Yquant, Cquant}, mj/common/tables.c:13-32 -- goes
// from rank 0 to every device as one 256-byte ncclBroadcast over xGMI.
//
// RCCL is resolved with dlopen("librccl.so.1") on first use, so single-GPU users of the
// library never load it (and a process that already has torch's RCCL shares that copy).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/mj423gpu.h"
#include "../../include/mj423io.h"
#include "mj423_internal.h"

namespace {

// The handful of RCCL entry points the group uses.
struct Rccl {
    bool tried = false, ok = false;
    std::string why;
    ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*CommCount)(const ncclComm_t, int*) = nullptr;
    ncclResult_t (*Broadcast)(const void*, void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

Rccl& rccl() {
    static Rccl r;
    static std::mutex mu;
    std::lock_guard<std::mutex> lk(mu);
    if (r.tried) return r;
    r.tried = true;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
        const char* e = dlerror();
        r.why = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
        return r;
    }
    auto sym = [&](const char* n) { return dlsym(h, n); };
    r.CommInitAll = (decltype(r.CommInitAll))sym("ncclCommInitAll");
    r.CommDestroy = (decltype(r.CommDestroy))sym("ncclCommDestroy");
    r.CommCount = (decltype(r.CommCount))sym("ncclCommCount");
    r.Broadcast = (decltype(r.Broadcast))sym("ncclBroadcast");
    r.GroupStart = (decltype(r.GroupStart))sym("ncclGroupStart");
    r.GroupEnd = (decltype(r.GroupEnd))sym("ncclGroupEnd");
    r.GetErrorString = (decltype(r.GetErrorString))sym("ncclGetErrorString");
    r.ok = r.CommInitAll && r.CommDestroy && r.CommCount && r.Broadcast && r.GroupStart && r.GroupEnd && r.GetErrorString;
    if (!r.ok) r.why = "librccl.so.1 lacks an ncclCommInitAll/ncclBroadcast/ncclGroup* symbol";
    return r;
}

int ncclfail(ncclResult_t e, const char* what) {
    return mj423_set_error(MJ423_EHIP, std::string("RCCL ") + what + ": " + rccl().GetErrorString(e));
}

int hipfail(hipError_t e, const std::string& what) {
    return mj423_set_error(MJ423_EHIP, what + ": " + hipGetErrorName(e) + " (" + hipGetErrorString(e) + ")");
}

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

// Runs body(rank) on one host thread per rank (ranks' host-side work -- pageable copies,
// front-end walks -- overlaps); returns the first failure and carries its message, which
// the worker recorded in its own thread's mj423_last_error(), to the calling thread.
template <class F>
int for_each_rank_parallel(int n, F&& body) {
    std::vector<int> rc(n, 0);
    std::vector<std::string> msg(n);
    std::vector<std::thread> ts;
    ts.reserve(n);
    for (int r = 0; r < n; r++)
        ts.emplace_back([&, r]() {
            rc[r] = mj423_guarded([&]() -> int { return body(r); });
            if (rc[r]) msg[r] = mj423_last_error();
        });
    for (auto& t : ts) t.join();
    for (int r = 0; r < n; r++)
        if (rc[r]) return mj423_set_error(rc[r], "rank " + std::to_string(r) + ": " + msg[r]);
    return 0;
}

}  // namespace

struct mj423_multi {
    std::vector<int> devices;
    std::vector<mj423_ctx*> ctx;
    std::vector<ncclComm_t> comm;  // empty with MJ423_MULTI_NO_COMM
    std::vector<void*> d_bcast;    // 256-B broadcast buffer per rank
    std::vector<void*> d_in, d_out;  // host-buffer decode staging per rank
    std::vector<size_t> in_cap, out_cap;
    std::vector<hipEvent_t> ev0, ev1;
};

namespace {

void release(mj423_multi* m) {
    if (!m) return;
    for (size_t r = 0; r < m->ctx.size(); r++) {
        DeviceGuard dg(m->devices[r]);
        if (m->ctx[r]) (void)mj423_ctx_synchronize(m->ctx[r]);
        if (r < m->d_bcast.size() && m->d_bcast[r]) (void)hipFree(m->d_bcast[r]);
        if (r < m->d_in.size() && m->d_in[r]) (void)hipFree(m->d_in[r]);
        if (r < m->d_out.size() && m->d_out[r]) (void)hipFree(m->d_out[r]);
        if (r < m->ev0.size() && m->ev0[r]) (void)hipEventDestroy(m->ev0[r]);
        if (r < m->ev1.size() && m->ev1[r]) (void)hipEventDestroy(m->ev1[r]);
    }
    for (ncclComm_t c : m->comm)
        if (c) (void)rccl().CommDestroy(c);
    for (mj423_ctx* c : m->ctx) mj423_ctx_destroy(c);
    delete m;
}

int grow(void** p, size_t* cap, size_t bytes) {
    if (bytes <= *cap) return 0;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    *cap = 0;
    if (hipError_t e = hipMalloc(p, bytes)) {
        *p = nullptr;
        return hipfail(e, "hipMalloc (multi staging)");
    }
    *cap = bytes;
    return 0;
}

int check(const mj423_multi* m) { return m ? 0 : mj423_set_error(MJ423_EINVAL, "null multi-GPU group"); }

}  // namespace

extern "C" {

int mj423_frame_range(uint32_t rank, uint32_t world, uint64_t total, uint64_t* first, uint64_t* count) {
    if (!first || !count || world == 0 || rank >= world) return mj423_set_error(MJ423_EINVAL, "frame_range: bad rank/world");
    const uint64_t base = total / world, extra = total % world;
    *first = rank * base + std::min<uint64_t>(rank, extra);
    *count = base + (rank < extra ? 1 : 0);
    return 0;
}

int mj423_multi_create(mj423_multi** out, int ndev, const int* devices, int flags) {
    return mj423_guarded([&]() -> int {
        if (!out) return mj423_set_error(MJ423_EINVAL, "null group pointer");
        *out = nullptr;
        int visible = 0;
        if (hipGetDeviceCount(&visible) != hipSuccess || visible == 0)
            return mj423_set_error(MJ423_EHIP, "no HIP device available: the MI355X kernels cannot run (no CPU fallback exists)");
        if (ndev <= 0) ndev = visible;
        std::vector<int> devs(ndev);
        for (int r = 0; r < ndev; r++) {
            devs[r] = devices ? devices[r] : r;
            if (devs[r] < 0 || devs[r] >= visible)
                return mj423_set_error(MJ423_EINVAL, "device " + std::to_string(devs[r]) + " is not visible (" +
                                                         std::to_string(visible) + " visible)");
        }
        const bool comm = !(flags & MJ423_MULTI_NO_COMM);
        if (comm) {
            std::vector<int> s = devs;
            std::sort(s.begin(), s.end());
            if (std::adjacent_find(s.begin(), s.end()) != s.end())
                return mj423_set_error(MJ423_EINVAL, "a device appears twice: RCCL needs one rank per GPU "
                                                     "(MJ423_MULTI_NO_COMM allows repeats for rehearsals)");
        }
        mj423_multi* m = new mj423_multi();
        m->devices = devs;
        m->ctx.assign(ndev, nullptr);
        m->d_bcast.assign(ndev, nullptr);
        m->d_in.assign(ndev, nullptr);
        m->d_out.assign(ndev, nullptr);
        m->in_cap.assign(ndev, 0);
        m->out_cap.assign(ndev, 0);
        m->ev0.assign(ndev, nullptr);
        m->ev1.assign(ndev, nullptr);
        for (int r = 0; r < ndev; r++) {
            if (int rc = mj423_ctx_create(&m->ctx[r], devs[r])) {
                std::string why = mj423_last_error();
                release(m);
                return mj423_set_error(rc, "rank " + std::to_string(r) + ": " + why);
            }
            DeviceGuard dg(devs[r]);
            hipError_t e;
            if ((e = hipMalloc(&m->d_bcast[r], 256)) != hipSuccess || (e = hipEventCreate(&m->ev0[r])) != hipSuccess ||
                (e = hipEventCreate(&m->ev1[r])) != hipSuccess) {
                release(m);
                return hipfail(e, "rank " + std::to_string(r) + " resources");
            }
        }
        if (comm) {
            Rccl& R = rccl();
            if (!R.ok) {
                release(m);
                return mj423_set_error(MJ423_EHIP, R.why);
            }
            m->comm.assign(ndev, nullptr);
            if (ncclResult_t e = R.CommInitAll(m->comm.data(), ndev, devs.data())) {
                m->comm.assign(0, nullptr);
                int rc = ncclfail(e, "ncclCommInitAll");
                release(m);
                return rc;
            }
        }
        *out = m;
        return 0;
    });
}

void mj423_multi_destroy(mj423_multi* m) { release(m); }

int mj423_multi_size(const mj423_multi* m) { return m ? (int)m->ctx.size() : 0; }

mj423_ctx* mj423_multi_ctx(mj423_multi* m, int rank) {
    if (!m || rank < 0 || rank >= (int)m->ctx.size()) return nullptr;
    return m->ctx[rank];
}

int mj423_multi_comm_ranks(const mj423_multi* m) {
    if (!m || m->comm.empty()) return 0;
    int n = 0;
    if (rccl().CommCount(m->comm[0], &n) != ncclSuccess) return -1;
    return n;
}

int mj423_multi_set_quant(mj423_multi* m, const int16_t yq[64], const int16_t cq[64]) {
    return mj423_guarded([&]() -> int {
        if (int rc = check(m)) return rc;
        const int n = (int)m->ctx.size();
        if (int rc = mj423_ctx_set_quant(m->ctx[0], yq, cq)) return rc;
        int16_t host[128];
        if (int rc = mj423_ctx_get_quant(m->ctx[0], host, host + 64)) return rc;
        {
            DeviceGuard dg(m->devices[0]);
            if (hipError_t e = hipMemcpy(m->d_bcast[0], host, 256, hipMemcpyHostToDevice)) return hipfail(e, "stage tables");
        }
        if (!m->comm.empty()) {  // rank 0's 256 B to every rank over RCCL (xGMI between GPUs)
            Rccl& R = rccl();
            if (ncclResult_t e = R.GroupStart()) return ncclfail(e, "ncclGroupStart");
            ncclResult_t first_err = ncclSuccess;
            for (int r = 0; r < n; r++) {
                DeviceGuard dg(m->devices[r]);
                ncclResult_t e = R.Broadcast(m->d_bcast[r], m->d_bcast[r], 256, ncclUint8, 0, m->comm[r],
                                             (hipStream_t)mj423_ctx_stream(m->ctx[r]));
                if (e != ncclSuccess && first_err == ncclSuccess) first_err = e;
            }
            ncclResult_t ge = R.GroupEnd();
            if (first_err != ncclSuccess) return ncclfail(first_err, "ncclBroadcast");
            if (ge != ncclSuccess) return ncclfail(ge, "ncclGroupEnd");
        } else {  // rehearsal without RCCL: the same bytes by plain copies
            for (int r = 1; r < n; r++) {
                DeviceGuard dg(m->devices[r]);
                if (hipError_t e = hipMemcpy(m->d_bcast[r], host, 256, hipMemcpyHostToDevice)) return hipfail(e, "copy tables");
            }
        }
        for (int r = 1; r < n; r++) {  // each rank adopts what reached its device
            int16_t got[128];
            DeviceGuard dg(m->devices[r]);
            if (hipError_t e = hipMemcpyAsync(got, m->d_bcast[r], 256, hipMemcpyDeviceToHost,
                                              (hipStream_t)mj423_ctx_stream(m->ctx[r])))
                return hipfail(e, "read broadcast tables");
            if (int rc = mj423_ctx_synchronize(m->ctx[r])) return rc;
            if (int rc = mj423_ctx_set_quant(m->ctx[r], got, got + 64)) return rc;
        }
        return 0;
    });
}

int mj423_multi_decode_frames(mj423_multi* m, uint64_t n, const int16_t* coef, rgb_pixel_t* out, uint32_t w, uint32_t h,
                              int chroma, int input_form) {
    return mj423_guarded([&]() -> int {
        if (int rc = check(m)) return rc;
        mj423_geometry_t g;
        if (int rc = mj423_geometry(w, h, chroma, &g)) return rc;
        if (n && (!coef || !out)) return mj423_set_error(MJ423_EINVAL, "null buffer");
        if (input_form != MJ423_INPUT_QUANTIZED && input_form != MJ423_INPUT_DEQUANTIZED)
            return mj423_set_error(MJ423_EINVAL, "unknown input_form");
        const int world = (int)m->ctx.size();
        const uint64_t px = (uint64_t)w * h;
        return for_each_rank_parallel(world, [&](int r) -> int {
            uint64_t first, cnt;
            mj423_frame_range((uint32_t)r, (uint32_t)world, n, &first, &cnt);
            if (cnt == 0) return 0;
            if (cnt > 0xffffffffull) return mj423_set_error(MJ423_EINVAL, "too many frames for one rank");
            DeviceGuard dg(m->devices[r]);
            const size_t in_b = (size_t)cnt * g.coef_per_frame * 2, out_b = (size_t)cnt * px * 4;
            if (int rc = grow(&m->d_in[r], &m->in_cap[r], in_b)) return rc;
            if (int rc = grow(&m->d_out[r], &m->out_cap[r], out_b)) return rc;
            hipStream_t s = (hipStream_t)mj423_ctx_stream(m->ctx[r]);
            if (hipError_t e = hipMemcpyAsync(m->d_in[r], coef + first * g.coef_per_frame, in_b, hipMemcpyHostToDevice, s))
                return hipfail(e, "upload");
            const int16_t* y = (const int16_t*)m->d_in[r];
            mj423_frames_desc_t d = {y, y + 64ull * g.y_blocks, y + 64ull * (g.y_blocks + g.c_blocks), g.coef_per_frame,
                                     (rgb_pixel_t*)m->d_out[r], px, w, (uint32_t)cnt, w, h, chroma, input_form};
            if (int rc = mj423_decode_frames_device(m->ctx[r], &d)) return rc;
            if (hipError_t e = hipMemcpyAsync(out + first * px, m->d_out[r], out_b, hipMemcpyDeviceToHost, s))
                return hipfail(e, "download");
            if (hipError_t e = hipStreamSynchronize(s)) return hipfail(e, "synchronize");
            return 0;
        });
    });
}

int mj423_multi_decode_frames_device(mj423_multi* m, const mj423_frames_desc_t* descs) {
    return mj423_guarded([&]() -> int {
        if (int rc = check(m)) return rc;
        if (!descs) return mj423_set_error(MJ423_EINVAL, "null descriptors");
        for (size_t r = 0; r < m->ctx.size(); r++) {
            if (descs[r].nframes == 0) continue;
            if (int rc = mj423_decode_frames_device(m->ctx[r], &descs[r]))
                return mj423_set_error(rc, "rank " + std::to_string(r) + ": " + mj423_last_error());
        }
        return 0;
    });
}

int mj423_multi_synth_frames_device(mj423_multi* m, int16_t* const* coef, const uint64_t* frame0, const uint32_t* nframes,
                                    uint32_t w, uint32_t h, int chroma, uint64_t seed) {
    return mj423_guarded([&]() -> int {
        if (int rc = check(m)) return rc;
        if (!coef || !frame0 || !nframes) return mj423_set_error(MJ423_EINVAL, "null argument");
        for (size_t r = 0; r < m->ctx.size(); r++) {
            if (nframes[r] == 0) continue;
            if (int rc = mj423_synth_frames_device(m->ctx[r], coef[r], w, h, chroma, nframes[r], frame0[r], seed))
                return mj423_set_error(rc, "rank " + std::to_string(r) + ": " + mj423_last_error());
        }
        return 0;
    });
}

int mj423_multi_synchronize(mj423_multi* m) {
    if (int rc = check(m)) return rc;
    for (size_t r = 0; r < m->ctx.size(); r++)
        if (int rc = mj423_ctx_synchronize(m->ctx[r])) return rc;
    return 0;
}

int mj423_multi_time_decode(mj423_multi* m, const mj423_frames_desc_t* descs, uint32_t steps, double* max_ms,
                            double* per_rank_ms, double* wall_ms) {
    return mj423_guarded([&]() -> int {
        if (int rc = check(m)) return rc;
        if (!descs || !max_ms) return mj423_set_error(MJ423_EINVAL, "null argument");
        const int n = (int)m->ctx.size();
        if (int rc = mj423_multi_synchronize(m)) return rc;  // every device drained: a common start line
        const auto t0 = std::chrono::steady_clock::now();
        for (int r = 0; r < n; r++) {
            DeviceGuard dg(m->devices[r]);
            if (hipError_t e = hipEventRecord(m->ev0[r], (hipStream_t)mj423_ctx_stream(m->ctx[r]))) return hipfail(e, "event");
        }
        for (uint32_t s = 0; s < steps; s++)  // ranks interleaved so every device gets its first launch at once
            if (int rc = mj423_multi_decode_frames_device(m, descs)) return rc;
        for (int r = 0; r < n; r++) {
            DeviceGuard dg(m->devices[r]);
            if (hipError_t e = hipEventRecord(m->ev1[r], (hipStream_t)mj423_ctx_stream(m->ctx[r]))) return hipfail(e, "event");
        }
        if (int rc = mj423_multi_synchronize(m)) return rc;
        const auto t1 = std::chrono::steady_clock::now();
        double mx = 0.0;
        for (int r = 0; r < n; r++) {
            float ms = 0.f;
            DeviceGuard dg(m->devices[r]);
            if (hipError_t e = hipEventElapsedTime(&ms, m->ev0[r], m->ev1[r])) return hipfail(e, "event time");
            if (per_rank_ms) per_rank_ms[r] = ms;
            mx = std::max(mx, (double)ms);
        }
        *max_ms = mx;
        if (wall_ms) *wall_ms = std::chrono::duration<double, std::milli>(t1 - t0).count();
        return 0;
    });
}

// ------------------------------------------------------------ .mpg across devices
int mj423_mpg_gop_ranges(const mj423_mpg* f, uint32_t first, uint32_t count, uint32_t world, uint32_t* range_first,
                         uint32_t* range_count) {
    return mj423_guarded([&]() -> int {
        if (!f || !range_first || !range_count || world == 0) return mj423_set_error(MJ423_EINVAL, "gop_ranges: bad argument");
        mj423_mpg_header_t hdr;
        if (int rc = mj423_mpg_header(f, &hdr)) return rc;
        if ((uint64_t)first + count > hdr.num_frames) return mj423_set_error(MJ423_EINVAL, "gop_ranges: frame range out of range");
        // cut candidates: the I-frames inside (first, first+count)  (mj/decoder/lossless_decode.c:77-78: an
        // I-frame resets the accumulation, so a range starting there needs no earlier frame)
        std::vector<uint32_t> iframes;
        for (uint32_t i = first + 1; i < first + count; i++) {
            mj423_mpg_frame_t fr;
            if (int rc = mj423_mpg_frame(f, i, &fr)) return rc;
            if (fr.frame_type == 0) iframes.push_back(i);
        }
        std::vector<uint32_t> cuts = {first};
        for (uint32_t r = 1; r < world; r++) {  // the I-frame nearest each balanced cut point
            const double target = first + (double)r * count / world;
            uint32_t best = cuts.back();
            double bd = 1e300;
            for (uint32_t i : iframes) {
                const double d = std::abs((double)i - target);
                if (i > cuts.back() && d < bd) {
                    bd = d;
                    best = i;
                }
            }
            cuts.push_back(best);  // == previous cut when no I-frame is left: that rank gets nothing
        }
        cuts.push_back(first + count);
        for (uint32_t r = 0; r < world; r++) {
            range_first[r] = cuts[r];
            range_count[r] = cuts[r + 1] - cuts[r];
        }
        return 0;
    });
}

int mj423_multi_decode_mpg_gpu(mj423_multi* m, const mj423_mpg* f, uint32_t first, uint32_t count, rgb_pixel_t* const* d_out,
                               uint64_t out_frame_stride, uint32_t* range_first, uint32_t* range_count) {
    return mj423_guarded([&]() -> int {
        if (int rc = check(m)) return rc;
        if (!f || !d_out) return mj423_set_error(MJ423_EINVAL, "multi decode_mpg: null argument");
        const int n = (int)m->ctx.size();
        std::vector<uint32_t> rf(n), rcnt(n);
        if (int rc = mj423_mpg_gop_ranges(f, first, count, (uint32_t)n, rf.data(), rcnt.data())) return rc;
        if (range_first) std::copy(rf.begin(), rf.end(), range_first);
        if (range_count) std::copy(rcnt.begin(), rcnt.end(), range_count);
        for (int r = 0; r < n; r++)
            if (rcnt[r] && !d_out[r]) return mj423_set_error(MJ423_EINVAL, "multi decode_mpg: null output for a rank with frames");
        mj423_mpg_header_t hdr;
        if (int rc = mj423_mpg_header(f, &hdr)) return rc;
        if (out_frame_stride == 0) out_frame_stride = (uint64_t)hdr.width * hdr.height;  // 0: packed frames
        (void)mj423_mpg_pinned(f);  // the page-locked copy, once, before the ranks upload from it concurrently
        return for_each_rank_parallel(n, [&](int r) -> int {
            if (rcnt[r] == 0) return 0;
            return mj423_mpg_decode_gpu(m->ctx[r], f, rf[r], rcnt[r], d_out[r], out_frame_stride, 0);
        });
    });
}

}  // extern "C"
