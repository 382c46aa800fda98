// mj423_io.cpp -- host side around the GPU hot path (include/mj423io.h):
// entropy front end, .mpg container + GOP index (row 2),
// BMP sink (row 4), and the whole-file decoder that drives the GPU.
//
// Reference paths under core0/software/common/libs/mjpeg423/.
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <hip/hip_runtime.h>

#include "../../include/mj423io.h"
#include "mj423_internal.h"
#include "mj423_walk.hpp"

// ===================================================================== front end
// The block walk itself is in mj423_walk.hpp.
using mj423fe::walk;
using mj423fe::walk_sparse;

extern "C" void lossless_decode(int num_blocks, void* bitstream, dct_block_t* DCACq, dct_block_t quant, int P) {
    mj423_dropin_flush_point();  // deferred idct()/ycbcr_to_rgb() calls of the previous frame (mj423_dropin.cpp)
    if (num_blocks <= 0 || !bitstream || !DCACq || !quant) return;
    walk<false>(num_blocks, (const uint8_t*)bitstream, nullptr, &DCACq[0][0][0], &quant[0][0], P != 0, nullptr);
}

extern "C" size_t mj423_lossless_decode_q(int num_blocks, const void* bitstream, size_t nbytes, int16_t* q_abs,
                                          int P) {
    if (num_blocks <= 0 || !bitstream || !q_abs) return num_blocks == 0 ? 0 : (size_t)-1;
    bool over = false;
    const uint8_t* bs = (const uint8_t*)bitstream;
    const size_t used = walk<true>(num_blocks, bs, bs + nbytes, q_abs, nullptr, P != 0, &over);
    return (over && used > nbytes) ? (size_t)-1 : used;
}

// ===================================================================== container
// A file's bytes live in plain page-aligned heap memory: opening, indexing and entropy-decoding
// a file on the host touch no HIP API.  The whole-GPU decoder (mj423_gpu_frontend.cpp) and the
// multi-GPU group upload from a page-locked copy of them, made once on the first GPU use
// (mj423_mpg_pinned: hipHostMalloc + one memcpy) and freed with the file.  No heap memory is ever
// registered with the runtime (round 5 registered each file's heap buffer in place with
// hipHostRegister and unregistered it at close -- DESIGN §5, "The intermittent illegal address").
template <class T>
struct PageAlloc {
    using value_type = T;
    PageAlloc() = default;
    template <class U>
    PageAlloc(const PageAlloc<U>&) {}
    T* allocate(size_t n) {
        const size_t bytes = (n * sizeof(T) + 4095) & ~(size_t)4095;
        void* p = std::aligned_alloc(4096, bytes ? bytes : 4096);
        if (!p) throw std::bad_alloc();
        return static_cast<T*>(p);
    }
    void deallocate(T* p, size_t) { std::free(p); }
    template <class U>
    bool operator==(const PageAlloc<U>&) const { return true; }
    template <class U>
    bool operator!=(const PageAlloc<U>&) const { return false; }
};

struct mj423_mpg {
    std::vector<uint8_t, PageAlloc<uint8_t>> bytes;
    std::mutex pin_mu;
    bool pin_tried = false;
    void* pinned = nullptr;  // page-locked copy of `bytes` (hipHostMalloc), made on the first GPU use
    ~mj423_mpg() {
        if (pinned) (void)hipHostFree(pinned);
    }
    mj423_mpg_header_t hdr{};
    std::vector<mj423_mpg_frame_t> frames;
    std::vector<uint32_t> trailer_index, trailer_pos;
};

namespace {

inline uint32_t rd32(const uint8_t* p) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return v;  // the reference writes host-endian u32 (little-endian on every target it ran on)
}

int index_file(mj423_mpg* m) {
    const size_t n = m->bytes.size();
    const uint8_t* b = m->bytes.data();
    if (n < 20) return mj423_set_error(MJ423_EINVAL, "mpg: file shorter than its 20-byte header");
    m->hdr = {rd32(b), rd32(b + 4), rd32(b + 8), rd32(b + 12), rd32(b + 16)};
    const auto& h = m->hdr;
    // Any size the encoder accepts: it codes the w/8 x h/8 whole blocks (mjpeg423_encoder.c:21-24,
    // 83-84) and the decoder decodes exactly those (mjpeg423_decoder.c:45-48,120-124).
    if (h.width == 0 || h.height == 0 || h.width > (1u << 20) || h.height > (1u << 20))
        return mj423_set_error(MJ423_EINVAL, "mpg: width/height must be in [1, 2^20]");
    size_t off = 20;
    // a frame needs at least its 16-byte header: a corrupt count cannot make us allocate more
    if (h.num_frames > (n - 20) / 16) return mj423_set_error(MJ423_EINVAL, "mpg: frame count exceeds the file");
    m->frames.reserve(h.num_frames);
    for (uint32_t i = 0; i < h.num_frames; i++) {  // mjpeg423_decoder.c:94-107
        if (off + 16 > n) return mj423_set_error(MJ423_EINVAL, "mpg: truncated frame header");
        mj423_mpg_frame_t f{};
        f.index = i;
        f.position = off;
        f.frame_size = rd32(b + off);
        f.frame_type = rd32(b + off + 4);
        f.y_size = rd32(b + off + 8);
        f.cb_size = rd32(b + off + 12);
        if (f.frame_size < 16 || off + f.frame_size > n || (uint64_t)f.y_size + f.cb_size > f.frame_size - 16u)
            return mj423_set_error(MJ423_EINVAL, "mpg: frame " + std::to_string(i) + " sizes out of range");
        if (f.frame_type > 1) return mj423_set_error(MJ423_EINVAL, "mpg: unknown frame type");
        if (i == 0 && f.frame_type != 0) return mj423_set_error(MJ423_EINVAL, "mpg: first frame is not an I-frame");
        f.y = b + off + 16;
        f.cb = f.y + f.y_size;
        f.cr = f.cb + f.cb_size;
        f.cr_size = f.frame_size - 16 - f.y_size - f.cb_size;
        m->frames.push_back(f);
        off += f.frame_size;
    }
    // trailer at 20 + payload_size (mjpeg423_decoder.c:78-86)
    const size_t toff = 20 + (size_t)h.payload_size;
    if (h.num_iframes <= h.num_frames && toff + 8ull * h.num_iframes <= n) {
        for (uint32_t i = 0; i < h.num_iframes; i++) {
            m->trailer_index.push_back(rd32(b + toff + 8 * i));
            m->trailer_pos.push_back(rd32(b + toff + 8 * i + 4));
        }
    }
    return 0;
}

}  // namespace

extern "C" int mj423_mpg_open_memory(const void* data, size_t nbytes, mj423_mpg** out) {
    return mj423_guarded([&]() -> int {
        if (!out || (!data && nbytes)) return mj423_set_error(MJ423_EINVAL, "mpg: null argument");
        *out = nullptr;
        std::unique_ptr<mj423_mpg> m(new mj423_mpg());
        m->bytes.assign((const uint8_t*)data, (const uint8_t*)data + nbytes);
        if (int rc = index_file(m.get())) return rc;
        *out = m.release();
        return 0;
    });
}

extern "C" int mj423_mpg_open(const char* path, mj423_mpg** out) {
    return mj423_guarded([&]() -> int {
        if (!path || !out) return mj423_set_error(MJ423_EINVAL, "mpg: null argument");
        *out = nullptr;
        FILE* fp = std::fopen(path, "rb");
        if (!fp) return mj423_set_error(MJ423_EINVAL, std::string("cannot open input file ") + path);
        std::unique_ptr<FILE, int (*)(FILE*)> f(fp, &std::fclose);
        std::unique_ptr<mj423_mpg> m(new mj423_mpg());
        std::fseek(fp, 0, SEEK_END);
        const long sz = std::ftell(fp);
        std::fseek(fp, 0, SEEK_SET);
        m->bytes.resize(sz > 0 ? (size_t)sz : 0);
        const size_t got = m->bytes.empty() ? 0 : std::fread(m->bytes.data(), 1, m->bytes.size(), fp);
        f.reset();
        if (got != m->bytes.size()) return mj423_set_error(MJ423_EINVAL, "cannot read input file");
        if (int rc = index_file(m.get())) return rc;
        *out = m.release();
        return 0;
    });
}

extern "C" void mj423_mpg_close(mj423_mpg* m) { delete m; }

const uint8_t* mj423_mpg_pinned(const mj423_mpg* cm) {
    mj423_mpg* m = const_cast<mj423_mpg*>(cm);  // a page-locked copy changes no observable state
    std::lock_guard<std::mutex> lk(m->pin_mu);
    if (!m->pin_tried && !m->bytes.empty()) {
        m->pin_tried = true;
        void* p = nullptr;
        // portable: any device of a multi-GPU group may upload from it
        if (hipHostMalloc(&p, m->bytes.size(), hipHostMallocPortable) == hipSuccess) {
            std::memcpy(p, m->bytes.data(), m->bytes.size());
            m->pinned = p;
        } else {
            (void)hipGetLastError();  // (refused: the GPU decoder uploads from pageable memory, synchronously staged)
        }
    }
    return static_cast<const uint8_t*>(m->pinned);
}

int mj423_coded_geometry_444(uint32_t w, uint32_t h, mj423_geometry_t* g) {
    const uint32_t cw = w & ~7u, ch = h & ~7u;  // the whole blocks (mjpeg423_decoder.c:45-48)
    if (cw && ch) return mj423_geometry(cw, ch, MJ423_CHROMA_444, g);
    *g = mj423_geometry_t{};  // narrower or lower than one block: no block at all
    g->width = g->coded_w = cw;
    g->height = g->coded_h = ch;
    g->chroma = MJ423_CHROMA_444;
    g->mcu_w = g->mcu_h = 8;
    return 0;
}

extern "C" int mj423_mpg_geometry(const mj423_mpg* m, mj423_geometry_t* g) {
    if (!m || !g) return mj423_set_error(MJ423_EINVAL, "mpg: null argument");
    return mj423_coded_geometry_444(m->hdr.width, m->hdr.height, g);
}

extern "C" int mj423_mpg_header(const mj423_mpg* m, mj423_mpg_header_t* h) {
    if (!m || !h) return mj423_set_error(MJ423_EINVAL, "mpg: null argument");
    *h = m->hdr;
    return 0;
}

extern "C" int mj423_mpg_frame(const mj423_mpg* m, uint32_t index, mj423_mpg_frame_t* f) {
    if (!m || !f) return mj423_set_error(MJ423_EINVAL, "mpg: null argument");
    if (index >= m->frames.size()) return mj423_set_error(MJ423_EINVAL, "mpg: frame index out of range");
    *f = m->frames[index];
    return 0;
}

extern "C" int mj423_mpg_trailer(const mj423_mpg* m, uint32_t* idx, uint32_t* pos, uint32_t max) {
    if (!m) return mj423_set_error(MJ423_EINVAL, "mpg: null argument");
    const uint32_t n = (uint32_t)std::min<size_t>(max, m->trailer_index.size());
    for (uint32_t i = 0; i < n; i++) {
        if (idx) idx[i] = m->trailer_index[i];
        if (pos) pos[i] = m->trailer_pos[i];
    }
    return (int)m->trailer_index.size();
}

extern "C" int mj423_mpg_gop_start(const mj423_mpg* m, uint32_t index, uint32_t* gop_start) {
    if (!m || !gop_start) return mj423_set_error(MJ423_EINVAL, "mpg: null argument");
    if (index >= m->frames.size()) return mj423_set_error(MJ423_EINVAL, "mpg: frame index out of range");
    uint32_t i = index;
    while (i > 0 && m->frames[i].frame_type != 0) i--;
    *gop_start = i;
    return 0;
}

extern "C" int mj423_mpg_entropy_decode(const mj423_mpg* m, uint32_t first, uint32_t count, int16_t* coef,
                                        int nthreads) {
    return mj423_guarded([&]() -> int {
        if (!m) return mj423_set_error(MJ423_EINVAL, "mpg: null argument");
        if (count == 0) return 0;
        if ((uint64_t)first + count > m->frames.size()) return mj423_set_error(MJ423_EINVAL, "mpg: frame range out of range");
        mj423_geometry_t g;
        if (int rc = mj423_mpg_geometry(m, &g)) return rc;
        const size_t fstride = g.coef_per_frame;
        if (fstride == 0) return 0;  // no whole block: nothing coded
        if (!coef) return mj423_set_error(MJ423_EINVAL, "mpg: null argument");
        const size_t plane_off[3] = {0, 64ull * g.y_blocks, 64ull * (g.y_blocks + g.c_blocks)};
        const int plane_blocks[3] = {(int)g.y_blocks, (int)g.c_blocks, (int)g.c_blocks};
        // Tasks = (GOP segment, plane).  A segment starts at an I-frame (or at `first`,
        // whose state is rebuilt from its GOP start) and runs to the next I-frame.
        struct Seg {
            uint32_t begin, end;  // frames [begin, end) written to the output
            uint32_t warm;        // first frame to decode (GOP start, <= begin)
        };
        std::vector<Seg> segs;
        uint32_t s = first;
        while (s < first + count) {
            uint32_t e = s + 1;
            while (e < first + count && m->frames[e].frame_type != 0) e++;
            uint32_t warm = s;
            if (m->frames[s].frame_type != 0) (void)mj423_mpg_gop_start(m, s, &warm);
            segs.push_back({s, e, warm});
            s = e;
        }
        const size_t ntasks = segs.size() * 3;
        std::atomic<size_t> next{0};
        std::atomic<int> bad{0};
        auto worker = [&]() {
            std::vector<int16_t> scratch;
            for (size_t t; (t = next.fetch_add(1)) < ntasks;) {
                const Seg& sg = segs[t / 3];
                const int plane = (int)(t % 3);
                for (uint32_t f = sg.warm; f < sg.end; f++) {
                    const mj423_mpg_frame_t& fr = m->frames[f];
                    const uint8_t* bs = plane == 0 ? fr.y : plane == 1 ? fr.cb : fr.cr;
                    const size_t nb = plane == 0 ? fr.y_size : plane == 1 ? fr.cb_size : fr.cr_size;
                    int16_t* dst;
                    if (f >= sg.begin) {
                        dst = coef + (size_t)(f - first) * fstride + plane_off[plane];
                        if (f > sg.begin && fr.frame_type != 0)  // P-frame accumulates onto the previous frame
                            std::memcpy(dst, dst - fstride, (size_t)plane_blocks[plane] * 128);
                        else if (f == sg.begin && fr.frame_type != 0)
                            std::memcpy(dst, scratch.data(), (size_t)plane_blocks[plane] * 128);
                    } else {  // warm-up frames before `first`: decode into scratch
                        scratch.resize((size_t)plane_blocks[plane] * 64);
                        dst = scratch.data();
                    }
                    if (mj423_lossless_decode_q(plane_blocks[plane], bs, nb, dst, fr.frame_type != 0) == (size_t)-1)
                        bad.store(1);
                }
            }
        };
        int nt = nthreads > 0 ? nthreads : mj423_host_threads();
        nt = std::max(1, std::min<int>(nt, (int)ntasks));
        std::vector<std::thread> pool;
        for (int i = 1; i < nt; i++) pool.emplace_back(worker);
        worker();
        for (auto& th : pool) th.join();
        if (bad.load()) return mj423_set_error(MJ423_EINVAL, "mpg: a bitstream ended before all of its blocks were decoded");
        return 0;
    });
}

int mj423_delta_plane_task(const mj423_mpg* m, uint32_t f, int plane, int16_t* frame_coef, uint8_t* frame_type) {
    const mj423_mpg_frame_t& fr = m->frames[f];
    const uint32_t nblk = (m->hdr.width / 8) * (m->hdr.height / 8);  // 4:4:4: every plane alike
    if (plane == 0) *frame_type = (uint8_t)fr.frame_type;
    if (nblk == 0) return 0;  // narrower or lower than one block: nothing coded
    int16_t* dst = frame_coef + (size_t)plane * nblk * 64;
    const uint8_t* bs = plane == 0 ? fr.y : plane == 1 ? fr.cb : fr.cr;
    const size_t nb = plane == 0 ? fr.y_size : plane == 1 ? fr.cb_size : fr.cr_size;
    // I: absolute (P = 0 clears and prefix-sums DC); P: deltas onto a cleared plane
    if (fr.frame_type != 0) std::memset(dst, 0, (size_t)nblk * 128);
    return mj423_lossless_decode_q((int)nblk, bs, nb, dst, fr.frame_type != 0) == (size_t)-1 ? -1 : 0;
}

long mj423_sparse_plane_task(const mj423_mpg* m, uint32_t f, int plane, uint8_t* counts, uint32_t* seg_off,
                             uint32_t* ent, uint8_t* frame_type) {
    const mj423_mpg_frame_t& fr = m->frames[f];
    const uint32_t nblk = (m->hdr.width / 8) * (m->hdr.height / 8);
    if (plane == 0) *frame_type = (uint8_t)fr.frame_type;
    const uint8_t* bs = plane == 0 ? fr.y : plane == 1 ? fr.cb : fr.cr;
    const size_t nb = plane == 0 ? fr.y_size : plane == 1 ? fr.cb_size : fr.cr_size;
    bool over = false;
    size_t used = 0;
    const size_t n = walk_sparse((int)nblk, bs, bs + nb, fr.frame_type != 0, counts, seg_off, ent, &over, &used);
    if (over && used > nb) return -1;  // the blocks needed bits past the stream's end
    return (long)n;
}

extern "C" int mj423_mpg_entropy_decode_deltas(const mj423_mpg* m, uint32_t first, uint32_t count, int16_t* coef,
                                               uint8_t* frame_types, int nthreads) {
    return mj423_guarded([&]() -> int {
        if (!m || ((!frame_types || (!coef && m->hdr.width >= 8 && m->hdr.height >= 8)) && count))
            return mj423_set_error(MJ423_EINVAL, "mpg: null argument");
        if (count == 0) return 0;
        if ((uint64_t)first + count > m->frames.size()) return mj423_set_error(MJ423_EINVAL, "mpg: frame range out of range");
        mj423_geometry_t g;
        if (int rc = mj423_mpg_geometry(m, &g)) return rc;
        const size_t fstride = g.coef_per_frame;
        const size_t ntasks = (size_t)count * 3;  // (frame, plane): all independent
        std::atomic<size_t> next{0};
        std::atomic<int> bad{0};
        auto worker = [&]() {
            for (size_t t; (t = next.fetch_add(1)) < ntasks;) {
                const uint32_t f = first + (uint32_t)(t / 3);
                if (mj423_delta_plane_task(m, f, (int)(t % 3), coef + (size_t)(f - first) * fstride,
                                           frame_types + (f - first)) != 0)
                    bad.store(1);
            }
        };
        int nt = nthreads > 0 ? nthreads : mj423_host_threads();
        nt = std::max(1, std::min<int>(nt, (int)ntasks));
        std::vector<std::thread> pool;
        for (int i = 1; i < nt; i++) pool.emplace_back(worker);
        worker();
        for (auto& th : pool) th.join();
        if (bad.load()) return mj423_set_error(MJ423_EINVAL, "mpg: a bitstream ended before all of its blocks were decoded");
        return 0;
    });
}

extern "C" int mj423_decode_mpg(mj423_ctx* ctx, const mj423_mpg* m, uint32_t first, uint32_t count, rgb_pixel_t* out,
                                int nthreads) {
    return mj423_guarded([&]() -> int {
        if (!ctx || !m || (!out && count)) return mj423_set_error(MJ423_EINVAL, "null argument");
        if (count == 0) return 0;
        if ((uint64_t)first + count > m->frames.size()) return mj423_set_error(MJ423_EINVAL, "mpg: frame range out of range");
        const uint32_t w = m->hdr.width, h = m->hdr.height;
        mj423_geometry_t g;
        if (int rc = mj423_mpg_geometry(m, &g)) return rc;
        // Host: per-frame deltas on all threads.  GPU: accumulate + dequant + IDCT + CSC.
        std::vector<int16_t> coef(std::max<size_t>(1, (size_t)count * g.coef_per_frame));
        std::vector<uint8_t> types(count);
        if (int rc = mj423_mpg_entropy_decode_deltas(m, first, count, coef.data(), types.data(), nthreads)) return rc;
        std::vector<int16_t> state;
        if (types[0] != 0 && g.y_blocks) {  // seek into a GOP: absolute coefficients of frame first-1
            state.resize(g.coef_per_frame);
            if (int rc = mj423_mpg_entropy_decode(m, first - 1, 1, state.data(), nthreads)) return rc;
        }
        const size_t in_bytes = coef.size() * 2, st_bytes = (size_t)g.coef_per_frame * 2;
        const size_t out_bytes = (size_t)count * w * h * 4;
        void *d_in = nullptr, *d_out = nullptr, *d_st = nullptr;
        int rc = 0;
        hipStream_t s = (hipStream_t)mj423_ctx_stream(ctx);
        if (hipMalloc(&d_in, in_bytes) != hipSuccess || hipMalloc(&d_out, out_bytes) != hipSuccess ||
            (!state.empty() && hipMalloc(&d_st, st_bytes) != hipSuccess)) {
            rc = mj423_set_error(MJ423_ENOMEM, "decode_mpg: device allocation failed");
        } else if (hipMemcpyAsync(d_in, coef.data(), in_bytes, hipMemcpyHostToDevice, s) != hipSuccess ||
                   (d_st && hipMemcpyAsync(d_st, state.data(), st_bytes, hipMemcpyHostToDevice, s) != hipSuccess)) {
            rc = mj423_set_error(MJ423_EHIP, "decode_mpg: upload failed");
        } else {
            // the coded region (whole blocks) at pitch w, then the defined fill of the rest
            const int16_t* y = (const int16_t*)d_in;
            mj423_frames_desc_t d = {y, y + 64ull * g.y_blocks, y + 64ull * (g.y_blocks + g.c_blocks), g.coef_per_frame,
                                     (rgb_pixel_t*)d_out, (uint64_t)w * h, w, count, g.width, g.height, MJ423_CHROMA_444,
                                     MJ423_INPUT_QUANTIZED};
            if (g.y_blocks) rc = mj423_decode_stream_device(ctx, &d, types.data(), (const int16_t*)d_st, nullptr);
            if (rc == 0 && mj423_launch_fill_margin((rgb_pixel_t*)d_out, (uint64_t)w * h, w, g.width, g.height, w, h, count,
                                                    s) != 0)
                rc = mj423_set_error(MJ423_EHIP, "decode_mpg: margin fill failed");
            if (rc == 0 && (hipMemcpyAsync(out, d_out, out_bytes, hipMemcpyDeviceToHost, s) != hipSuccess ||
                            hipStreamSynchronize(s) != hipSuccess))
                rc = mj423_set_error(MJ423_EHIP, "decode_mpg: download failed");
        }
        if (d_in) (void)hipFree(d_in);
        if (d_out) (void)hipFree(d_out);
        if (d_st) (void)hipFree(d_st);
        return rc;
    });
}

int mj423_host_threads() {
    static const int n = [] {
        int cpus = (int)std::thread::hardware_concurrency();
        cpu_set_t set;
        if (sched_getaffinity(0, sizeof set, &set) == 0) cpus = CPU_COUNT(&set);
        auto read_ll = [](const char* path, long long* v) {
            FILE* f = std::fopen(path, "r");
            const bool ok = f && std::fscanf(f, "%lld", v) == 1;
            if (f) std::fclose(f);
            return ok;
        };
        long long quota = 0, period = 0;
        if (FILE* f = std::fopen("/sys/fs/cgroup/cpu.max", "r")) {  // v2: "max 100000" or "<quota> <period>"
            if (std::fscanf(f, "%lld %lld", &quota, &period) != 2) quota = period = 0;
            std::fclose(f);
        } else if (!read_ll("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", &quota) ||  // v1: -1 = no limit
                   !read_ll("/sys/fs/cgroup/cpu/cpu.cfs_period_us", &period)) {
            quota = period = 0;
        }
        if (quota > 0 && period > 0) cpus = (int)std::min<long long>(cpus, (quota + period - 1) / period);
        return std::max(1, cpus);
    }();
    return n;
}

// ===================================================================== BMP sink
extern "C" int mj423_write_bmp(const char* filename, const rgb_pixel_t* rgb, uint32_t w, uint32_t h) {
    return mj423_guarded([&]() -> int {
        if (!filename || !rgb || w == 0 || h == 0) return mj423_set_error(MJ423_EINVAL, "bmp: bad argument");
        // bmp_create_e(w, h, 32) + bmp_save (mj/libbmp/bmpfile.c:287-330,628-700):
        // 14-byte file header, 40-byte BITMAPINFOHEADER, BI_RGB, 3780 px/m (96 dpi),
        // no palette, rows bottom-up, 4 bytes per pixel in rgb_pixel_t order.
        const uint32_t line = 4 * w, img = line * h;
        uint8_t hdr[54] = {0};
        auto put16 = [&](int o, uint32_t v) { hdr[o] = (uint8_t)v; hdr[o + 1] = (uint8_t)(v >> 8); };
        auto put32 = [&](int o, uint32_t v) { put16(o, v & 0xffff); put16(o + 2, v >> 16); };
        hdr[0] = 'B';
        hdr[1] = 'M';
        put32(2, 54 + img);
        put32(10, 54);
        put32(14, 40);
        put32(18, w);
        put32(22, h);
        put16(26, 1);
        put16(28, 32);
        put32(34, img);
        put32(38, 3780);
        put32(42, 3780);
        FILE* fp = std::fopen(filename, "wb");
        if (!fp) return mj423_set_error(MJ423_EINVAL, std::string("bmp: cannot create ") + filename);
        bool ok = std::fwrite(hdr, 1, 54, fp) == 54;
        for (uint32_t row = h; ok && row-- > 0;) ok = std::fwrite(rgb + (size_t)row * w, 4, w, fp) == w;
        ok = (std::fclose(fp) == 0) && ok;
        return ok ? 0 : mj423_set_error(MJ423_EINVAL, std::string("bmp: write failed for ") + filename);
    });
}

extern "C" void encode_bmp(rgb_pixel_t* rgbblock, uint32_t w_size, uint32_t h_size, const char* filename) {
    mj423_dropin_flush_point();  // the frame's deferred ycbcr_to_rgb() calls land in rgbblock first
    (void)mj423_write_bmp(filename, rgbblock, w_size, h_size);
}

// ============================================================ whole-file decoder
namespace {
// One BMP per frame; called concurrently for different frames (mj423_pipeline_create_for's
// unordered sink), so each call builds its own name.
struct BmpSink {
    std::string base;  // "name0000.bmp": the last 8 characters are replaced (mjpeg423_decoder.c:128-131)
    static int put(void* user, uint32_t fi, const rgb_pixel_t* bgra, uint32_t w, uint32_t h) {
        std::string name = ((const BmpSink*)user)->base;
        const size_t pos = name.size() - 8;
        name[pos] = (char)(fi / 1000 + '0');
        name[pos + 1] = (char)(fi / 100 % 10 + '0');
        name[pos + 2] = (char)(fi / 10 % 10 + '0');
        name[pos + 3] = (char)(fi % 10 + '0');
        return mj423_write_bmp(name.c_str(), bgra, w, h);
    }
};
// BMP writers: the reference writes one file at a time (the frame loop's encode_bmp,
// mjpeg423_decoder.c:132); independent files scale with writer threads into the page cache
// (1080p: 4-5 ms per frame on one thread, profiles/r04/e2e/).
#ifndef MJ423_BMP_WRITERS  // (-DMJ423_BMP_WRITERS=n for A/B builds, tools/ab_bmp_writers.sh)
#define MJ423_BMP_WRITERS 8
#endif
constexpr int kBmpWriters = MJ423_BMP_WRITERS;
}  // namespace

extern "C" int mj423_decode_file(const char* filename_in, const char* filenamebase_out) {
    return mj423_guarded([&]() -> int {
        if (!filename_in || !filenamebase_out || std::strlen(filenamebase_out) < 8)
            return mj423_set_error(MJ423_EINVAL, "output name base must end in NNNN.bmp");
        mj423_mpg* m = nullptr;
        if (int rc = mj423_mpg_open(filename_in, &m)) return rc;
        mj423_ctx* ctx = mj423_default_ctx();
        if (!ctx) {
            mj423_mpg_close(m);
            return MJ423_EHIP;
        }
        BmpSink sink{filenamebase_out};
        int rc = 0;
        if (m->hdr.num_frames) {
            std::lock_guard<std::mutex> lk(mj423_default_mutex());
            const int writers = std::min(kBmpWriters, mj423_host_threads());
            mj423_pipeline* p = nullptr;
            rc = mj423_pipeline_create_for(&p, ctx, m->hdr.width, m->hdr.height, 0, 0, m, 0, m->hdr.num_frames, writers);
            if (rc == 0) rc = mj423_pipeline_decode(p, m, 0, m->hdr.num_frames, &BmpSink::put, &sink, nullptr);
            mj423_pipeline_destroy(p);
        }
        mj423_mpg_close(m);
        return rc;
    });
}

extern "C" void mjpeg423_decode(const char* filename_in, const char* filenamebase_out) {
    (void)mj423_decode_file(filename_in, filenamebase_out);
}
