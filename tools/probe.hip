// tools/probe.hip -- bandwidth probe for the decode kernel (run on the GPU box).
//
// In ONE process, interleaved rounds (cdna_hip_programming.md §5.4 rule 24):
//   * decode_kernel tile-shape / cache-policy / ablation variants on a BASELINE workload
//   * streaming copies with the same byte mix (read the coefficient bytes, write the
//     BGRA bytes) -> the practical HBM ceiling for this mix on this device
//   * read-only and write-only streams
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/probe.hip -o tools/probe
// Run:   tools/probe <420|422|444> <width> <height> <frames> [rounds]
#include "../mjpeg423-video-decoder-software_amd/csrc/mj423_kernels.hip"
#include "probe_variants.hip"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <array>
#include <optional>
#include <dlfcn.h>
#include <string>
#include <vector>

#define CK(x)                                                                                \
    do {                                                                                     \
        hipError_t e = (x);                                                                  \
        if (e != hipSuccess) {                                                               \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
            exit(1);                                                                         \
        }                                                                                    \
    } while (0)

using mj423::u32x4;

// U 16-B loads per lane issued before any store; one-shot grid (no grid-stride loop).
template <int U>
__global__ void __launch_bounds__(256) copy_unroll(const u32x4* __restrict__ in, size_t nin, u32x4* __restrict__ out,
                                                   size_t nout) {
    const size_t base = (size_t)blockIdx.x * 256 * U + threadIdx.x;
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = base + (size_t)u * 256;
        v[u] = (u32x4){(uint32_t)i, 1u, 2u, 3u};
        if (i < nin) v[u] = __builtin_nontemporal_load(in + i);
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = base + (size_t)u * 256;
        if (i < nout) __builtin_nontemporal_store(v[u], out + i);
    }
}

// Copy-ceiling variants: THREADS lanes, U loads in flight per lane, NT = non-temporal,
// GRID_STRIDE = persistent grid-stride loop instead of one-shot.
template <int THREADS, int U, bool NT, bool GRID_STRIDE>
__global__ void __launch_bounds__(THREADS) copy_var(const u32x4* __restrict__ in, size_t nin, u32x4* __restrict__ out,
                                                    size_t nout) {
    const size_t step = GRID_STRIDE ? (size_t)gridDim.x * THREADS * U : 0;
    const size_t n = nin > nout ? nin : nout;  // 4:4:4 reads more than it writes
    for (size_t base = (size_t)blockIdx.x * THREADS * U + threadIdx.x; base < n; base += step) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t i = base + (size_t)u * THREADS;
            v[u] = (u32x4){(uint32_t)i, 1u, 2u, 3u};
            if (i < nin) v[u] = NT ? __builtin_nontemporal_load(in + i) : in[i];
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const size_t i = base + (size_t)u * THREADS;
            if (i < nout) {
                if (NT)
                    __builtin_nontemporal_store(v[u], out + i);
                else
                    out[i] = v[u];
            }
        }
        if (!GRID_STRIDE) break;
    }
}

__global__ void __launch_bounds__(256) read_kernel(const u32x4* __restrict__ in, size_t nin, uint32_t* sink) {
    const size_t stride = (size_t)gridDim.x * 256;
    uint32_t acc = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nin; i += stride) {
        u32x4 v = __builtin_nontemporal_load(in + i);
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

__global__ void __launch_bounds__(256) write_kernel(u32x4* __restrict__ out, size_t nout) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < nout; i += stride) {
        u32x4 v = {(uint32_t)i, 1u, 2u, 3u};
        __builtin_nontemporal_store(v, out + i);
    }
}

// Write-pattern variants (PROBE_WRITES=1): what store shape reaches the highest HBM write rate.
// MODE 0 nt 16 B/lane (one 1-KiB wave store per instruction, U per lane in flight, one-shot grid)
//      1 temporal, 2 sc1, 3 sc0 sc1, 4 nt with each lane writing 16*U contiguous bytes.
template <int MODE, int U>
__global__ void __launch_bounds__(256) write_var(u32x4* __restrict__ out, size_t nout) {
    const size_t base = (size_t)blockIdx.x * 256 * U;
#pragma unroll
    for (int u = 0; u < U; u++) {
        const size_t i = MODE == 4 ? base + (size_t)threadIdx.x * U + u : base + (size_t)u * 256 + threadIdx.x;
        if (i >= nout) continue;
        const u32x4 v = {(uint32_t)i, 1u, 2u, 3u};
        if (MODE == 0 || MODE == 4)
            __builtin_nontemporal_store(v, out + i);
        else if (MODE == 1)
            out[i] = v;
        else if (MODE == 2)
            asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(out + i), "v"(v) : "memory");
        else
            asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1" ::"v"(out + i), "v"(v) : "memory");
    }
}

// One 16-B store per lane; a workgroup of T lanes writes T*16 contiguous bytes.  ORDER 0:
// workgroup b -> chunk b; 1: chunk (b % 8) * per + b / 8 (each XCD a contiguous range);
// 2: chunk b ^ 8-way shuffle inside groups of 64 chunks (b / 8 + (b % 8) * 8 within 64).
template <int T, int ORDER>
__global__ void __launch_bounds__(T) write_one(u32x4* __restrict__ out, size_t nout) {
    const size_t nchunk = (nout + T - 1) / T;
    size_t c = blockIdx.x;
    if (ORDER == 1) {
        const size_t per = (nchunk + 7) / 8;
        c = (blockIdx.x % 8) * per + blockIdx.x / 8;
    } else if (ORDER == 2) {
        c = (blockIdx.x & ~63u) | ((blockIdx.x & 7) << 3) | ((blockIdx.x >> 3) & 7);
    }
    const size_t i = c * T + threadIdx.x;
    if (c < nchunk && i < nout) __builtin_nontemporal_store((u32x4){(uint32_t)i, 1u, 2u, 3u}, out + i);
}

// 2-D tile writes shaped like the decode kernel's CSC output: workgroup (256 lanes) writes
// R rows x WB bytes at pitch PB of an image of H rows, frames back to back; tiles in raster
// order within a frame.  ORDER 0: workgroup b -> tile b (frame-major); 1: each XCD a
// contiguous tile range; 2: frame groups of 8 (tile position p of frames 8g..8g+7 on
// consecutive workgroups, like the batch kernel's fgroup 8).
template <int R, int WB, int ORDER, int T = 256>
__global__ void __launch_bounds__(T) write_tile(uint8_t* __restrict__ out, uint32_t PB, uint32_t H, uint32_t nf) {
    const uint32_t tpr = PB / WB, tpf = (H / R) * tpr, nt = tpf * nf;
    uint32_t t = blockIdx.x;
    if (ORDER == 1) {
        const uint32_t per = (nt + 7) / 8;
        t = (blockIdx.x % 8) * per + blockIdx.x / 8;
    } else if (ORDER == 2) {
        const uint32_t G = 8, grp = G * tpf, fg = t / grp, i = t % grp, gs = min(G, nf - fg * G);
        t = (fg * G + i % gs) * tpf + i / gs;
    }
    if (t >= nt) return;
    const uint32_t f = t / tpf, ti = t % tpf, ty = ti / tpr, tx = ti % tpr;
    uint8_t* base = out + ((size_t)f * H + (size_t)ty * R) * PB + (size_t)tx * WB;
    constexpr int PER_ROW = WB / 16, TOTAL = R * PER_ROW;
    for (int j = threadIdx.x; j < TOTAL; j += T) {
        const int r = j / PER_ROW, c = j % PER_ROW;
        __builtin_nontemporal_store((u32x4){(uint32_t)j, 1u, 2u, 3u}, reinterpret_cast<u32x4*>(base + (size_t)r * PB + 16 * c));
    }
}

// P-frames as deltas (what the stream kernel is fed in production): walking each coefficient
// back from the last frame, frame f -= frame f - 1 wherever f is a P-frame.
__global__ void __launch_bounds__(256) to_deltas(int16_t* c, uint64_t per_frame, const uint8_t* ft, uint32_t nf) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < per_frame; i += (uint64_t)gridDim.x * 256)
        for (uint32_t f = nf - 1; f >= 1; f--)
            if (ft[f]) c[f * per_frame + i] -= c[(f - 1) * per_frame + i];
}

__global__ void __launch_bounds__(256) count_diff(const u32x4* __restrict__ a, const u32x4* __restrict__ b, size_t n,
                                                  unsigned long long* bad) {
    unsigned long long m = 0;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const u32x4 x = a[i], y = b[i];
        m += (x.x != y.x) + (x.y != y.y) + (x.z != y.z) + (x.w != y.w);
    }
    if (m) atomicAdd(bad, m);
}

static const int16_t kY[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                               14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                               18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                               49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
static const int16_t kC[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                               24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                               99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                               99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
static const int32_t kZZ[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

struct Case {
    std::string name;
    double bytes;
    std::function<void()> f;
};

struct Bench {
    int mode;
    uint32_t W, H, NF;
    uint32_t mw, mh;  // MCU size
    uint64_t yblocks, cblocks, coef_pf, in_bytes, out_bytes;
    uint64_t coef_stride = 0;  // int16 per frame in memory (coef_pf + PROBE_FPAD padding)
    int16_t* coef;
    uint32_t* out;
    mj423::DecodeParams base;

    // the runtime's workgroup order for this geometry (mj423_batch_fgroup)
    uint32_t fgroup(int mode, uint32_t twmax) const {
        uint32_t tpf;
        if (mode == 420) {
            const uint32_t tpr = (base.mcu_cols + twmax - 1) / twmax;
            tpf = base.mcu_rows * tpr;
        } else {
            tpf = (base.mcu_cols * base.mcu_rows + twmax - 1) / twmax;
        }
        return mj423_batch_fgroup(mode, tpf);
    }

    // Stream (GOP) kernel on the same frames, I every `gop` frames (the P-frames' data are
    // the synthetic frames themselves: timing only, no parity here).
    uint32_t* qt_dev = nullptr;
    uint8_t* ftype_dev = nullptr;
    uint32_t* seg_dev = nullptr;
    uint32_t nseg = 0;
    void gop_setup(uint32_t gop) {
        std::vector<uint8_t> ft(NF);
        std::vector<uint32_t> seg;
        for (uint32_t f = 0; f < NF; f++) {
            ft[f] = f % gop ? 1 : 0;
            if (!ft[f]) seg.push_back(f);
        }
        seg.push_back(NF);
        nseg = (uint32_t)seg.size() - 1;
        CK(hipMalloc(&qt_dev, 256));
        CK(hipMemcpy(qt_dev, base.qt, 256, hipMemcpyHostToDevice));
        CK(hipMalloc(&ftype_dev, NF));
        CK(hipMemcpy(ftype_dev, ft.data(), NF, hipMemcpyHostToDevice));
        CK(hipMalloc(&seg_dev, seg.size() * 4));
        CK(hipMemcpy(seg_dev, seg.data(), seg.size() * 4, hipMemcpyHostToDevice));
        if (getenv("PROBE_DELTAS")) {  // real P-frame deltas instead of absolute frames fed as deltas
            hipLaunchKernelGGL(to_deltas, dim3(4096), dim3(256), 0, 0, coef, coef_stride, ftype_dev, NF);
            CK(hipDeviceSynchronize());
        }
    }
    template <int MODE, int TW, int THREADS, int FLAGS, int WPE = 0>
    Case gop_case(const char* tag) {
        mj423::DecodeParams q = base;
        q.mcus_per_frame = q.mcu_cols * q.mcu_rows;
        q.cols_magic = (uint32_t)std::min<uint64_t>((1ull << 32) / q.mcu_cols, 0xffffffffull);
        if (MODE == 420) {
            q.tiles_per_row = (q.mcu_cols + TW - 1) / TW;
            q.tw = align420 ? TW : (q.mcu_cols + q.tiles_per_row - 1) / q.tiles_per_row;
            q.tiles_per_frame = q.mcu_rows * q.tiles_per_row;
        } else {
            q.tw = TW;
            q.tiles_per_frame = (q.mcus_per_frame + TW - 1) / TW;
        }
        q.ntiles = NF * q.tiles_per_frame;
        q.qt_dev = qt_dev;
        q.ftype = ftype_dev;
        q.seg_start = seg_dev;
        q.nseg = nseg;
        // bit 18 of the probe flags: XCD-contiguous job order (1-D grid)
        // bit 22: XCD eighths of every segment (gop_order 2, 1-D grid)
        q.gop_order = (FLAGS & 262144) ? mj423::kFgroupXcd : (FLAGS & (1 << 22)) ? 2u : 0u;
        const dim3 grid = (FLAGS & 262144) ? dim3(8 * ((q.tiles_per_frame * nseg + 7) / 8))
                          : (FLAGS & (1 << 22)) ? dim3(8 * ((q.tiles_per_frame + 7) / 8) * nseg)
                                                 : dim3(q.tiles_per_frame, nseg);
        char name[96];
        snprintf(name, sizeof(name), "gop<%d,%d,%d> %s", MODE, TW, THREADS, tag);
        return {name, (double)(in_bytes + out_bytes), [q, grid] {
                    if constexpr (WPE != 0)  // loader/compute-wave kernel, 2 * THREADS lanes
                        hipLaunchKernelGGL((mj423::decode_gop_ws_kernel<MODE, TW, THREADS, FLAGS & ~262144, WPE>), grid,
                                           dim3(2 * THREADS), 0, 0, q);
                    else if constexpr ((FLAGS & 16384) != 0)
                        hipLaunchKernelGGL((mj423::decode_gop_reg_kernel<MODE, TW, THREADS, FLAGS & ~16384 & ~262144>), grid,
                                           dim3(THREADS), 0, 0, q);
                    else
                        hipLaunchKernelGGL((mj423::decode_gop_kernel<MODE, TW, THREADS, FLAGS & ~262144 & ~(1 << 22)>), grid, dim3(THREADS), 0, 0, q);
                }};
    }

    // The same launch through the product library's own code object (dlopen: same kernel
    // source, compiled in the library's translation unit) -- separates code placement from
    // everything else when the bench and the probe disagree.
    std::optional<Case> lib_case(int mode, uint32_t twmax) {
        void* h = dlopen("mjpeg423-video-decoder-software_amd/libmj423gpu.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) return std::nullopt;
        using Fn = hipError_t (*)(const mj423::DecodeParams*, uint32_t, int, hipStream_t);
        auto fn = (Fn)dlsym(h, "mj423_launch_decode");
        if (!fn) return std::nullopt;
        mj423::DecodeParams q = base;
        q.fgroup = fgroup(mode, twmax);
        q.mcus_per_frame = q.mcu_cols * q.mcu_rows;
        q.cols_magic = (uint32_t)std::min<uint64_t>((1ull << 32) / q.mcu_cols, 0xffffffffull);
        if (mode == 420) {
            q.tiles_per_row = (q.mcu_cols + twmax - 1) / twmax;
            q.tw = (q.mcu_cols + q.tiles_per_row - 1) / q.tiles_per_row;
            q.tiles_per_frame = q.mcu_rows * q.tiles_per_row;
        } else {
            q.tw = twmax;
            q.tiles_per_frame = (q.mcus_per_frame + twmax - 1) / twmax;
        }
        q.ntiles = NF * q.tiles_per_frame;
        const uint32_t nf = NF;
        return Case{"libmj423gpu.so mj423_launch_decode", (double)(in_bytes + out_bytes),
                    [fn, q, nf, mode] { CK(fn(&q, nf, mode, 0)); }};
    }

    // LDS-state stream kernel with STAGE staging lanes out of THREADS, at WPE waves per SIMD.
    template <int MODE, int TW, int THREADS, int FLAGS, int STAGE, int WPE>
    Case gop_wide_case(const char* tag) {
        Case c = gop_case<MODE, TW, STAGE, FLAGS>(tag);  // same parameters and grid
        mj423::DecodeParams q = gop_params<MODE, TW>();
        const dim3 grid(q.tiles_per_frame, nseg);
        char name[128];
        snprintf(name, sizeof(name), "gop<%d,%d,%d> stage %d wpe %d %s", MODE, TW, THREADS, STAGE, WPE, tag);
        c.name = name;
        c.f = [q, grid] {
            hipLaunchKernelGGL((mj423::decode_gop_wide_kernel<MODE, TW, THREADS, FLAGS, STAGE, WPE>), grid, dim3(THREADS), 0, 0, q);
        };
        return c;
    }
    // LDS-state stream kernel with LW dedicated loader waves (decode_gop_lw_kernel).
    // Register-state stream kernel (decode_gop_reg_kernel) at WPE waves per SIMD.
    template <int MODE, int TW, int THREADS, int FLAGS, int WPE>
    Case gop_reg_case(const char* tag) {
        Case c = gop_case<MODE, TW, THREADS, FLAGS>(tag);
        mj423::DecodeParams q = gop_params<MODE, TW>();
        const dim3 grid(q.tiles_per_frame, nseg);
        char name[128];
        snprintf(name, sizeof(name), "gop<%d,%d,%d> reg state wpe %d %s", MODE, TW, THREADS, WPE, tag);
        c.name = name;
        c.f = [q, grid] {
            hipLaunchKernelGGL((mj423::decode_gop_reg_kernel<MODE, TW, THREADS, FLAGS, WPE>), grid, dim3(THREADS), 0, 0, q);
        };
        return c;
    }
    // Pipelined stream kernel (decode_gop_pipe_kernel): 3 IDCT + 4 CSC waves.
    template <int MODE, int TW, int FLAGS, int WPE>
    Case gop_pipe_case(const char* tag) {
        Case c = gop_case<MODE, TW, 256, FLAGS>(tag);
        mj423::DecodeParams q = gop_params<MODE, TW>();
        const dim3 grid(q.tiles_per_frame, nseg);
        char name[128];
        snprintf(name, sizeof(name), "gop<%d,%d> pipelined wpe %d %s", MODE, TW, WPE, tag);
        c.name = name;
        c.f = [q, grid] { hipLaunchKernelGGL((mj423::decode_gop_pipe_kernel<MODE, TW, FLAGS, WPE>), grid, dim3(448), 0, 0, q); };
        return c;
    }
    // Overlaid-planes stream kernel (decode_gop_ovl_kernel).
    template <int MODE, int TW, int THREADS, int FLAGS, int OVL, int WPE>
    Case gop_ovl_case(const char* tag) {
        Case c = gop_case<MODE, TW, THREADS, FLAGS>(tag);
        mj423::DecodeParams q = gop_params<MODE, TW>();
        const dim3 grid(q.tiles_per_frame, nseg);
        char name[128];
        snprintf(name, sizeof(name), "gop<%d,%d,%d> ovl %d wpe %d %s", MODE, TW, THREADS, OVL, WPE, tag);
        c.name = name;
        c.f = [q, grid] {
            hipLaunchKernelGGL((mj423::decode_gop_ovl_kernel<MODE, TW, THREADS, FLAGS, OVL, WPE>), grid, dim3(THREADS), 0, 0, q);
        };
        return c;
    }
    template <int MODE, int TW, int THREADS, int FLAGS, int LW, int WPE, int D = 1>
    Case gop_lw_case(const char* tag) {
        Case c = gop_case<MODE, TW, THREADS, FLAGS>(tag);
        mj423::DecodeParams q = gop_params<MODE, TW>();
        const dim3 grid(q.tiles_per_frame, nseg);
        char name[128];
        snprintf(name, sizeof(name), "gop<%d,%d,%d> +%d loader waves wpe %d depth %d %s", MODE, TW, THREADS, LW, WPE, D, tag);
        c.name = name;
        c.f = [q, grid] {
            hipLaunchKernelGGL((mj423::decode_gop_lw_kernel<MODE, TW, THREADS, FLAGS, LW, WPE, D>), grid, dim3(THREADS + 64 * LW), 0,
                               0, q);
        };
        return c;
    }
    // Record-input stream kernel (decode_gop_rec_kernel): records made once from the dense frames.
    uint32_t* recs = nullptr;
    template <int MODE, int TW, int THREADS, int FLAGS>
    Case gop_rec_case(const char* tag) {
        Case c = gop_case<MODE, TW, THREADS, FLAGS>(tag);
        mj423::DecodeParams q = gop_params<MODE, TW>();
        if (!recs) {
            const uint64_t nblocks = in_bytes / 128;
            unsigned long long* dn = nullptr;
            CK(hipMalloc(&recs, nblocks * 64));
            CK(hipMalloc(&dn, 8));
            CK(hipMemset(dn, 0, 8));
            hipLaunchKernelGGL(mj423::make_records_kernel, dim3((unsigned)((nblocks + 255) / 256)), dim3(256), 0, 0,
                               (const int16_t*)coef, recs, nblocks, dn);
            unsigned long long ndense = 0;
            CK(hipMemcpy(&ndense, dn, 8, hipMemcpyDeviceToHost));
            printf("records: %llu blocks, %llu (%.2f %%) dense (> 15 coefficients)\n", (unsigned long long)nblocks, ndense,
                   100.0 * ndense / nblocks);
        }
        q.state = (const int16_t*)recs;
        q.coef = base.coef;
        q.out = base.out;
        const dim3 grid(q.tiles_per_frame, nseg);
        char name[128];
        snprintf(name, sizeof(name), "gop<%d,%d,%d> records %s", MODE, TW, THREADS, tag);
        c.name = name;
        c.f = [q, grid] { hipLaunchKernelGGL((mj423::decode_gop_rec_kernel<MODE, TW, THREADS, FLAGS>), grid, dim3(THREADS), 0, 0, q); };
        return c;
    }
    // Global-state stream kernel (decode_gop_gs_kernel); the records are allocated once.
    void* gs_state = nullptr;
    template <int MODE, int TW, int THREADS, int FLAGS, int WPE>
    Case gop_gs_case(const char* tag) {
        Case c = gop_case<MODE, TW, THREADS, FLAGS>(tag);
        mj423::DecodeParams q = gop_params<MODE, TW>();
        using T = mj423::Tile<MODE, TW, THREADS>;
        const size_t bytes = (size_t)q.tiles_per_frame * nseg * T::CHUNKS * THREADS * 16;
        if (!gs_state) CK(hipMalloc(&gs_state, bytes));  // sized by the first case (same tile for every mode's cases)
        q.state_out = (int16_t*)gs_state;
        const dim3 grid(q.tiles_per_frame, nseg);
        char name[128];
        snprintf(name, sizeof(name), "gop<%d,%d,%d> global state wpe %d %s", MODE, TW, THREADS, WPE, tag);
        c.name = name;
        c.f = [q, grid] {
            hipLaunchKernelGGL((mj423::decode_gop_gs_kernel<MODE, TW, THREADS, FLAGS, WPE>), grid, dim3(THREADS), 0, 0, q);
        };
        return c;
    }
    template <int MODE, int TW>
    mj423::DecodeParams gop_params() {
        mj423::DecodeParams q = base;
        q.mcus_per_frame = q.mcu_cols * q.mcu_rows;
        q.cols_magic = (uint32_t)std::min<uint64_t>((1ull << 32) / q.mcu_cols, 0xffffffffull);
        if (MODE == 420) {
            q.tiles_per_row = (q.mcu_cols + TW - 1) / TW;
            q.tw = (q.mcu_cols + q.tiles_per_row - 1) / q.tiles_per_row;
            q.tiles_per_frame = q.mcu_rows * q.tiles_per_row;
        } else {
            q.tw = TW;
            q.tiles_per_frame = (q.mcus_per_frame + TW - 1) / TW;
        }
        q.ntiles = NF * q.tiles_per_frame;
        q.qt_dev = qt_dev;
        q.ftype = ftype_dev;
        q.seg_start = seg_dev;
        q.nseg = nseg;
        q.gop_order = 0;
        return q;
    }

    template <int MODE, int TW>
    mj423::DecodeParams persist_params() {  // the batch kernel's parameters (frame-major tile numbering)
        mj423::DecodeParams q = base;
        q.fgroup = 0;
        q.mcus_per_frame = q.mcu_cols * q.mcu_rows;
        q.cols_magic = (uint32_t)std::min<uint64_t>((1ull << 32) / q.mcu_cols, 0xffffffffull);
        q.tiles_per_row = (q.mcu_cols + TW - 1) / TW;
        q.tw = (q.mcu_cols + q.tiles_per_row - 1) / q.tiles_per_row;
        q.tiles_per_frame = q.mcu_rows * q.tiles_per_row;
        q.ntiles = NF * q.tiles_per_frame;
        return q;
    }
    bool align420 = false;  // 4:2:0 tiles of exactly TW MCUs (2-KiB aligned rows at TW 32), a short last tile per row
    template <int MODE, int TW, int THREADS, int FLAGS>
    Case decode_case(const char* tag, uint32_t fgroup = 0) {
        mj423::DecodeParams q = base;
        q.fgroup = fgroup;
        q.mcus_per_frame = q.mcu_cols * q.mcu_rows;
        q.cols_magic = (uint32_t)std::min<uint64_t>((1ull << 32) / q.mcu_cols, 0xffffffffull);
        if (MODE == 420) {
            q.tiles_per_row = (q.mcu_cols + TW - 1) / TW;
            q.tw = align420 ? TW : (q.mcu_cols + q.tiles_per_row - 1) / q.tiles_per_row;
            q.tiles_per_frame = q.mcu_rows * q.tiles_per_row;
        } else {
            q.tw = TW;
            q.tiles_per_frame = (q.mcus_per_frame + TW - 1) / TW;
        }
        q.ntiles = NF * q.tiles_per_frame;
        // kOrderXcd maps workgroup b to tile (b % 8) * per + b / 8: a bijection on 8 * per workgroups
        const uint32_t tiles = ((FLAGS & 64) || fgroup == mj423::kFgroupXcd) ? 8 * ((q.ntiles + 7) / 8) : q.ntiles;
        char name[96];
        if (fgroup == mj423::kFgroupXcd)
            snprintf(name, sizeof(name), "decode<%d,%d,%d> %s order xcd", MODE, TW, THREADS, tag);
        else if (fgroup > 1)
            snprintf(name, sizeof(name), "decode<%d,%d,%d> %s fgroup %u", MODE, TW, THREADS, tag, fgroup);
        else
            snprintf(name, sizeof(name), "decode<%d,%d,%d> %s", MODE, TW, THREADS, tag);
        return {name, (double)(in_bytes + out_bytes), [q, tiles] {
                    hipLaunchKernelGGL((mj423::decode_kernel<MODE, TW, THREADS, FLAGS>), dim3(tiles), dim3(THREADS), 0,
                                       0, q);
                }};
    }
};

int main(int argc, char** argv) {
    Bench b;
    b.mode = argc > 1 ? atoi(argv[1]) : 420;
    b.W = argc > 2 ? (uint32_t)atoi(argv[2]) : 3840;
    b.H = argc > 3 ? (uint32_t)atoi(argv[3]) : 2160;
    b.NF = argc > 4 ? (uint32_t)atoi(argv[4]) : 300;
    const int rounds = argc > 5 ? atoi(argv[5]) : 7;
    const uint32_t sx = b.mode == 444 ? 1 : 2, sy = b.mode == 420 ? 2 : 1;
    b.mw = 8 * sx;
    b.mh = 8 * sy;
    const uint32_t cw = (b.W + b.mw - 1) / b.mw * b.mw, ch = (b.H + b.mh - 1) / b.mh * b.mh;
    const uint32_t ybw = cw / 8, ybh = ch / 8, cbw = ybw / sx, cbh = ybh / sy;
    b.yblocks = (uint64_t)ybw * ybh;
    b.cblocks = (uint64_t)cbw * cbh;
    b.coef_pf = 64 * (b.yblocks + 2 * b.cblocks);
    b.in_bytes = 2 * b.coef_pf * b.NF;
    // PROBE_PITCH=<pixels>: pad output rows (layout experiment; bytes counted stay displayed pixels)
    const uint32_t pitch = getenv("PROBE_PITCH") ? (uint32_t)atoi(getenv("PROBE_PITCH")) : b.W;
    b.out_bytes = 4ull * b.W * b.H * b.NF;
    // PROBE_FPAD=<bytes> (multiple of 16): gap between consecutive frames of the coefficient and the
    // output buffers (address-mapping diagnostic; bytes counted stay the algorithmic ones; only the
    // PROBE_FPAD case list may run with it, the other modes size their second buffers unpadded)
    const uint64_t fpad = getenv("PROBE_FPAD") ? strtoull(getenv("PROBE_FPAD"), nullptr, 10) / 16 * 16 : 0;
    b.coef_stride = b.coef_pf + fpad / 2;
    const uint64_t out_fs = (uint64_t)pitch * b.H + fpad / 4;
    const uint64_t out_alloc = 4ull * out_fs * b.NF + (getenv("PROBE_OFFSETS") ? (64ull << 20) : 0);
    printf("workload %ux%u %d x%u frames: in %.3f GB out %.3f GB\n", b.W, b.H, b.mode, b.NF, b.in_bytes / 1e9,
           b.out_bytes / 1e9);
    uint32_t* sink;
    CK(hipMalloc(&b.coef, 2 * b.coef_stride * b.NF));
    CK(hipMalloc(&b.out, out_alloc));
    CK(hipMalloc(&sink, 64));

    mj423::SynthParams sp;
    memset(&sp, 0, sizeof(sp));
    sp.coef = b.coef;
    sp.frame_stride = b.coef_stride;
    sp.y_blocks = (uint32_t)b.yblocks;
    sp.c_blocks = (uint32_t)b.cblocks;
    sp.nframes = b.NF;
    sp.seed = 0x4D4A3432;
    memcpy(sp.yq, kY, 128);
    memcpy(sp.cq, kC, 128);
    memcpy(sp.zigzag, kZZ, 256);
    for (int k = 1; k < 64; k++) sp.ac_thresh[k] = (uint32_t)(0.6 * exp(-k / 8.0) * 4294967296.0);
    CK(mj423_launch_synth(&sp, 0));

    mj423::DecodeParams& p = b.base;
    memset(&p, 0, sizeof(p));
    p.coef = b.coef;
    p.cb_off = (int64_t)(64 * b.yblocks);
    p.cr_off = (int64_t)(64 * (b.yblocks + b.cblocks));
    p.plane_fstride = b.coef_stride;
    p.out = b.out;
    p.out_fstride = out_fs;
    p.out_pitch = pitch;
    p.aligned16 = (pitch % 4 == 0) ? 1 : 0;
    p.width = b.W;
    p.height = b.H;
    p.y_bw = ybw;
    p.c_bw = cbw;
    p.mcu_cols = cw / b.mw;
    p.mcu_rows = ch / b.mh;
    for (int i = 0; i < 32; i++) {
        p.qt[0][i] = (uint16_t)kY[2 * i] | ((uint32_t)(uint16_t)kY[2 * i + 1] << 16);
        p.qt[1][i] = (uint16_t)kC[2 * i] | ((uint32_t)(uint16_t)kC[2 * i + 1] << 16);
    }
    // PROBE_LOC=out: every frame writes frame 0's output; =in: every frame reads frame 0's
    // coefficients (DRAM-locality diagnostics; the bytes counted stay the algorithmic ones)
    if (const char* loc = getenv("PROBE_LOC")) {
        if (strstr(loc, "out")) p.out_fstride = 0;
        if (strstr(loc, "in")) p.plane_fstride = 0;
        printf("locality diagnostic: %s\n", loc);
    }
    const size_t nin = b.in_bytes / 16, nout = b.out_bytes / 16;
    std::vector<Case> cases;
    if (const char* bo = getenv("PROBE_BIGOFF")) {
        // One physically contiguous allocation (hipDeviceMallocContiguous; plain hipMalloc if refused):
        // coefficients at its start, the output at (coefficient bytes rounded up to 1 GiB) + d MiB
        // for each d in the list -- the batch kernel's rate against the streams' relative placement.
        std::vector<uint64_t> ds;
        for (const char* q = bo; *q;) {
            ds.push_back(strtoull(q, nullptr, 10) << 20);
            while (*q && *q != ',') q++;
            if (*q == ',') q++;
        }
        const uint64_t base_off = (b.in_bytes + (1ull << 30) - 1) & ~((1ull << 30) - 1);
        const uint64_t dmax = *std::max_element(ds.begin(), ds.end());
        const uint64_t total = base_off + dmax + b.out_bytes;
        uint8_t* big = nullptr;
        const bool contig = hipExtMallocWithFlags((void**)&big, total, hipDeviceMallocContiguous) == hipSuccess;
        if (!contig) CK(hipMalloc(&big, total));
        printf("big allocation %.1f GB, %s\n", total / 1e9, contig ? "contiguous" : "plain hipMalloc");
        mj423::SynthParams sp2 = sp;
        sp2.coef = (int16_t*)big;
        CK(mj423_launch_synth(&sp2, 0));
        CK(hipDeviceSynchronize());
        b.base.coef = (int16_t*)big;
        for (uint64_t d : ds) {
            b.base.out = (uint32_t*)(big + base_off + d);
            char tag[64];
            snprintf(tag, sizeof(tag), "out at +%llu MiB", (unsigned long long)(d >> 20));
            if (b.mode == 420) cases.push_back(b.decode_case<420, 32, 256, 3>(tag, b.fgroup(420, 32)));
            else if (b.mode == 422) cases.push_back(b.decode_case<422, 64, 256, 3>(tag, b.fgroup(422, 64)));
            else cases.push_back(b.decode_case<444, 64, 256, 3>(tag, b.fgroup(444, 64)));
        }
        b.base.coef = b.coef;
        b.base.out = b.out;
    } else if (const char* pe = getenv("PROBE_PAIRS")) {
        // Physical-placement sensitivity: N separately allocated (coefficients, output) pairs,
        // each synthesised, the production batch kernel timed on every pair, interleaved.
        const int n = std::max(1, atoi(pe));
        for (int k = 0; k < n; k++) {
            int16_t* c2 = b.coef;
            uint32_t* o2 = b.out;
            bool contig = false;
            // PROBE_PAIRS_KEEP=coef: every case reads pair 0's coefficients (only the output differs);
            // =out: every case writes pair 0's output (only the coefficients differ)
            const char* keep = getenv("PROBE_PAIRS_KEEP");
            const bool keep_coef = keep && strcmp(keep, "coef") == 0, keep_out = keep && strcmp(keep, "out") == 0;
            if (k > 0) {
                // PROBE_PAIRS_CONTIG=1: odd pairs physically contiguous (hipDeviceMallocContiguous)
                contig = getenv("PROBE_PAIRS_CONTIG") && (k & 1);
                if (contig) {
                    if (hipExtMallocWithFlags((void**)&c2, b.in_bytes, hipDeviceMallocContiguous) != hipSuccess ||
                        hipExtMallocWithFlags((void**)&o2, b.out_bytes, hipDeviceMallocContiguous) != hipSuccess) {
                        printf("pair %d: contiguous allocation refused\n", k);
                        continue;
                    }
                } else {
                    CK(hipMalloc(&c2, b.in_bytes));
                    CK(hipMalloc(&o2, b.out_bytes));
                }
                mj423::SynthParams sp2 = sp;
                sp2.coef = c2;
                CK(mj423_launch_synth(&sp2, 0));
            }
            b.base.coef = keep_coef ? b.coef : c2;
            b.base.out = keep_out ? b.out : o2;
            char tag[64];
            snprintf(tag, sizeof(tag), "pair %d%s", k, contig ? " contiguous" : "");
            if (b.mode == 420 && getenv("PROBE_PAIRS_ORDERS")) {  // placement x workgroup order
                cases.push_back(b.decode_case<420, 32, 256, 3>(tag, b.fgroup(420, 32)));
                cases.push_back(b.decode_case<420, 32, 256, 3>(tag, 8));
                cases.push_back(b.decode_case<420, 32, 256, 3>(tag, 0));
            } else if (b.mode == 420) cases.push_back(b.decode_case<420, 32, 256, 3>(tag, b.fgroup(420, 32)));
            else if (b.mode == 422) cases.push_back(b.decode_case<422, 64, 256, 3>(tag, b.fgroup(422, 64)));
            else cases.push_back(b.decode_case<444, 64, 256, 3>(tag, b.fgroup(444, 64)));
        }
        b.base.coef = b.coef;
        b.base.out = b.out;
        CK(hipDeviceSynchronize());
    } else {
    if (getenv("PROBE_GOP") && getenv("PROBE_GOP_ORDERS")) {
        // stream-kernel workgroup orders on the same buffers: tile (grid), XCD-contiguous jobs, XCD eighths
        b.gop_setup((uint32_t)atoi(getenv("PROBE_GOP")));
        if (b.mode == 420) {
            cases.push_back(b.gop_case<420, 32, 256, 3 | (3 << 26) | 2048 | 8192 | 32768>("order tile"));
            cases.push_back(b.gop_case<420, 32, 256, 3 | (3 << 26) | 2048 | 8192 | 32768 | 262144>("order xcd"));
            cases.push_back(b.gop_case<420, 32, 256, 3 | (3 << 26) | 2048 | 8192 | 32768 | (1 << 22)>("order eighths"));
            cases.push_back(b.gop_case<420, 32, 256, 3 | (3 << 26) | 2048 | 8192 | 32768 | (int)(1u << 31)>("order tile, fair"));
            cases.push_back(b.gop_case<420, 32, 256, 3 | (3 << 26) | 2048 | 8192 | 32768 | 262144 | (int)(1u << 31)>("order xcd, fair"));
            cases.push_back(b.gop_case<420, 32, 256, 3 | (3 << 26) | 2048 | 8192 | 32768 | (1 << 22) | (int)(1u << 31)>("order eighths, fair"));
            cases.push_back(b.gop_case<420, 32, 256, 3 | (3 << 26) | 2048 | 8192 | 32768 | (1 << 24)>("order tile, load priority"));
            cases.push_back(b.gop_case<420, 32, 256, 3 | (3 << 26) | 2048 | 32768 | (1 << 25)>("order tile, scalar-load quant table"));
            cases.push_back(b.gop_case<420, 32, 256, 3 | (3 << 26) | 2048 | 8192 | 32768 | 4>("order tile, ablate-math"));
            cases.push_back(b.gop_case<420, 32, 256, 3 | (3 << 26) | 2048 | 8192 | 32768 | 32>("order tile, ablate-store"));
        } else if (b.mode == 422) {
            cases.push_back(b.gop_case<422, 64, 256, 3 | (3 << 26) | 4096 | 8192 | 32768>("order tile"));
            cases.push_back(b.gop_case<422, 64, 256, 3 | (3 << 26) | 4096 | 8192 | 32768 | 262144>("order xcd"));
            cases.push_back(b.gop_case<422, 64, 256, 3 | (3 << 26) | 4096 | 8192 | 32768 | (1 << 22)>("order eighths"));
            cases.push_back(b.gop_case<422, 64, 256, 3 | (3 << 26) | 4096 | 8192 | 32768 | (int)(1u << 31)>("order tile, fair"));
            cases.push_back(b.gop_case<422, 64, 256, 3 | (3 << 26) | 4096 | 8192 | 32768 | 262144 | (int)(1u << 31)>("order xcd, fair"));
            cases.push_back(b.gop_case<422, 64, 256, 3 | (3 << 26) | 4096 | 8192 | 32768 | (1 << 24)>("order tile, load priority"));
            cases.push_back(b.gop_case<422, 64, 256, 3 | (3 << 26) | 4096 | 32768 | (1 << 25)>("order tile, scalar-load quant table"));
            cases.push_back(b.gop_case<422, 32, 128, 3 | (3 << 26) | 4096 | 8192 | 32768>("order tile, 32-MCU tiles / 128 lanes"));
            cases.push_back(b.gop_case<422, 32, 256, 3 | (3 << 26) | 4096 | 8192 | 32768>("order tile, 32-MCU tiles / 256 lanes"));
            cases.push_back(b.gop_case<422, 64, 256, 3 | (3 << 26) | 4096 | 8192 | 32768 | 4>("order tile, ablate-math"));
            cases.push_back(b.gop_case<422, 64, 256, 3 | (3 << 26) | 4096 | 8192 | 32768 | 32>("order tile, ablate-store"));
        } else {
            cases.push_back(b.gop_case<444, 64, 256, 3 | (3 << 26) | 4096 | 8192 | 32768>("order tile"));
            cases.push_back(b.gop_case<444, 64, 256, 3 | (3 << 26) | 4096 | 8192 | 32768 | 262144>("order xcd"));
            cases.push_back(b.gop_case<444, 64, 256, 3 | (3 << 26) | 4096 | 8192 | 32768 | (1 << 22)>("order eighths"));
            cases.push_back(b.gop_case<444, 64, 256, 3 | (3 << 26) | 4096 | 8192 | 32768 | (int)(1u << 31)>("order tile, fair"));
            cases.push_back(b.gop_case<444, 64, 256, 3 | (3 << 26) | 4096 | 8192 | 32768 | 262144 | (int)(1u << 31)>("order xcd, fair"));
            cases.push_back(b.gop_case<444, 64, 256, 3 | (3 << 26) | 4096 | 8192 | 32768 | (1 << 24)>("order tile, load priority"));
            cases.push_back(b.gop_case<444, 64, 256, 3 | (3 << 26) | 4096 | 32768 | (1 << 25)>("order tile, scalar-load quant table"));
            cases.push_back(b.gop_case<444, 128, 512, 3 | (3 << 26) | 4096 | 8192 | 32768>("order tile, 128-MCU tiles / 512 lanes"));
            cases.push_back(b.gop_case<444, 64, 256, 3 | (3 << 26) | 4096 | 8192 | 32768 | 4>("order tile, ablate-math"));
            cases.push_back(b.gop_case<444, 64, 256, 3 | (3 << 26) | 4096 | 8192 | 32768 | 32>("order tile, ablate-store"));
        }
    } else if (getenv("PROBE_GOP") && getenv("PROBE_ALIGN") && b.mode == 420) {
        // balanced 4:2:0 tiles (production: 30 MCUs = 1920-B rows at 4K and 1080p) against tiles of
        // exactly 32 MCUs (2048-B, 2-KiB aligned rows; the row's last tile 16 / 24 MCUs)
        b.gop_setup((uint32_t)atoi(getenv("PROBE_GOP")));
        for (int a = 0; a < 2; a++) {
            b.align420 = a == 1;
            cases.push_back(b.decode_case<420, 32, 256, 3>(a ? "aligned 32-MCU tiles" : "balanced tiles (production)", b.fgroup(420, 32)));
            cases.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768>(a ? "aligned 32-MCU tiles" : "balanced tiles (production)"));
        }
        b.align420 = false;
    } else if (getenv("PROBE_GOP") && getenv("PROBE_OFFSETS")) {
        // Address-offset sensitivity: the production batch and stream kernels with the output
        // buffer moved by each listed byte offset (< 64 MiB, multiple of 16) against the input.
        b.gop_setup((uint32_t)atoi(getenv("PROBE_GOP")));
        std::string list = getenv("PROBE_OFFSETS");
        uint32_t* const out0 = b.base.out;
        for (size_t pos = 0; pos < list.size();) {
            size_t e = list.find(',', pos);
            if (e == std::string::npos) e = list.size();
            const uint64_t off = strtoull(list.substr(pos, e - pos).c_str(), nullptr, 0) & ~15ull;
            pos = e + 1;
            if (off >= (64ull << 20)) continue;
            b.base.out = out0 + off / 4;
            char tag[96];
            snprintf(tag, sizeof(tag), "out +%llu B", (unsigned long long)off);
            if (b.mode == 420) {
                cases.push_back(b.decode_case<420, 32, 256, 3>(tag, b.fgroup(420, 32)));
                cases.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768>(tag));
            } else if (b.mode == 422) {
                cases.push_back(b.decode_case<422, 64, 256, 3>(tag, b.fgroup(422, 64)));
                cases.push_back(b.gop_case<422, 64, 256, 3 | 4096 | 8192 | 32768>(tag));
            } else {
                cases.push_back(b.decode_case<444, 64, 256, 3>(tag, b.fgroup(444, 64)));
                cases.push_back(b.gop_case<444, 64, 256, 3 | 4096 | 8192 | 32768>(tag));
            }
        }
        b.base.out = out0;
    } else if (getenv("PROBE_R03")) {  // round 3: int16-workspace IDCT and 16-bit CSC vs the round-2 forms
        // 1 << 26 = kIdctI32 (int32 workspace always), 1 << 27 = kCscI32 (round-2 4:2:x CSC)
        constexpr int I = 1 << 26, C = 1 << 27, XO = mj423::kFgroupXcd;
        if (b.mode == 420) {
            cases.push_back(b.decode_case<420, 32, 256, 3>("(round 3)", XO));
            cases.push_back(b.decode_case<420, 32, 256, 3 | I>("int32 IDCT", XO));
            cases.push_back(b.decode_case<420, 32, 256, 3 | C>("round-2 CSC", XO));
            cases.push_back(b.decode_case<420, 32, 256, 3 | I | C>("(round 2)", XO));
        } else if (b.mode == 422) {
            cases.push_back(b.decode_case<422, 64, 256, 3>("(round 3)", XO));
            cases.push_back(b.decode_case<422, 64, 256, 3 | I | C>("(round 2)", XO));
        } else {
            cases.push_back(b.decode_case<444, 64, 256, 3>("(round 3)", XO));
            cases.push_back(b.decode_case<444, 64, 256, 3 | I>("(round 2)", XO));
        }
        if (getenv("PROBE_GOP")) {
            b.gop_setup((uint32_t)atoi(getenv("PROBE_GOP")));
            constexpr int W = 1 << 28;  // kIdctW16Only
            constexpr int S8 = 1 << 29;  // kGopState8
            constexpr int GI = I | C;    // the stream kernel's production transform + CSC
            if (getenv("PROBE_BPRIO")) {  // batch kernel: raised wave priority at load issue / during the CSC
                const uint32_t fg = b.fgroup(b.mode, b.mode == 420 ? 32 : 64);
                if (b.mode == 420) {
                    cases.push_back(b.decode_case<420, 32, 256, 3>("(production)", fg));
                    cases.push_back(b.decode_case<420, 32, 256, 3 | 2048>("priority at load issue", fg));
                    cases.push_back(b.decode_case<420, 32, 256, 3 | 4096>("priority during CSC", fg));
                    cases.push_back(b.decode_case<420, 32, 256, 3 | 2048 | 4096>("both", fg));
                } else if (b.mode == 422) {
                    cases.push_back(b.decode_case<422, 64, 256, 3>("(production)", fg));
                    cases.push_back(b.decode_case<422, 64, 256, 3 | 2048>("priority at load issue", fg));
                    cases.push_back(b.decode_case<422, 64, 256, 3 | 4096>("priority during CSC", fg));
                } else {
                    cases.push_back(b.decode_case<444, 64, 256, 3>("(production)", fg));
                    cases.push_back(b.decode_case<444, 64, 256, 3 | 2048>("priority at load issue", fg));
                    cases.push_back(b.decode_case<444, 64, 256, 3 | 4096>("priority during CSC", fg));
                }
            } else
            if (getenv("PROBE_CHAIN")) {  // one-shot chain stream kernel (state handed between workgroups) vs production
                const uint32_t L = (uint32_t)atoi(getenv("PROBE_GOP"));
                if (b.NF % L) { printf("PROBE_CHAIN needs frames %% GOP == 0\n"); return 1; }
                const uint32_t Bt = getenv("PROBE_CHAIN_B") ? (uint32_t)atoi(getenv("PROBE_CHAIN_B")) : 120;
                mj423::DecodeParams qc = b.persist_params<420, 32>();
                const uint32_t tpf = qc.tiles_per_frame, nseg = b.NF / L, nb = (tpf + Bt - 1) / Bt, U = nseg * nb;
                const uint32_t grid = 8 * ((U + 7) / 8) * L * Bt;
                using TT = mj423::Tile<420, 32, 256>;
                u32x4* rec = nullptr;
                uint32_t* fl = nullptr;
                CK(hipMalloc(&rec, (size_t)nseg * tpf * TT::CHUNKS * 256 * 16));
                CK(hipMalloc(&fl, (size_t)nseg * tpf * 4));
                printf("chain: %u tiles per frame, bands of %u tiles (%u per frame), %u units, grid %u\n", tpf, Bt, nb, U, grid);
                Case chainc{"chain kernel (one-shot, state handed over)", (double)(b.in_bytes + b.out_bytes), [=] {
                                CK(hipMemsetAsync(fl, 0, (size_t)nseg * tpf * 4, 0));
                                hipLaunchKernelGGL((mj423::decode_chain_kernel<420, 32, 256, 3>), dim3(grid), dim3(256), 0, 0, qc, rec, fl,
                                                   Bt, L, nb, U);
                            }};
                Case prod = b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768 | GI>("stream kernel (production)");
                // correctness: production into b.out, the chain kernel into a second buffer
                uint32_t* out2 = nullptr;
                unsigned long long* bad = nullptr;
                CK(hipMalloc(&out2, b.out_bytes));
                CK(hipMalloc(&bad, 8));
                CK(hipMemset(b.out, 0, b.out_bytes));
                prod.f();
                mj423::DecodeParams q2 = qc;
                q2.out = out2;
                CK(hipMemset(out2, 0xff, b.out_bytes));
                CK(hipMemset(fl, 0, (size_t)nseg * tpf * 4));
                hipLaunchKernelGGL((mj423::decode_chain_kernel<420, 32, 256, 3>), dim3(grid), dim3(256), 0, 0, q2, rec, fl, Bt, L, nb, U);
                CK(hipDeviceSynchronize());
                CK(hipMemset(bad, 0, 8));
                hipLaunchKernelGGL(count_diff, dim3(4096), dim3(256), 0, 0, (const u32x4*)b.out, (const u32x4*)out2, (size_t)(b.out_bytes / 16), bad);
                unsigned long long nbad = 0;
                CK(hipMemcpy(&nbad, bad, 8, hipMemcpyDeviceToHost));
                printf("chain kernel vs production: %llu differing dwords of %llu\n", nbad, (unsigned long long)(b.out_bytes / 4));
                CK(hipFree(out2));
                cases.push_back(b.decode_case<420, 32, 256, 3>("batch one-shot (production)", mj423::kFgroupXcd));
                cases.push_back(prod);
                cases.push_back(chainc);
            } else
            if (getenv("PROBE_FPAD")) {  // frame-stride padding: batch, one-shot orders, stream (4:2:0)
                if (b.mode != 420) { printf("PROBE_FPAD: 4:2:0 only\n"); return 1; }
                printf("frame padding %llu bytes\n", (unsigned long long)fpad);
                constexpr int PAD = 65536, I32 = 3 << 26, FAIR = (int)(1u << 31);
                const mj423::DecodeParams qa = b.persist_params<420, 32>();
                const uint32_t Tf = qa.tiles_per_frame, E = (Tf + 7) / 8, nf = b.NF;
                auto k4 = mj423::decode_order_kernel<420, 32, 256, 3 | PAD | I32>;
                auto k6 = mj423::decode_order_kernel<420, 32, 256, 3>;
                cases.push_back(b.decode_case<420, 32, 256, 3>("one-shot (production)", mj423::kFgroupXcd));
                cases.push_back(b.decode_case<420, 32, 256, 3>("one-shot, frame-major"));
                cases.push_back({"one-shot production, bands", (double)(b.in_bytes + b.out_bytes), [=] {
                                     hipLaunchKernelGGL(k6, dim3(8 * E * nf), dim3(256), 0, 0, qa, 2u, nf, 0u);
                                 }});
                const uint32_t G = 128;
                const uint32_t nw = 8 * ((E + G - 1) / G) * G * nf;
                cases.push_back({"one-shot 4/CU int32, band walks G=128", (double)(b.in_bytes + b.out_bytes), [=] {
                                     hipLaunchKernelGGL(k4, dim3(nw), dim3(256), 0, 0, qa, 4u, nf, G);
                                 }});
                const uint32_t nw5 = 8 * ((Tf + G - 1) / G) * G * ((nf + 7) / 8);
                cases.push_back({"one-shot production, distant band walks G=128", (double)(b.in_bytes + b.out_bytes), [=] {
                                     hipLaunchKernelGGL(k6, dim3(nw5), dim3(256), 0, 0, qa, 5u, nf, G);
                                 }});
                cases.push_back({"one-shot 4/CU int32, distant band walks G=128", (double)(b.in_bytes + b.out_bytes), [=] {
                                     hipLaunchKernelGGL(k4, dim3(nw5), dim3(256), 0, 0, qa, 5u, nf, G);
                                 }});
                cases.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768 | GI>("stream kernel (production)"));
                cases.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768 | GI | FAIR>("stream kernel, frames-left priority"));
                cases.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768 | GI | 262144>("stream kernel, XCD-contiguous jobs"));
            } else
            if (getenv("PROBE_ORDERS")) {  // one-shot batch body under stream-like workgroup orders (decode_order_kernel)
                if (b.mode != 420) { printf("PROBE_ORDERS: 4:2:0 only\n"); return 1; }
                constexpr int PAD = 65536, I32 = 3 << 26;
                const mj423::DecodeParams qa = b.persist_params<420, 32>();
                const uint32_t Tf = qa.tiles_per_frame, E = (Tf + 7) / 8, nf = b.NF;
                auto order_case = [&](auto kern, const char* nm, uint32_t order, uint32_t G) -> Case {
                    uint64_t n = order == 2 ? 8ull * E * nf : order == 3 ? 8ull * Tf * ((nf + 7) / 8)
                                                                          : 8ull * ((E + G - 1) / G) * G * nf;
                    return {nm, (double)(b.in_bytes + b.out_bytes), [=] {
                                hipLaunchKernelGGL(kern, dim3((uint32_t)n), dim3(256), 0, 0, qa, order, nf, G);
                            }};
                };
                auto k4 = mj423::decode_order_kernel<420, 32, 256, 3 | PAD | I32>;
                auto k6 = mj423::decode_order_kernel<420, 32, 256, 3>;
                std::vector<Case> ord = {
                    order_case(k4, "one-shot 4/CU int32, bands (XCD x: eighth x of every frame)", 2, 0),
                    order_case(k4, "one-shot 4/CU int32, whole frames per XCD", 3, 0),
                    order_case(k4, "one-shot 4/CU int32, band walks G=128 (stream-like)", 4, 128),
                    order_case(k4, "one-shot 4/CU int32, band walks G=32", 4, 32),
                    order_case(k6, "one-shot production, bands", 2, 0),
                    order_case(k6, "one-shot production, band walks G=192", 4, 192),
                };
                // coverage check: every order writes the same frames as production
                uint32_t* out0 = b.base.out;
                uint32_t* out2 = nullptr;
                unsigned long long* bad = nullptr;
                CK(hipMalloc(&out2, b.out_bytes));
                CK(hipMalloc(&bad, 8));
                b.decode_case<420, 32, 256, 3>("check", mj423::kFgroupXcd).f();
                for (size_t k = 0; k < ord.size(); k++) {
                    mj423::DecodeParams q2 = qa;
                    q2.out = out2;
                    CK(hipMemset(out2, 0xff, b.out_bytes));
                    const uint32_t order = k == 0 || k == 4 ? 2 : k == 1 ? 3 : 4, G = k == 2 ? 128 : k == 3 ? 32 : 192;
                    const uint64_t n = order == 2 ? 8ull * E * nf : order == 3 ? 8ull * Tf * ((nf + 7) / 8)
                                                                               : 8ull * ((E + G - 1) / G) * G * nf;
                    if (k < 4)
                        hipLaunchKernelGGL(k4, dim3((uint32_t)n), dim3(256), 0, 0, q2, order, nf, G);
                    else
                        hipLaunchKernelGGL(k6, dim3((uint32_t)n), dim3(256), 0, 0, q2, order, nf, G);
                    CK(hipDeviceSynchronize());
                    CK(hipMemset(bad, 0, 8));
                    hipLaunchKernelGGL(count_diff, dim3(4096), dim3(256), 0, 0, (const u32x4*)out0, (const u32x4*)out2,
                                       (size_t)(b.out_bytes / 16), bad);
                    unsigned long long nbad = 0;
                    CK(hipMemcpy(&nbad, bad, 8, hipMemcpyDeviceToHost));
                    printf("%s vs production: %llu differing dwords\n", ord[k].name.c_str(), nbad);
                    if (nbad) return 1;
                }
                CK(hipFree(out2));
                cases.push_back(b.decode_case<420, 32, 256, 3>("one-shot (production)", mj423::kFgroupXcd));
                cases.push_back(b.decode_case<420, 32, 256, 3 | PAD | I32>("one-shot, 4 per CU, int32 forms", mj423::kFgroupXcd));
                cases.push_back(b.decode_case<420, 32, 256, 3 | PAD | I32>("one-shot, 4 per CU, int32 forms, frame-major"));
                cases.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768 | GI>("stream kernel (production)"));
                for (auto& c : ord) cases.push_back(c);
            } else
            if (getenv("PROBE_PERSIST")) {  // batch kernel one-shot vs persistent (a loop per workgroup, like the stream kernel)
                // all at the stream kernel's LDS (kPadLds: four per CU) and transform/CSC forms (int32)
                constexpr int PAD = 65536, I32 = 3 << 26;
                if (b.mode == 420) {
                    cases.push_back(b.decode_case<420, 32, 256, 3>("one-shot (production)", mj423::kFgroupXcd));
                    cases.push_back(b.decode_case<420, 32, 256, 3 | PAD | I32>("one-shot, 4 per CU, int32 forms", mj423::kFgroupXcd));
                    cases.push_back(b.decode_case<420, 32, 256, 3 | PAD | I32>("one-shot, 4 per CU, int32 forms, frame-major"));
                    cases.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768 | GI>("stream kernel (production)"));
                    const mj423::DecodeParams qa = b.persist_params<420, 32>();
                    const uint32_t G = 256 * 4;
                    cases.push_back({"persistent, grid stride, 4 per CU, int32 forms", (double)(b.in_bytes + b.out_bytes), [qa, G] {
                                         hipLaunchKernelGGL((mj423::decode_kernel<420, 32, 256, 3 | 16 | PAD | I32>), dim3(G), dim3(256), 0, 0, qa);
                                     }});
                    cases.push_back({"persistent, XCD eighths, 4 per CU, int32 forms", (double)(b.in_bytes + b.out_bytes), [qa, G] {
                                         hipLaunchKernelGGL((mj423::decode_kernel<420, 32, 256, 3 | 16 | 64 | PAD | I32>), dim3(G), dim3(256), 0, 0, qa);
                                     }});
                }
            } else
            if (getenv("PROBE_TRACE")) {  // per-frame phase timestamps of the stream kernel (kGopTrace)
                constexpr int TR = 1 << 19, OPT = 3 | 32768 | S8 | (1 << 30) | 2048;
                const uint32_t tpf = b.mode == 420 ? b.base.mcu_rows * ((b.base.mcu_cols + 31) / 32)
                                                   : (b.base.mcu_cols * b.base.mcu_rows + 63) / 64;
                const uint32_t jobs = tpf * b.nseg;
                const size_t rec = 1 + 4 * 32;
                uint64_t* tr = nullptr;
                uint32_t* jf = nullptr;
                CK(hipMalloc(&tr, (size_t)jobs * rec * 8));
                CK(hipMalloc(&jf, (size_t)jobs * 4 + 16));
                CK(hipMemset(jf, 0, (size_t)jobs * 4 + 16));
                b.base.trace = tr;
                b.base.jobflag = jf;
                std::vector<Case> v;
                if (b.mode == 420) {
                    v.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768 | GI | TR>("production"));
                    v.push_back(b.gop_case<420, 32, 256, OPT | 8192 | TR>("optimistic, 6 per CU"));
                    v.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768 | GI | TR | (int)(1u << 31)>("production, fair priority"));
                } else if (b.mode == 422) {
                    v.push_back(b.gop_case<422, 64, 256, 3 | 4096 | 8192 | 32768 | GI | TR>("production"));
                    v.push_back(b.gop_case<422, 64, 256, OPT | (1 << 25) | TR>("optimistic, 5 per CU"));
                } else {
                    v.push_back(b.gop_case<444, 64, 256, 3 | 4096 | 8192 | 32768 | GI | TR>("production"));
                    v.push_back(b.gop_case<444, 64, 256, OPT | 8192 | TR>("optimistic, 6 per CU"));
                    v.push_back(b.gop_case<444, 64, 256, 3 | 4096 | 8192 | 32768 | GI | TR | (int)(1u << 31)>("production, fair priority"));
                }
                {  // the batch kernel (XCD-contiguous order) on the same frames: one tile per workgroup
                    std::vector<Case> bc;
                    if (b.mode == 420) bc.push_back(b.decode_case<420, 32, 256, 3 | TR>("batch", mj423::kFgroupXcd));
                    else if (b.mode == 422) bc.push_back(b.decode_case<422, 64, 256, 3 | TR>("batch", mj423::kFgroupXcd));
                    else bc.push_back(b.decode_case<444, 64, 256, 3 | TR>("batch", mj423::kFgroupXcd));
                    const uint32_t nwg = 8 * ((tpf * b.NF + 7) / 8);
                    uint64_t* bt = nullptr;
                    CK(hipMalloc(&bt, (size_t)nwg * 5 * 8));
                    b.base.trace = bt;
                    bc.clear();
                    if (b.mode == 420) bc.push_back(b.decode_case<420, 32, 256, 3 | TR>("batch", mj423::kFgroupXcd));
                    else if (b.mode == 422) bc.push_back(b.decode_case<422, 64, 256, 3 | TR>("batch", mj423::kFgroupXcd));
                    else bc.push_back(b.decode_case<444, 64, 256, 3 | TR>("batch", mj423::kFgroupXcd));
                    b.base.trace = tr;
                    for (int w = 0; w < 3; w++) bc[0].f();
                    CK(hipMemset(bt, 0, (size_t)nwg * 5 * 8));
                    CK(hipDeviceSynchronize());
                    bc[0].f();
                    CK(hipDeviceSynchronize());
                    std::vector<uint64_t> hb((size_t)nwg * 5);
                    CK(hipMemcpy(hb.data(), bt, hb.size() * 8, hipMemcpyDeviceToHost));
                    std::vector<double> ph[3];
                    for (uint32_t i = 0; i < nwg; i++) {
                        const uint64_t* r = &hb[(size_t)i * 5];
                        if (!r[1] || !r[4]) continue;
                        for (int k = 0; k < 3; k++) ph[k].push_back((double)(r[k + 2] - r[k + 1]) * 0.48e-3);
                    }
                    for (int k = 0; k < 3; k++) std::sort(ph[k].begin(), ph[k].end());
                    if (!ph[0].empty())
                        printf("trace batch kernel: per tile (median us, tick ~0.48 ns): load+stage %.2f  IDCT %.2f  CSC %.2f "
                               "(p90 %.2f / %.2f / %.2f)\n", ph[0][ph[0].size() / 2], ph[1][ph[1].size() / 2], ph[2][ph[2].size() / 2],
                               ph[0][ph[0].size() * 9 / 10], ph[1][ph[1].size() * 9 / 10], ph[2][ph[2].size() * 9 / 10]);
                    CK(hipFree(bt));
                }
                std::vector<uint64_t> h((size_t)jobs * rec);
                for (auto& c : v) {
                    for (int w = 0; w < 3; w++) c.f();  // warm
                    CK(hipMemset(tr, 0, h.size() * 8));
                    hipEvent_t a0, a1;
                    CK(hipEventCreate(&a0));
                    CK(hipEventCreate(&a1));
                    CK(hipEventRecord(a0, 0));
                    c.f();
                    CK(hipEventRecord(a1, 0));
                    CK(hipEventSynchronize(a1));
                    float ms = 0;
                    CK(hipEventElapsedTime(&ms, a0, a1));
                    CK(hipMemcpy(h.data(), tr, h.size() * 8, hipMemcpyDeviceToHost));
                    // per-frame phase durations (ticks): wait+stage, IDCT, CSC issue, loop back
                    std::vector<double> ph[4], period;
                    uint64_t tmin = ~0ull, tmax = 0;
                    std::map<uint64_t, std::vector<std::array<uint64_t, 4>>> percu;  // CU -> frame intervals
                    for (uint32_t j = 0; j < jobs; j++) {
                        const uint64_t* r = &h[(size_t)j * rec];
                        const uint32_t id = (uint32_t)r[0], xcc = (uint32_t)(r[0] >> 32) & 0xf;
                        const uint64_t cu = ((uint64_t)xcc << 16) | (((id >> 13) & 7) << 12) | (((id >> 12) & 1) << 8) | ((id >> 8) & 0xf);
                        for (int f = 0; f < 32; f++) {
                            const uint64_t* t = r + 1 + 4 * f;
                            if (!t[0] || !t[3]) break;
                            ph[0].push_back((double)(t[1] - t[0]));
                            ph[1].push_back((double)(t[2] - t[1]));
                            ph[2].push_back((double)(t[3] - t[2]));
                            if (f + 1 < 32 && t[4]) {
                                ph[3].push_back((double)(t[4] - t[3]));
                                period.push_back((double)(t[4] - t[0]));
                            }
                            percu[cu].push_back({t[0], t[1], t[2], t[3]});
                            tmin = std::min(tmin, t[0]);
                            tmax = std::max(tmax, t[3]);
                        }
                    }
                    auto med = [](std::vector<double> x) {
                        if (x.empty()) return 0.0;
                        std::sort(x.begin(), x.end());
                        return x[x.size() / 2];
                    };
                    auto mean = [](const std::vector<double>& x) {
                        double s = 0;
                        for (double y : x) s += y;
                        return x.empty() ? 0.0 : s / x.size();
                    };
                    // average number of this CU's workgroups in each phase (time-weighted over the CU's busy span)
                    double occ[3] = {0, 0, 0}, span = 0;
                    std::vector<double> spans;  // s_memtime counters differ between XCDs: scale per CU
                    for (auto& kv : percu) {
                        uint64_t lo = ~0ull, hi = 0;
                        double in[3] = {0, 0, 0};
                        for (auto& t : kv.second) {
                            lo = std::min(lo, t[0]);
                            hi = std::max(hi, t[3]);
                            for (int k = 0; k < 3; k++) in[k] += (double)(t[k + 1] - t[k]);
                        }
                        for (int k = 0; k < 3; k++) occ[k] += in[k];
                        span += (double)(hi - lo);
                        spans.push_back((double)(hi - lo));
                    }
                    (void)tmin;
                    (void)tmax;
                    std::sort(spans.begin(), spans.end());
                    const double tick_ns = ms * 1e6 / spans[spans.size() - 1];  // the longest CU span ~ the kernel
                    // by frame index within the job: mean duration of each phase (startup and tail effects)
                    {
                        double sum[32][4] = {}, cnt[32] = {};
                        for (uint32_t j = 0; j < jobs; j++) {
                            const uint64_t* r = &h[(size_t)j * rec];
                            for (int f = 0; f < 32; f++) {
                                const uint64_t* t = r + 1 + 4 * f;
                                if (!t[0] || !t[3]) break;
                                for (int k = 0; k < 3; k++) sum[f][k] += (double)(t[k + 1] - t[k]);
                                if (f + 1 < 32 && t[4]) sum[f][3] += (double)(t[4] - t[0]);
                                cnt[f]++;
                            }
                        }
                        printf("trace %s by frame (mean us: wait+stage / IDCT / CSC / period):", c.name.c_str());
                        for (int f = 0; f < 32 && cnt[f] > 0; f++)
                            if (f < 3 || f % 6 == 5 || f >= 22)
                                printf(" f%d %.2f/%.2f/%.2f/%.2f", f, sum[f][0] / cnt[f] * tick_ns * 1e-3, sum[f][1] / cnt[f] * tick_ns * 1e-3,
                                       sum[f][2] / cnt[f] * tick_ns * 1e-3, sum[f][3] / cnt[f] * tick_ns * 1e-3);
                        printf("\n");
                        // per CU: jobs held and busy span (load balance of a one-round grid)
                        std::map<size_t, std::pair<double, int>> byjobs;  // frames on the CU -> (sum of spans, CUs)
                        for (auto& kv : percu) {
                            uint64_t lo = ~0ull, hi = 0;
                            for (auto& t : kv.second) {
                                lo = std::min(lo, t[0]);
                                hi = std::max(hi, t[3]);
                            }
                            auto& e = byjobs[kv.second.size()];
                            e.first += (double)(hi - lo) * tick_ns * 1e-3;
                            e.second++;
                        }
                        printf("trace %s CU span by tile-frames on the CU (frames: CUs, mean us):", c.name.c_str());
                        for (auto& kv : byjobs) printf(" %zu: %d, %.1f;", kv.first, kv.second.second, kv.second.first / kv.second.second);
                        printf("\n");
                    }
                    printf("trace %-26s %.3f ms, %zu CUs, tick %.3f ns; per frame (median us): wait+stage %.2f  IDCT %.2f  "
                           "CSC %.2f  back %.2f  period %.2f (mean %.2f); workgroups per CU in each phase: %.2f %.2f %.2f\n",
                           c.name.c_str(), ms, percu.size(), tick_ns, med(ph[0]) * tick_ns / 1e3, med(ph[1]) * tick_ns / 1e3,
                           med(ph[2]) * tick_ns / 1e3, med(ph[3]) * tick_ns / 1e3, med(period) * tick_ns / 1e3,
                           mean(period) * tick_ns / 1e3, occ[0] / span, occ[1] / span, occ[2] / span);
                }
                return 0;
            }
            if (getenv("PROBE_OPT")) {  // optimistic stream kernel (+ the exact re-run of marked jobs) vs production
                // kGopOpt* of mj423_kernels.hip: int8 state, int16 IDCT with escape, 16-bit CSC, prefetch
                constexpr int OPT = 3 | 32768 | S8 | (1 << 30) | 2048, FIX = 32768 | (1 << 21), LQ = 8192, SQ = 1 << 25;
                const uint32_t tpf = b.mode == 420 ? b.base.mcu_rows * ((b.base.mcu_cols + 31) / 32)
                                                   : (b.base.mcu_cols * b.base.mcu_rows + 63) / 64;
                const size_t fbytes = ((size_t)tpf * b.nseg * 4 + 15) / 16 * 16;
                uint32_t* jf = nullptr;
                uint32_t* zero = nullptr;
                CK(hipMalloc(&jf, fbytes));
                CK(hipMalloc(&zero, fbytes));
                CK(hipMemset(jf, 0, fbytes));
                CK(hipMemset(zero, 0, fbytes));
                b.base.jobflag = jf;
                uint32_t* out0 = b.base.out;
                uint32_t* out2 = nullptr;
                unsigned long long* bad = nullptr;
                CK(hipMalloc(&out2, b.out_bytes));
                CK(hipMalloc(&bad, 8));
                // variants: production, exact forms, optimistic forms (index 2 = the re-run pass)
                constexpr int E = 4096, P = 2048, W5 = 1024, CP = 1 << 20, FAIR = (int)(1u << 31);
                auto variants = [&](std::vector<Case>& v) {
                    constexpr int LW = 65536;  // kGopEntryWait: first frame's loads waited for before the loop
                    if (getenv("PROBE_WAIT")) {  // the loop-header wait: stores drained every frame (production) or left in flight (LW)
                        if (b.mode == 420) {
                            v.push_back(b.gop_case<420, 32, 256, 3 | P | LQ | 32768 | GI>("(production)"));
                            v.push_back(b.gop_case<420, 32, 256, 3 | P | LQ | 32768 | GI | LW>("stores left in flight"));
                            v.push_back(b.gop_case<420, 32, 256, 3 | P | LQ | GI | FIX>("re-run pass (nothing marked)"));
                            v.push_back(b.gop_case<420, 32, 256, 3 | P | LQ | 32768 | GI | FAIR>("priority by frames left"));
                            v.push_back(b.gop_case<420, 32, 256, 3 | P | LQ | 32768 | GI | FAIR | LW>("priority by frames left, stores in flight"));
                            v.push_back(b.gop_case<420, 32, 256, OPT | LQ>("optimistic, 6 per CU"));
                            v.push_back(b.gop_case<420, 32, 256, OPT | LQ | LW>("optimistic, 6 per CU, stores in flight"));
                        } else if (b.mode == 422) {
                            v.push_back(b.gop_case<422, 64, 256, 3 | E | LQ | 32768 | GI>("(production)"));
                            v.push_back(b.gop_case<422, 64, 256, 3 | E | LQ | 32768 | GI | LW>("stores left in flight"));
                            v.push_back(b.gop_case<422, 64, 256, 3 | E | LQ | GI | FIX>("re-run pass (nothing marked)"));
                            v.push_back(b.gop_case<422, 64, 256, OPT | SQ>("optimistic, 5 per CU"));
                            v.push_back(b.gop_case<422, 64, 256, OPT | SQ | LW>("optimistic, 5 per CU, stores in flight"));
                            v.push_back(b.gop_case<422, 64, 256, OPT | SQ | FAIR>("optimistic, priority by frames left"));
                            v.push_back(b.gop_case<422, 64, 256, OPT | SQ | FAIR | LW>("optimistic, priority by frames left, stores in flight"));
                        } else {
                            v.push_back(b.gop_case<444, 64, 256, 3 | E | LQ | 32768 | GI>("(production)"));
                            v.push_back(b.gop_case<444, 64, 256, 3 | E | LQ | 32768 | GI | LW>("stores left in flight"));
                            v.push_back(b.gop_case<444, 64, 256, 3 | E | LQ | GI | FIX>("re-run pass (nothing marked)"));
                            v.push_back(b.gop_case<444, 64, 256, 3 | E | LQ | 32768 | GI | FAIR>("priority by frames left"));
                            v.push_back(b.gop_case<444, 64, 256, 3 | E | LQ | 32768 | GI | FAIR | LW>("priority by frames left, stores in flight"));
                            v.push_back(b.gop_case<444, 64, 256, OPT | LQ>("optimistic, 6 per CU"));
                            v.push_back(b.gop_case<444, 64, 256, OPT | LQ | LW>("optimistic, 6 per CU, stores in flight"));
                        }
                        return;
                    }
                    if (getenv("PROBE_LOCK")) {  // groups of G jobs per XCD band in loose lock step (kGopLockstep)
                        constexpr int EI = 1 << 22, LK = 64;
                        uint32_t* cnt = nullptr;  // group counters, zeroed before each launch
                        const size_t cb = (size_t)b.nseg * 8 * 1024 * 4;
                        CK(hipMalloc(&cnt, cb));
                        auto wrap = [cnt, cb](Case cs) {
                            const auto f0 = cs.f;
                            cs.f = [f0, cnt, cb] { CK(hipMemsetAsync(cnt, 0, cb, 0)); f0(); };
                            return cs;
                        };
                        if (b.mode == 420) {
                            v.push_back(b.gop_case<420, 32, 256, 3 | P | LQ | 32768 | GI>("(production)"));
                            v.push_back(b.gop_case<420, 32, 256, 3 | P | LQ | 32768 | GI | EI>("eighths"));
                            v.push_back(b.gop_case<420, 32, 256, 3 | P | LQ | GI | FIX>("re-run pass (nothing marked)"));
                            for (auto gd : {std::pair<uint32_t, uint32_t>{128, 2}, {128, 1}, {64, 2}, {32, 2}, {128, 4}}) {
                                char nm[80];
                                snprintf(nm, sizeof(nm), "eighths, lock step G=%u D=%u", gd.first, gd.second);
                                b.base.stagger = gd.first | (gd.second << 16);  // gop_case copies base
                                b.base.trace = reinterpret_cast<uint64_t*>(cnt);
                                v.push_back(wrap(b.gop_case<420, 32, 256, 3 | P | LQ | 32768 | GI | EI | LK>(strdup(nm))));
                            }
                            b.base.stagger = 0;
                            b.base.trace = nullptr;
                            v.push_back(b.gop_case<420, 32, 256, 3 | P | LQ | 32768 | GI | FAIR>("priority by frames left"));
                        } else if (b.mode == 444) {
                            v.push_back(b.gop_case<444, 64, 256, 3 | E | LQ | 32768 | GI>("(production)"));
                            v.push_back(b.gop_case<444, 64, 256, 3 | E | LQ | 32768 | GI | EI>("eighths"));
                            v.push_back(b.gop_case<444, 64, 256, 3 | E | LQ | GI | FIX>("re-run pass (nothing marked)"));
                            for (auto gd : {std::pair<uint32_t, uint32_t>{128, 2}, {64, 2}}) {
                                char nm[80];
                                snprintf(nm, sizeof(nm), "eighths, lock step G=%u D=%u", gd.first, gd.second);
                                b.base.stagger = gd.first | (gd.second << 16);
                                b.base.trace = reinterpret_cast<uint64_t*>(cnt);
                                v.push_back(wrap(b.gop_case<444, 64, 256, 3 | E | LQ | 32768 | GI | EI | LK>(strdup(nm))));
                            }
                            b.base.stagger = 0;
                            b.base.trace = nullptr;
                            v.push_back(b.gop_case<444, 64, 256, 3 | E | LQ | 32768 | GI | FAIR>("priority by frames left"));
                        } else {
                            printf("PROBE_LOCK: 4:2:0 / 4:4:4\n");
                            exit(1);
                        }
                        return;
                    }
                    if (getenv("PROBE_EARLY420")) {  // 4:2:0: next frame's loads before the IDCT (kGopEarly) vs after it
                        constexpr int LW = 65536;
                        v.push_back(b.gop_case<420, 32, 256, 3 | P | LQ | 32768 | GI>("(production: loads after the IDCT)"));
                        v.push_back(b.gop_case<420, 32, 256, 3 | E | LQ | 32768 | GI>("loads before the IDCT"));
                        v.push_back(b.gop_case<420, 32, 256, 3 | P | LQ | GI | FIX>("re-run pass (nothing marked)"));
                        v.push_back(b.gop_case<420, 32, 256, 3 | E | LQ | 32768 | GI | LW>("loads before the IDCT, stores in flight"));
                        v.push_back(b.gop_case<420, 32, 256, 3 | P | LQ | 32768 | GI | FAIR>("loads after, frames-left priority"));
                        v.push_back(b.gop_case<420, 32, 256, 3 | E | LQ | 32768 | GI | FAIR>("loads before, frames-left priority"));
                        v.push_back(b.gop_case<420, 32, 256, 3 | E | LQ | 32768>("loads before, int16 IDCT + 16-bit CSC"));
                        return;
                    }
                    if (getenv("PROBE_S8X")) {  // int8 state with the exact int32 transform + CSC (only int8 overflow escapes)
                        constexpr int S8X = 3 | 32768 | S8 | GI | P;
                        if (b.mode == 420) {
                            v.push_back(b.gop_case<420, 32, 256, 3 | P | LQ | 32768 | GI>("(production)"));
                            v.push_back(b.gop_case<420, 32, 256, S8X | LQ>("int8 state, int32 forms, 6 per CU"));
                            v.push_back(b.gop_case<420, 32, 256, 3 | P | LQ | GI | FIX>("re-run pass (nothing marked)"));
                            v.push_back(b.gop_case<420, 32, 256, S8X | LQ | W5>("int8 state, int32 forms, 5 per CU"));
                            v.push_back(b.gop_case<420, 32, 256, S8X | SQ>("int8 state, int32 forms, smem qt, 6 per CU"));
                            v.push_back(b.gop_case<420, 32, 256, OPT | LQ>("optimistic (int16 forms), 6 per CU"));
                            v.push_back(b.gop_case<420, 32, 256, 3 | P | LQ | 32768 | GI | FAIR>("priority by frames left"));
                            v.push_back(b.gop_case<420, 32, 256, S8X | LQ | FAIR>("int8 state, int32 forms, 6 per CU, frames-left priority"));
                        } else if (b.mode == 422) {
                            v.push_back(b.gop_case<422, 64, 256, 3 | E | LQ | 32768 | GI>("(production, exact)"));
                            v.push_back(b.gop_case<422, 64, 256, S8X | SQ>("int8 state, int32 forms, 5 per CU"));
                            v.push_back(b.gop_case<422, 64, 256, 3 | E | LQ | GI | FIX>("re-run pass (nothing marked)"));
                            v.push_back(b.gop_case<422, 64, 256, OPT | SQ>("optimistic (int16 forms, production), 5 per CU"));
                            v.push_back(b.gop_case<422, 64, 256, S8X | SQ | FAIR>("int8 state, int32 forms, frames-left priority"));
                            v.push_back(b.gop_case<422, 64, 256, OPT | SQ | FAIR>("optimistic, frames-left priority"));
                        } else {
                            v.push_back(b.gop_case<444, 64, 256, 3 | E | LQ | 32768 | GI>("(production)"));
                            v.push_back(b.gop_case<444, 64, 256, S8X | LQ>("int8 state, int32 forms, 6 per CU"));
                            v.push_back(b.gop_case<444, 64, 256, 3 | E | LQ | GI | FIX>("re-run pass (nothing marked)"));
                            v.push_back(b.gop_case<444, 64, 256, S8X | LQ | W5>("int8 state, int32 forms, 5 per CU"));
                            v.push_back(b.gop_case<444, 64, 256, (S8X & ~P) | E | LQ>("int8 state, int32 forms, early, 6 per CU"));
                            v.push_back(b.gop_case<444, 64, 256, 3 | E | LQ | 32768 | GI | FAIR>("priority by frames left"));
                            v.push_back(b.gop_case<444, 64, 256, S8X | LQ | FAIR>("int8 state, int32 forms, 6 per CU, frames-left priority"));
                        }
                        return;
                    }
                    if (b.mode == 420) {
                        v.push_back(b.gop_case<420, 32, 256, 3 | P | LQ | 32768 | GI>("(production)"));
                        v.push_back(b.gop_case<420, 32, 256, OPT | LQ>("optimistic, 6 per CU"));
                        v.push_back(b.gop_case<420, 32, 256, 3 | P | LQ | GI | FIX>("re-run pass (nothing marked)"));
                        v.push_back(b.gop_case<420, 32, 256, 3 | P | LQ | 32768 | GI | FAIR>("priority by frames left"));
                        v.push_back(b.gop_case<420, 32, 256, OPT | LQ | FAIR>("optimistic, 6 per CU, priority by frames left"));
                    } else if (b.mode == 422) {
                        v.push_back(b.gop_case<422, 64, 256, 3 | E | LQ | 32768 | GI>("(production)"));
                        v.push_back(b.gop_case<422, 64, 256, OPT | SQ>("optimistic, 5 per CU"));
                        v.push_back(b.gop_case<422, 64, 256, 3 | E | LQ | GI | FIX>("re-run pass (nothing marked)"));
                        v.push_back(b.gop_case<422, 64, 256, 3 | E | LQ | 32768 | GI | FAIR>("priority by frames left"));
                        v.push_back(b.gop_case<422, 64, 256, OPT | SQ | FAIR>("optimistic, 5 per CU, priority by frames left"));
                    } else {
                        v.push_back(b.gop_case<444, 64, 256, 3 | E | LQ | 32768 | GI>("(production)"));
                        v.push_back(b.gop_case<444, 64, 256, OPT | LQ>("optimistic, 6 per CU"));
                        v.push_back(b.gop_case<444, 64, 256, 3 | E | LQ | GI | FIX>("re-run pass (nothing marked)"));
                        v.push_back(b.gop_case<444, 64, 256, (OPT & ~P) | E | LQ | W5>("optimistic, early, 5 waves"));
                        v.push_back(b.gop_case<444, 64, 256, 3 | E | LQ | 32768 | GI | FAIR>("priority by frames left"));
                        v.push_back(b.gop_case<444, 64, 256, 3 | E | LQ | 32768 | GI | FAIR | (1 << 23)>("priority by frames left + start jitter"));
                        v.push_back(b.gop_case<444, 64, 256, 3 | E | LQ | 32768 | GI | (1 << 23)>("start jitter"));
                        // (the arrival-order start delay measured here before, profiles/r03/fair/stagger2/, gave
                        // its flag bit to kGopLockstep: PROBE_LOCK)
                    }
                };
                auto ndiff = [&](const void* x, const void* y, size_t bytes) {
                    CK(hipMemset(bad, 0, 8));
                    hipLaunchKernelGGL(count_diff, dim3(4096), dim3(256), 0, 0, (const u32x4*)x, (const u32x4*)y, bytes / 16, bad);
                    unsigned long long n = 0;
                    CK(hipMemcpy(&n, bad, 8, hipMemcpyDeviceToHost));
                    return n;
                };
                std::vector<Case> c0, chk;  // checks: production into b.out, every other variant into out2
                variants(c0);
                b.base.out = out2;
                variants(chk);
                b.base.out = out0;
                CK(hipMemset(b.out, 0, b.out_bytes));
                c0[0].f();
                for (size_t i = 1; i < chk.size(); i++) {
                    if (i == 2) continue;  // the re-run pass: checked after each optimistic variant
                    CK(hipMemset(out2, 0xff, b.out_bytes));
                    chk[i].f();
                    const unsigned long long marked = ndiff(jf, zero, fbytes);
                    const unsigned long long before = ndiff(b.out, out2, b.out_bytes);
                    chk[2].f();
                    const unsigned long long after = ndiff(b.out, out2, b.out_bytes), left = ndiff(jf, zero, fbytes);
                    printf("%s vs production: %llu of %u jobs marked, %llu differing dwords before the re-run, %llu after "
                           "(of %llu), %llu marks left\n", chk[i].name.c_str(), marked, tpf * b.nseg, before, after,
                           (unsigned long long)(b.out_bytes / 4), left);
                    if (after || left) return 1;
                }
                CK(hipFree(out2));
                for (auto& c : c0) cases.push_back(c);
            } else
            if (b.mode == 420) {
                cases.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768>("(round 3)"));
                cases.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768 | W>("int16 IDCT, no test"));
                cases.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768 | I>("int32 IDCT"));
                cases.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768 | I | C>("(round 2)"));
            } else if (b.mode == 422) {
                cases.push_back(b.gop_case<422, 64, 256, 3 | 4096 | 8192 | 32768>("(round 3)"));
                cases.push_back(b.gop_case<422, 64, 256, 3 | 4096 | 8192 | 32768 | I | C>("(round 2)"));
            } else {
                cases.push_back(b.gop_case<444, 64, 256, 3 | 4096 | 8192 | 32768>("(round 3)"));
                cases.push_back(b.gop_case<444, 64, 256, 3 | 4096 | 8192 | 32768 | W>("int16 IDCT, no test"));
                cases.push_back(b.gop_case<444, 64, 256, 3 | 4096 | 8192 | 32768 | I>("(round 2)"));
            }
        }
    } else if (getenv("PROBE_GOP")) {  // stream-kernel variants, GOP PROBE_GOP
        b.gop_setup((uint32_t)atoi(getenv("PROBE_GOP")));
        // 3 = nt loads + nt stores; 2048 prefetch, 4096 early, 8192 LDS tables, 16384 register
        // state (decode_gop_reg_kernel), 32768 static stores
        if (getenv("PROBE_REC")) {  // record-input kernel: outputs checked against production, then timed
            uint32_t* out0 = b.base.out;
            uint32_t* out2 = nullptr;
            unsigned long long* bad = nullptr;
            CK(hipMalloc(&out2, b.out_bytes));
            CK(hipMalloc(&bad, 8));
            std::vector<Case> chk;
            if (b.mode == 420) {
                chk.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768>("check: production"));
                b.base.out = out2;
                chk.push_back(b.gop_rec_case<420, 32, 256, 3 | 8192 | 32768>("check"));
            } else if (b.mode == 422) {
                chk.push_back(b.gop_case<422, 64, 256, 3 | 4096 | 8192 | 32768>("check: production"));
                b.base.out = out2;
                chk.push_back(b.gop_rec_case<422, 64, 256, 3 | 8192 | 32768>("check"));
            } else {
                chk.push_back(b.gop_case<444, 64, 256, 3 | 4096 | 8192 | 32768>("check: production"));
                b.base.out = out2;
                chk.push_back(b.gop_rec_case<444, 64, 256, 3 | 8192 | 32768>("check"));
            }
            b.base.out = out0;
            CK(hipMemset(b.out, 0, b.out_bytes));
            CK(hipMemset(out2, 0xff, b.out_bytes));
            chk[0].f();
            chk[1].f();
            CK(hipMemset(bad, 0, 8));
            hipLaunchKernelGGL(count_diff, dim3(4096), dim3(256), 0, 0, (const u32x4*)b.out, (const u32x4*)out2,
                               (size_t)(b.out_bytes / 16), bad);
            unsigned long long nbad = 0;
            CK(hipMemcpy(&nbad, bad, 8, hipMemcpyDeviceToHost));
            printf("record-input kernel vs production: %llu differing dwords of %llu\n", nbad,
                   (unsigned long long)(b.out_bytes / 4));
            CK(hipFree(out2));
            if (nbad) return 1;
            if (b.mode == 420) {
                cases.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768>("(production)"));
                cases.push_back(b.gop_rec_case<420, 32, 256, 3 | 8192 | 32768>("(dense-equivalent rate)"));
            } else if (b.mode == 422) {
                cases.push_back(b.gop_case<422, 64, 256, 3 | 4096 | 8192 | 32768>("(production)"));
                cases.push_back(b.gop_rec_case<422, 64, 256, 3 | 8192 | 32768>("(dense-equivalent rate)"));
            } else {
                cases.push_back(b.gop_case<444, 64, 256, 3 | 4096 | 8192 | 32768>("(production)"));
                cases.push_back(b.gop_rec_case<444, 64, 256, 3 | 8192 | 32768>("(dense-equivalent rate)"));
            }
        } else if (getenv("PROBE_GS")) {  // global-state kernel: outputs checked against production, then timed
            uint32_t* out0 = b.base.out;
            uint32_t* out2 = nullptr;
            unsigned long long* bad = nullptr;
            CK(hipMalloc(&out2, b.out_bytes));
            CK(hipMalloc(&bad, 8));
            std::vector<Case> chk;
            if (b.mode == 420) {
                chk.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768>("check: production"));
                b.base.out = out2;
                chk.push_back(b.gop_gs_case<420, 32, 256, 3, 6>("check"));
            } else if (b.mode == 422) {
                chk.push_back(b.gop_case<422, 64, 256, 3 | 4096 | 8192 | 32768>("check: production"));
                b.base.out = out2;
                chk.push_back(b.gop_gs_case<422, 64, 256, 3, 6>("check"));
            } else {
                chk.push_back(b.gop_case<444, 64, 256, 3 | 4096 | 8192 | 32768>("check: production"));
                b.base.out = out2;
                chk.push_back(b.gop_gs_case<444, 64, 256, 3, 6>("check"));
            }
            b.base.out = out0;
            CK(hipMemset(b.out, 0, b.out_bytes));
            CK(hipMemset(out2, 0xff, b.out_bytes));
            chk[0].f();
            chk[1].f();
            CK(hipMemset(bad, 0, 8));
            hipLaunchKernelGGL(count_diff, dim3(4096), dim3(256), 0, 0, (const u32x4*)b.out, (const u32x4*)out2,
                               (size_t)(b.out_bytes / 16), bad);
            unsigned long long nbad = 0;
            CK(hipMemcpy(&nbad, bad, 8, hipMemcpyDeviceToHost));
            printf("global-state kernel vs production: %llu differing dwords of %llu\n", nbad,
                   (unsigned long long)(b.out_bytes / 4));
            CK(hipFree(out2));
            if (nbad) return 1;
            if (b.mode == 420) {
                cases.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768>("(production)"));
                cases.push_back(b.decode_case<420, 32, 256, 3>("batch (production)", b.fgroup(420, 32)));
                cases.push_back(b.gop_gs_case<420, 32, 256, 3, 6>(""));
                cases.push_back(b.gop_gs_case<420, 32, 256, 3, 5>(""));
                cases.push_back(b.gop_gs_case<420, 32, 256, 3, 4>(""));
            } else if (b.mode == 422) {
                cases.push_back(b.gop_case<422, 64, 256, 3 | 4096 | 8192 | 32768>("(production)"));
                cases.push_back(b.decode_case<422, 64, 256, 3>("batch (production)", b.fgroup(422, 64)));
                cases.push_back(b.gop_gs_case<422, 64, 256, 3, 6>(""));
                cases.push_back(b.gop_gs_case<422, 64, 256, 3, 5>(""));
            } else {
                cases.push_back(b.gop_case<444, 64, 256, 3 | 4096 | 8192 | 32768>("(production)"));
                cases.push_back(b.decode_case<444, 64, 256, 3>("batch (production)", b.fgroup(444, 64)));
                cases.push_back(b.gop_gs_case<444, 64, 256, 3, 6>(""));
                cases.push_back(b.gop_gs_case<444, 64, 256, 3, 5>(""));
            }
        } else if (b.mode == 420) {
            cases.push_back(b.decode_case<420, 32, 256, 3>("batch (production)", b.fgroup(420, 32)));
            cases.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768>("prefetch ldsqt static, no jitter (r2 until run15)"));
            cases.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768 | (1 << 23)>("prefetch ldsqt static, jitter (production)"));
            cases.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768 | (1 << 23) | 262144>("prefetch ldsqt static, jitter, xcd order"));
            cases.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768 | 262144>("prefetch ldsqt static, xcd order"));
            cases.push_back(b.gop_case<420, 32, 256, 3 | 8192 | 32768>("no prefetch ldsqt static"));
            cases.push_back(b.gop_case<420, 32, 256, 3 | 8192 | 32768 | (1 << 23)>("no prefetch ldsqt static, jitter"));
            cases.push_back(b.gop_case<420, 32, 256, 3 | 8192>("no prefetch ldsqt"));
            cases.push_back(b.gop_ovl_case<420, 32, 256, 3 | 32768, 1, 5>("no prefetch static"));
            cases.push_back(b.gop_ovl_case<420, 32, 256, 3, 1, 5>("no prefetch"));
            cases.push_back(b.gop_ovl_case<420, 32, 256, 3 | 32768, 3, 6>("no prefetch static"));
            cases.push_back(b.gop_ovl_case<420, 32, 256, 3 | 32768, 1, 4>("no prefetch static"));
            cases.push_back(b.gop_case<420, 32, 256, 3 | 32768, 6>("loader waves static, 6/SIMD"));
        } else if (b.mode == 422) {
            cases.push_back(b.decode_case<422, 64, 256, 3>("batch (production)", b.fgroup(422, 64)));
            cases.push_back(b.gop_case<422, 64, 256, 3 | 4096 | 8192>("early ldsqt (r1)"));
            cases.push_back(b.gop_case<422, 64, 256, 3 | 4096 | 8192 | 32768>("early ldsqt static, no jitter (r2 until run15)"));
            cases.push_back(b.gop_case<422, 64, 256, 3 | 4096 | 8192 | 32768 | (1 << 23)>("early ldsqt static, jitter (production)"));
            cases.push_back(b.gop_case<422, 64, 256, 3 | 4096 | 8192 | 32768 | (1 << 23) | 262144>("early ldsqt static, jitter, xcd order"));
            cases.push_back(b.gop_case<422, 64, 256, 3 | 8192 | 32768>("no prefetch ldsqt static"));
            cases.push_back(b.gop_case<422, 64, 256, 3 | 8192 | 32768 | (1 << 23)>("no prefetch ldsqt static, jitter"));
            cases.push_back(b.gop_case<422, 64, 256, 3 | 32768, 5>("loader waves static, 5/SIMD"));
            cases.push_back(b.gop_case<422, 64, 256, 3 | 4096 | 8192 | 32768 | 262144>("early ldsqt static, xcd order"));
        } else {
            cases.push_back(b.decode_case<444, 64, 256, 3>("batch (production)", b.fgroup(444, 64)));
            cases.push_back(b.gop_case<444, 64, 256, 3 | 4096 | 8192>("early ldsqt (r1)"));
            cases.push_back(b.gop_case<444, 64, 256, 3 | 4096 | 8192 | 32768>("early ldsqt static, no jitter (r2 until run15)"));
            cases.push_back(b.gop_case<444, 64, 256, 3 | 4096 | 8192 | 32768 | (1 << 23)>("early ldsqt static, jitter (production)"));
            cases.push_back(b.gop_case<444, 64, 256, 3 | 4096 | 8192 | 32768 | (1 << 23) | 262144>("early ldsqt static, jitter, xcd order"));
            cases.push_back(b.gop_case<444, 64, 256, 3 | 32768, 6>("loader waves static, 6/SIMD"));
            cases.push_back(b.gop_case<444, 64, 256, 3 | 8192 | 32768>("no prefetch ldsqt static"));
            cases.push_back(b.gop_case<444, 64, 256, 3 | 8192 | 32768 | (1 << 23)>("no prefetch ldsqt static, jitter"));
            cases.push_back(b.gop_ovl_case<444, 64, 256, 3 | 32768, 1, 5>("no prefetch static"));
            cases.push_back(b.gop_ovl_case<444, 64, 256, 3 | 32768, 3, 6>("no prefetch static"));
            cases.push_back(b.gop_case<444, 64, 256, 3 | 4096 | 8192 | 32768 | 262144>("early ldsqt static, xcd order"));
            cases.push_back(b.gop_case<444, 64, 256, 3 | 32768 | 262144, 6>("loader waves static, xcd order"));
        }
    } else if (b.mode == 420) {
        const uint32_t g420 = b.fgroup(420, 32);
        cases.push_back(b.decode_case<420, 32, 256, 3>("nt (production)", g420));
        if (getenv("PROBE_POLICY")) {  // cache-policy sweep at the production shape and order
            cases.push_back(b.decode_case<420, 32, 256, 1>("nt loads, temporal stores", g420));
            cases.push_back(b.decode_case<420, 32, 256, 2>("temporal loads, nt stores", g420));
            cases.push_back(b.decode_case<420, 32, 256, 0>("temporal", g420));
            cases.push_back(b.decode_case<420, 32, 256, 1 | 128>("nt loads, sc1 stores", g420));
            cases.push_back(b.decode_case<420, 32, 256, 1 | 256>("nt loads, sc0 sc1 stores", g420));
            cases.push_back(b.decode_case<420, 32, 256, 3>("nt (production, again)", g420));
        }
        if (auto c = b.lib_case(420, 32)) cases.push_back(*c);
        cases.push_back(b.decode_case<420, 64, 512, 3>("nt (round-1 shape)"));
        cases.push_back(b.decode_case<420, 32, 256, 3>("nt frame-major"));
        cases.push_back(b.decode_case<420, 32, 256, 3 | 4>("ablate-math", g420));
        cases.push_back(b.decode_case<420, 32, 256, 3 | 32 | 4>("reads only", g420));
        cases.push_back(b.decode_case<420, 32, 256, 3 | 12>("writes only", g420));
        for (uint32_t g : {2u, 4u, 8u, 16u}) cases.push_back(b.decode_case<420, 32, 256, 3>("nt", g));
    } else if (b.mode == 422) {
        cases.push_back(b.decode_case<422, 64, 256, 3>("nt (production)", b.fgroup(422, 64)));
        cases.push_back(b.decode_case<422, 64, 256, 3>("nt"));
        cases.push_back(b.decode_case<422, 32, 128, 3>("nt"));
        cases.push_back(b.decode_case<422, 128, 512, 3>("nt"));
        cases.push_back(b.decode_case<422, 64, 256, 3 | 4>("ablate-math", b.fgroup(422, 64)));
        for (uint32_t g : {4u, 8u}) {
            cases.push_back(b.decode_case<422, 64, 256, 3>("nt", g));
            cases.push_back(b.decode_case<422, 32, 128, 3>("nt", g));
        }
    } else {
        cases.push_back(b.decode_case<444, 64, 256, 3>("nt (production)", b.fgroup(444, 64)));
        if (auto c = b.lib_case(444, 64)) cases.push_back(*c);
        cases.push_back(b.decode_case<444, 64, 256, 3>("nt frame-major"));
        cases.push_back(b.decode_case<444, 128, 512, 3>("nt"));
        cases.push_back(b.decode_case<444, 64, 256, 3 | 4>("ablate-math", b.fgroup(444, 64)));
        for (uint32_t g : {4u, 8u}) cases.push_back(b.decode_case<444, 64, 256, 3>("nt", g));
    }
    const double tot = (double)(b.in_bytes + b.out_bytes);
    cases.push_back({"copy unroll4 one-shot", tot, [=] {
                         hipLaunchKernelGGL(copy_unroll<4>, dim3((unsigned)((std::max(nin, nout) + 1023) / 1024)), dim3(256), 0, 0,
                                            (const u32x4*)b.coef, nin, (u32x4*)b.out, nout);
                     }});
    if (getenv("PROBE_COPY")) {
        auto add = [&](const char* name, auto kern, int threads, int u, unsigned grid) {
            cases.push_back({name, tot, [=] {
                                 const unsigned g = grid ? grid : (unsigned)((std::max(nin, nout) + (size_t)threads * u - 1) / ((size_t)threads * u));
                                 hipLaunchKernelGGL(kern, dim3(g), dim3(threads), 0, 0, (const u32x4*)b.coef, nin,
                                                    (u32x4*)b.out, nout);
                             }});
        };
        add("copy 256x8 nt one-shot", copy_var<256, 8, true, false>, 256, 8, 0);
        add("copy 512x4 nt one-shot", copy_var<512, 4, true, false>, 512, 4, 0);
        add("copy 1024x4 nt one-shot", copy_var<1024, 4, true, false>, 1024, 4, 0);
        add("copy 256x4 temporal one-shot", copy_var<256, 4, false, false>, 256, 4, 0);
        add("copy 256x4 nt stride g2048", copy_var<256, 4, true, true>, 256, 4, 2048);
        add("copy 256x4 nt stride g8192", copy_var<256, 4, true, true>, 256, 4, 8192);
        add("copy 512x8 nt stride g1024", copy_var<512, 8, true, true>, 512, 8, 1024);
    }
    if (getenv("PROBE_WRITES")) {
        auto addw = [&](const char* name, auto kern, int u) {
            cases.push_back({name, (double)b.out_bytes, [=] {
                                 hipLaunchKernelGGL(kern, dim3((unsigned)((nout + 256 * u - 1) / (256 * u))), dim3(256), 0, 0,
                                                    (u32x4*)b.out, nout);
                             }});
        };
        addw("write nt u1", write_var<0, 1>, 1);
        auto addo = [&](const char* name, auto kern, int t, int order) {
            cases.push_back({name, (double)b.out_bytes, [=] {
                                 size_t nch = (nout + t - 1) / t;
                                 if (order == 1) nch = 8 * ((nch + 7) / 8);
                                 if (order == 2) nch = 64 * ((nch + 63) / 64);
                                 hipLaunchKernelGGL(kern, dim3((unsigned)nch), dim3(t), 0, 0, (u32x4*)b.out, nout);
                             }});
        };
        if (b.W == 3840 && b.mode == 420) {
            const uint32_t PB = b.W * 4, H = 2160 / 16 * 16, nf = b.NF;
            auto addt = [&](const char* name, auto kern, int R, int WB, int T = 256) {
                const double bytes = (double)PB * H * nf;
                cases.push_back({name, bytes, [=] {
                                     const uint32_t nt = (PB / WB) * (H / R) * nf;
                                     hipLaunchKernelGGL(kern, dim3(8 * ((nt + 7) / 8)), dim3(T), 0, 0, (uint8_t*)b.out, PB, H, nf);
                                 }});
            };
            addt("tile 16x1920 xcd-contig 1024 lanes", write_tile<16, 1920, 1, 1024>, 16, 1920, 1024);
            addt("tile 16x1920 xcd-contig 512 lanes", write_tile<16, 1920, 1, 512>, 16, 1920, 512);
            addt("tile 2x1920 xcd-contig", write_tile<2, 1920, 1>, 2, 1920);
            addt("tile 16x256 xcd-contig", write_tile<16, 256, 1>, 16, 256);
            addt("tile 16x512 xcd-contig", write_tile<16, 512, 1>, 16, 512);
            addt("tile 16x1920 frame-major", write_tile<16, 1920, 0>, 16, 1920);
            addt("tile 16x1920 xcd-contig", write_tile<16, 1920, 1>, 16, 1920);
            addt("tile 16x1920 fgroup8", write_tile<16, 1920, 2>, 16, 1920);
            addt("tile 16x3840 xcd-contig", write_tile<16, 3840, 1>, 16, 3840);
            addt("tile 16x15360 xcd-contig", write_tile<16, 15360, 1>, 16, 15360);
            addt("tile 8x1920 xcd-contig", write_tile<8, 1920, 1>, 8, 1920);
            addt("tile 4x3840 xcd-contig", write_tile<4, 3840, 1>, 4, 3840);
            addt("tile 1x4096 xcd-contig", write_tile<1, 3840, 1>, 1, 3840);
        }
        addo("write one 64 lanes", write_one<64, 0>, 64, 0);
        addo("write one 128 lanes", write_one<128, 0>, 128, 0);
        addo("write one 256 lanes", write_one<256, 0>, 256, 0);
        addo("write one 512 lanes", write_one<512, 0>, 512, 0);
        addo("write one 1024 lanes", write_one<1024, 0>, 1024, 0);
        addo("write one 256 xcd-contig", write_one<256, 1>, 256, 1);
        addo("write one 256 xcd-8x8", write_one<256, 2>, 256, 2);
        addw("write nt u4", write_var<0, 4>, 4);
        addw("write nt u8", write_var<0, 8>, 8);
        addw("write temporal u4", write_var<1, 4>, 4);
        addw("write sc1 u4", write_var<2, 4>, 4);
        addw("write sc0sc1 u4", write_var<3, 4>, 4);
        addw("write nt lane64B u4", write_var<4, 4>, 4);
        addw("write nt lane128B u8", write_var<4, 8>, 8);
    }
    cases.push_back({"read only nt", (double)b.in_bytes, [=] {
                         hipLaunchKernelGGL(read_kernel, dim3(32768), dim3(256), 0, 0, (const u32x4*)b.coef, nin, sink);
                     }});
    cases.push_back({"write only nt", (double)b.out_bytes, [=] {
                         hipLaunchKernelGGL(write_kernel, dim3(32768), dim3(256), 0, 0, (u32x4*)b.out, nout);
                     }});
    }  // PROBE_PAIRS
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    auto run = [&](const Case& c) {
        CK(hipEventRecord(e0, 0));
        c.f();
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        return ms;
    };
    if (getenv("PROBE_PMC") && b.mode == 420 && getenv("PROBE_GOP")) {
        // counter runs (rocprofv3 --pmc): exactly four cases, dispatched in this order every round --
        // decode_kernel<420,32,256,3> alternates XCD-contiguous / frame-major, then the one-shot
        // bands order (decode_order_kernel), then the production stream kernel
        const mj423::DecodeParams qa = b.persist_params<420, 32>();
        const uint32_t E = (qa.tiles_per_frame + 7) / 8, nf = b.NF;
        auto k6 = mj423::decode_order_kernel<420, 32, 256, 3>;
        std::vector<Case> pc;
        pc.push_back(b.decode_case<420, 32, 256, 3>("one-shot XCD-contiguous (production)", mj423::kFgroupXcd));
        pc.push_back(b.decode_case<420, 32, 256, 3>("one-shot frame-major"));
        pc.push_back({"one-shot bands", (double)(b.in_bytes + b.out_bytes), [=] { hipLaunchKernelGGL(k6, dim3(8 * E * nf), dim3(256), 0, 0, qa, 2u, nf, 0u); }});
        pc.push_back(b.gop_case<420, 32, 256, 3 | 2048 | 8192 | 32768 | (1 << 26) | (1 << 27)>("stream kernel (production)"));
        cases = pc;
    }
    std::vector<std::vector<float>> ms(cases.size());
    for (auto& c : cases) run(c);  // warm-up
    if (const char* ws = getenv("PROBE_WARM_S")) {  // clocks ramp under sustained load: run the cases round-robin first
        const double warm = atof(ws);
        double spent = 0;
        while (spent < warm * 1e3)
            for (auto& c : cases) spent += run(c);
    }
    for (int r = 0; r < rounds; r++)
        for (size_t i = 0; i < cases.size(); i++) ms[i].push_back(run(cases[i]));
    for (size_t i = 0; i < cases.size(); i++) {
        auto v = ms[i];
        std::sort(v.begin(), v.end());
        const float med = v[v.size() / 2];
        printf("%-34s median %8.3f ms  min %8.3f ms  %7.1f GB/s (%.3f of 8 TB/s)\n", cases[i].name.c_str(), med, v[0],
               cases[i].bytes / (med * 1e-3) / 1e9, cases[i].bytes / (med * 1e-3) / 8e12);
    }
    return 0;
}
