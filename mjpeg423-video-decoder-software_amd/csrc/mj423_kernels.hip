// mj423_kernels.hip -- hand-written CDNA4 (gfx950) kernels for the MPEG423 hot path:
// fused dequantize -> 8x8 integer IDCT -> YCbCr->BGRA (with 4:2:2 / 4:2:0 chroma
// fetch), plus the stand-alone stage kernels behind the reference's per-block
// symbols and a synthetic-stream generator for the benchmark.
//
// Reference (paths under core0/software/common/libs/mjpeg423/):
//   per-frame body      decoder/mjpeg423_decoder.c:109-124
//   dequant             decoder/lossless_decode.c:89-129
//   idct                decoder/idct.c:22-181
//   ycbcr_to_rgb        decoder/ycbcr_to_rgb.c:26-49
//   accelerator contract c0 idct_ycbcr_to_rgb_accel.h:13-22, playback.c:71-121
//
// Fused kernel structure (one 256-thread workgroup per tile):
//   tile   = a run of up to TWMAX MCUs inside one MCU row of one frame
//   stage  : the tile's Y/Cb/Cr block runs (each contiguous in HBM) are copied
//            into LDS with 16-B coalesced loads, one LDS "slot" of 128 B per block
//   IDCT   : one lane per block (slot); each wave's blocks share a plane class so
//            the quant table sits in SGPRs; results go to uint8 plane tiles in LDS
//            (aliasing the coefficient slots after a barrier)
//   CSC    : each lane converts 4 horizontally adjacent pixels and writes them
//            as one 16-B store; a wave writes 1 KiB of contiguous BGRA row.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mj423_idct.hpp"
#include "mj423_kernels.h"

namespace mj423 {

template <int MODE>
struct Layout;
// 4:2:0: MCU 16x16 = 4 Y (2x2) + Cb + Cr.  Slots: Y row0 [0,64) Y row1 [64,128) Cb [128,160) Cr [160,192)
template <>
struct Layout<420> {
    static constexpr int TWMAX = 32, MW = 16, MH = 16, SX = 2, SY = 2, NSLOT = 192;
    static constexpr int YRUN = 64, CRUN = 32;  // slot capacity per run
};
// 4:2:2: MCU 16x8 = 2 Y (2x1) + Cb + Cr.  Slots: Y [0,128) Cb [128,192) Cr [192,256)
template <>
struct Layout<422> {
    static constexpr int TWMAX = 64, MW = 16, MH = 8, SX = 2, SY = 1, NSLOT = 256;
    static constexpr int YRUN = 128, CRUN = 64;
};
// 4:4:4: MCU 8x8 = Y + Cb + Cr.  Slots: Y [0,64) Cb [64,128) Cr [128,192)
template <>
struct Layout<444> {
    static constexpr int TWMAX = 64, MW = 8, MH = 8, SX = 1, SY = 1, NSLOT = 192;
    static constexpr int YRUN = 64, CRUN = 64;
};

template <int MODE>
struct Tile {
    using L = Layout<MODE>;
    static constexpr int YW = L::TWMAX * L::MW;  // Y plane tile width (px)
    static constexpr int CW = YW / L::SX;        // chroma plane tile width (px)
    static constexpr int CH = 8;                 // chroma rows per MCU row, every mode
    static constexpr int PLANE_BYTES = L::MH * YW + 2 * CH * CW;
    static constexpr int COEF_BYTES = L::NSLOT * 128;
    static constexpr int LDS_BYTES = COEF_BYTES > PLANE_BYTES ? COEF_BYTES : PLANE_BYTES;
    static constexpr int CHUNKS = L::NSLOT / 32;  // 16-B chunks per thread when staging

    // Runs: 0,1 = Y block rows (1 only in 4:2:0), 2 = Cb, 3 = Cr; each starts at a fixed slot.
    static constexpr int run_first_slot(int run) {
        return MODE == 420 ? (run == 0 ? 0 : run == 1 ? 64 : run == 2 ? 128 : 160)
                           : MODE == 422 ? (run <= 1 ? 0 : run == 2 ? 128 : 192)
                                         : (run <= 1 ? 0 : run == 2 ? 64 : 128);
    }
    // Staging chunk k of a thread covers slots [32k, 32k+32): its run is static.
    static constexpr int chunk_run(int k) {
        return MODE == 420 ? (k < 2 ? 0 : k < 4 ? 1 : k == 4 ? 2 : 3)
                           : MODE == 422 ? (k < 4 ? 0 : k < 6 ? 2 : 3) : (k < 2 ? 0 : k < 4 ? 2 : 3);
    }
    // IDCT wave w (slots [64w, 64w+64)) covers one plane class; 4:2:0 wave 2 = Cb|Cr halves.
    __device__ static __forceinline__ int slot_run(int s) {
        if (MODE == 420) return s < 64 ? 0 : s < 128 ? 1 : s < 160 ? 2 : 3;
        if (MODE == 422) return s < 128 ? 0 : s < 192 ? 2 : 3;
        return s < 64 ? 0 : s < 128 ? 2 : 3;
    }
};

// LDS position of row r of slot s: rows are XOR-swizzled by the slot so that the
// per-lane ds_read_b128 of "row r of my block" spreads over the banks.
__device__ __forceinline__ int coef_off(int s, int r) { return s * 128 + ((r ^ (s & 7)) << 4); }

template <int MODE>
__global__ void __launch_bounds__(256) decode_kernel(const DecodeParams p) {
    using L = Layout<MODE>;
    using T = Tile<MODE>;
    __shared__ __attribute__((aligned(16))) uint8_t lds[T::LDS_BYTES];

    const int tid = threadIdx.x;
    // ---- tile coordinates
    const uint32_t bid = blockIdx.x;
    const uint32_t tx = bid % p.tiles_per_row;
    const uint32_t t2 = bid / p.tiles_per_row;
    const uint32_t my = t2 % p.mcu_rows;
    const uint32_t f = t2 / p.mcu_rows;
    const uint32_t mx0 = tx * p.tw;
    const int tw = (int)min(p.tw, p.mcu_cols - mx0);  // MCUs in this tile

    // int16-element offset (from p.coef) of the first block of each run
    const int64_t fbase = (int64_t)f * (int64_t)p.plane_fstride;
    int64_t run_off[4];
    int run_len[4];
    if (MODE == 420) {
        run_off[0] = fbase + ((int64_t)(2 * my) * p.y_bw + 2 * mx0) * 64;
        run_off[1] = run_off[0] + (int64_t)p.y_bw * 64;
        run_len[0] = run_len[1] = 2 * tw;
    } else {
        constexpr int YPER = MODE == 422 ? 2 : 1;
        run_off[0] = run_off[1] = fbase + ((int64_t)my * p.y_bw + YPER * mx0) * 64;
        run_len[0] = run_len[1] = YPER * tw;
    }
    const int64_t coff = fbase + ((int64_t)my * p.c_bw + mx0) * 64;
    run_off[2] = coff + p.cb_off;
    run_off[3] = coff + p.cr_off;
    run_len[2] = run_len[3] = tw;

    // ---- stage: HBM -> LDS, 16 B per lane, every load issued before the first LDS write.
    //      Chunk k of thread t is (slot 32k + t/8, row t%8): a wave reads 1 KiB contiguous.
    //      Slots past the end of a short (edge) tile re-read block 0 of their run --
    //      the same cache lines the wave already fetches -- so the code stays branch-free
    //      and moves no extra HBM bytes; those slots are never computed.
    {
        u32x4 v[T::CHUNKS];
#pragma unroll
        for (int k = 0; k < T::CHUNKS; k++) {
            const int run = T::chunk_run(k);
            const int col = 32 * k + (tid >> 3) - T::run_first_slot(run);
            const int colc = col < run_len[run] ? col : 0;
            v[k] = __builtin_nontemporal_load(
                reinterpret_cast<const u32x4*>(p.coef + run_off[run] + colc * 64 + (tid & 7) * 8));
        }
#pragma unroll
        for (int k = 0; k < T::CHUNKS; k++)
            *reinterpret_cast<u32x4*>(lds + coef_off(32 * k + (tid >> 3), tid & 7)) = v[k];
    }
    __syncthreads();

    // ---- IDCT: one lane per slot; the wave's plane class (Y or chroma) is uniform,
    //      so its dequantization table is read through SGPRs.
    const int s = tid;
    const int run = T::slot_run(s);
    const int col = s - (MODE == 420 ? (run == 0 ? 0 : run == 1 ? 64 : run == 2 ? 128 : 160)
                                     : MODE == 422 ? (run == 0 ? 0 : run == 2 ? 128 : 192)
                                                   : (run == 0 ? 0 : run == 2 ? 64 : 128));
    const bool active = s < L::NSLOT && col < run_len[run];
    uint32_t d[8][4];
    if (s < L::NSLOT) {
        const int wave_chroma = __builtin_amdgcn_readfirstlane(run >= 2 ? 1 : 0);
        const uint32_t* qt = p.qt[wave_chroma];
#pragma unroll
        for (int r = 0; r < 8; r++) {
            const uint4 q = *reinterpret_cast<const uint4*>(lds + coef_off(s, r));
            d[r][0] = dequant_pair(q.x, qt[4 * r + 0]);
            d[r][1] = dequant_pair(q.y, qt[4 * r + 1]);
            d[r][2] = dequant_pair(q.z, qt[4 * r + 2]);
            d[r][3] = dequant_pair(q.w, qt[4 * r + 3]);
        }
    }
    __syncthreads();  // every coefficient is in registers: the slots become plane tiles
    uint8_t* yplane = lds;
    uint8_t* cbplane = lds + L::MH * T::YW;
    uint8_t* crplane = cbplane + T::CH * T::CW;
    if (active) {
        uint32_t o[8][2];
        idct8x8(d, o);
        uint8_t* dstp = run < 2 ? yplane + (run * 8) * T::YW + col * 8 : (run == 2 ? cbplane : crplane) + col * 8;
        const int pitch = run < 2 ? T::YW : T::CW;
#pragma unroll
        for (int r = 0; r < 8; r++) *reinterpret_cast<uint2*>(dstp + r * pitch) = make_uint2(o[r][0], o[r][1]);
    }
    __syncthreads();

    // ---- CSC: a lane takes 4 horizontally adjacent pixels of every luma row that
    //      shares one chroma row (2 rows in 4:2:0), computes the chroma terms once,
    //      and writes 16 B per row: a wave stores 1 KiB of contiguous BGRA.
    constexpr int QPR = T::YW / 4;          // quads per tile row
    constexpr int JOBS = QPR * T::CH;       // (quad, chroma row) pairs
    constexpr int ITERS = JOBS / 256;
    const int qcols = tw * L::MW / 4;       // quads present in this tile
    const uint32_t x_tile = mx0 * L::MW, y_tile = my * L::MH;
    uint32_t* outf = p.out + (size_t)f * p.out_fstride;
#pragma unroll 1
    for (int it = 0; it < ITERS; it++) {
        const int job = it * 256 + tid;
        const int qc = job % QPR, cy = job / QPR;
        if (qc >= qcols) continue;
        int32_t tr[4], tg[4], tb[4];
        if (L::SX == 2) {
            const uint32_t cb2 = *reinterpret_cast<const uint16_t*>(cbplane + cy * T::CW + qc * 2);
            const uint32_t cr2 = *reinterpret_cast<const uint16_t*>(crplane + cy * T::CW + qc * 2);
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const ChromaTerms t = chroma_terms((cb2 >> (8 * i)) & 0xff, (cr2 >> (8 * i)) & 0xff);
                tr[2 * i] = tr[2 * i + 1] = t.r;
                tg[2 * i] = tg[2 * i + 1] = t.g;
                tb[2 * i] = tb[2 * i + 1] = t.b;
            }
        } else {
            const uint32_t cb4 = *reinterpret_cast<const uint32_t*>(cbplane + cy * T::CW + qc * 4);
            const uint32_t cr4 = *reinterpret_cast<const uint32_t*>(crplane + cy * T::CW + qc * 4);
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const ChromaTerms t = chroma_terms((cb4 >> (8 * i)) & 0xff, (cr4 >> (8 * i)) & 0xff);
                tr[i] = t.r;
                tg[i] = t.g;
                tb[i] = t.b;
            }
        }
        const uint32_t gx = x_tile + qc * 4;
#pragma unroll
        for (int sub = 0; sub < L::SY; sub++) {
            const int ry = cy * L::SY + sub;
            const uint32_t gy = y_tile + ry;
            if (gy >= p.height) continue;
            const uint32_t yq = *reinterpret_cast<const uint32_t*>(yplane + ry * T::YW + qc * 4);
            uint32_t px[4];
            px[0] = bgra16(y16<0>(yq), ChromaTerms{tr[0], tg[0], tb[0]});
            px[1] = bgra16(y16<1>(yq), ChromaTerms{tr[1], tg[1], tb[1]});
            px[2] = bgra16(y16<2>(yq), ChromaTerms{tr[2], tg[2], tb[2]});
            px[3] = bgra16(y16<3>(yq), ChromaTerms{tr[3], tg[3], tb[3]});
            uint32_t* dst = outf + (size_t)gy * p.out_pitch + gx;
            if (p.aligned16 && gx + 4 <= p.width) {
                const u32x4 v4 = {px[0], px[1], px[2], px[3]};
                __builtin_nontemporal_store(v4, reinterpret_cast<u32x4*>(dst));
            } else {
#pragma unroll
                for (int i = 0; i < 4; i++)
                    if (gx + i < p.width) dst[i] = px[i];
            }
        }
    }
}

// ---------------------------------------------------------------------------------
// Stage kernels behind the reference's per-block symbols (HOT LOOP 1 / 2 forms).

// idct() over n blocks; one lane per block.  qt == nullptr: input already dequantized.
__global__ void __launch_bounds__(256) idct_blocks_kernel(const int16_t* __restrict__ in, uint8_t* __restrict__ out,
                                                          uint32_t n, const uint32_t* __restrict__ qt) {
    const uint32_t b = blockIdx.x * 256 + threadIdx.x;
    if (b >= n) return;
    const uint4* src = reinterpret_cast<const uint4*>(in + (size_t)b * 64);
    uint32_t d[8][4];
#pragma unroll
    for (int r = 0; r < 8; r++) {
        const uint4 q = src[r];
        d[r][0] = qt ? dequant_pair(q.x, qt[4 * r + 0]) : q.x;
        d[r][1] = qt ? dequant_pair(q.y, qt[4 * r + 1]) : q.y;
        d[r][2] = qt ? dequant_pair(q.z, qt[4 * r + 2]) : q.z;
        d[r][3] = qt ? dequant_pair(q.w, qt[4 * r + 3]) : q.w;
    }
    uint32_t o[8][2];
    idct8x8(d, o);
    uint2* dst = reinterpret_cast<uint2*>(out + (size_t)b * 64);
#pragma unroll
    for (int r = 0; r < 8; r++) dst[r] = make_uint2(o[r][0], o[r][1]);
}

// ycbcr_to_rgb() over a block-raster 4:4:4 frame (mjpeg423_decoder.c:120-124): one lane per pixel.
__global__ void __launch_bounds__(256) csc444_kernel(const uint8_t* __restrict__ Y, const uint8_t* __restrict__ Cb,
                                                     const uint8_t* __restrict__ Cr, uint32_t* __restrict__ rgb,
                                                     uint32_t w_size, uint32_t h_size, uint32_t out_pitch) {
    const uint32_t x = blockIdx.x * 256 + threadIdx.x, y = blockIdx.y;
    if (x >= w_size || y >= h_size) return;
    const size_t i = ((size_t)(y >> 3) * (w_size >> 3) + (x >> 3)) * 64 + (y & 7) * 8 + (x & 7);
    rgb[(size_t)y * out_pitch + x] = bgra(Y[i], chroma_terms(Cb[i], Cr[i]));
}

// ---------------------------------------------------------------------------------
// Synthetic quantized-coefficient stream: counter-based, keyed by
// (seed, global frame, plane, block), so every rank/launch reproduces the same
// frames without any host->device traffic.  One lane per block.
__device__ __forceinline__ uint64_t splitmix64(uint64_t& s) {
    uint64_t z = (s += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

struct Rng32 {
    uint64_t state, pool;
    int avail;
    __device__ __forceinline__ uint32_t next() {
        if (avail == 0) {
            pool = splitmix64(state);
            avail = 2;
        }
        const uint32_t v = (uint32_t)pool;
        pool >>= 32;
        avail--;
        return v;
    }
};

__global__ void __launch_bounds__(256) synth_kernel(const SynthParams p) {
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;  // block index over the batch
    const uint64_t per_frame = (uint64_t)p.y_blocks + 2ull * p.c_blocks;
    if (g >= per_frame * p.nframes) return;
    const uint64_t f = g / per_frame;
    const uint64_t bi = g % per_frame;  // [Y | Cb | Cr] block index inside the frame
    const int plane = bi < p.y_blocks ? 0 : (bi < (uint64_t)p.y_blocks + p.c_blocks ? 1 : 2);
    const int16_t* q = plane == 0 ? p.yq : p.cq;
    Rng32 rng;
    rng.state = p.seed ^ ((p.frame0 + f) * 0xD1B54A32D192ED03ull) ^ (bi * 0x8CB92BA72F3D8DD7ull) ^
                ((uint64_t)plane << 61);
    rng.pool = 0;
    rng.avail = 0;
    uint32_t w[32];  // packed natural-order block
#pragma unroll
    for (int i = 0; i < 32; i++) w[i] = 0;
    // DC ~ U[0, floor(2040 / q0)]: fdct DC <= 8*255 (fdct.c:118)
    const uint32_t dc = rng.next() % (2040u / (uint32_t)q[0] + 1u);
    w[0] = dc;
    for (int k = 1; k < 64; k++) {  // AC at zig-zag position k: non-zero w.p. 0.6 exp(-k/8)
        if (rng.next() >= p.ac_thresh[k]) continue;
        const int nat = p.zigzag[k];
        uint32_t m = 1;  // magnitude 1 + Geom(0.35), capped
        while (m < 16 && rng.next() < 0xA6666666u) m++;
        const uint32_t lim = max(1023u / (uint32_t)q[nat], 1u);  // |Q*q| <= 1023
        int32_t v = (int32_t)min(m, lim);
        if (rng.next() & 1u) v = -v;
        const uint32_t h = (uint32_t)(uint16_t)(int16_t)v;
        // nat is data-dependent: update the packed word without dynamic register indexing
#pragma unroll
        for (int i = 0; i < 32; i++)
            if ((nat >> 1) == i) w[i] |= (nat & 1) ? (h << 16) : h;
    }
    uint4* o4 = reinterpret_cast<uint4*>(p.coef + f * p.frame_stride + bi * 64);
#pragma unroll
    for (int i = 0; i < 8; i++) o4[i] = make_uint4(w[4 * i], w[4 * i + 1], w[4 * i + 2], w[4 * i + 3]);
}

}  // namespace mj423

// ------------------------------------------------------------------ launchers
extern "C" hipError_t mj423_launch_decode(const mj423::DecodeParams* p, uint32_t nframes, int chroma,
                                          hipStream_t stream) {
    const uint64_t tiles = (uint64_t)nframes * p->mcu_rows * p->tiles_per_row;
    if (tiles == 0) return hipSuccess;
    if (tiles > 0x7fffffffull) return hipErrorInvalidValue;
    const dim3 grid((uint32_t)tiles), block(256);
    switch (chroma) {
    case 420: hipLaunchKernelGGL(mj423::decode_kernel<420>, grid, block, 0, stream, *p); break;
    case 422: hipLaunchKernelGGL(mj423::decode_kernel<422>, grid, block, 0, stream, *p); break;
    case 444: hipLaunchKernelGGL(mj423::decode_kernel<444>, grid, block, 0, stream, *p); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

extern "C" int mj423_tile_max_mcus(int chroma) {
    switch (chroma) {
    case 420: return mj423::Layout<420>::TWMAX;
    case 422: return mj423::Layout<422>::TWMAX;
    case 444: return mj423::Layout<444>::TWMAX;
    default: return 0;
    }
}

extern "C" hipError_t mj423_launch_idct_blocks(const int16_t* in, uint8_t* out, uint32_t n, const uint32_t* qt,
                                               hipStream_t stream) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(mj423::idct_blocks_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, in, out, n, qt);
    return hipGetLastError();
}

extern "C" hipError_t mj423_launch_csc444(const uint8_t* Y, const uint8_t* Cb, const uint8_t* Cr, uint32_t* rgb,
                                          uint32_t w_size, uint32_t h_size, uint32_t out_pitch, hipStream_t stream) {
    if (w_size == 0 || h_size == 0) return hipSuccess;
    hipLaunchKernelGGL(mj423::csc444_kernel, dim3((w_size + 255) / 256, h_size), dim3(256), 0, stream, Y, Cb, Cr,
                       rgb, w_size, h_size, out_pitch);
    return hipGetLastError();
}

extern "C" hipError_t mj423_launch_synth(const mj423::SynthParams* p, hipStream_t stream) {
    const uint64_t n = ((uint64_t)p->y_blocks + 2ull * p->c_blocks) * p->nframes;
    if (n == 0) return hipSuccess;
    const uint64_t blocks = (n + 255) / 256;
    if (blocks > 0x7fffffffull) return hipErrorInvalidValue;
    hipLaunchKernelGGL(mj423::synth_kernel, dim3((uint32_t)blocks), dim3(256), 0, stream, *p);
    return hipGetLastError();
}
