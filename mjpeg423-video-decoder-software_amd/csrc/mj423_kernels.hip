// mj423_kernels.hip -- hand-written CDNA4 (gfx950) kernels for the MPEG423 hot path:
// fused dequantize -> 8x8 integer IDCT -> YCbCr->BGRA (with 4:2:2 / 4:2:0 chroma
// fetch) for batches of absolute frames (decode_kernel) and for I/P streams with the
// P-frame deltas accumulated on chip (decode_gop_kernel), plus the stand-alone stage
// kernels behind the reference's per-block symbols, the GPU entropy front end and a
// synthetic-stream generator for the benchmark.  The tile building blocks both fused
// kernels share are in mj423_tile.hpp.
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
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <type_traits>

#include "mj423_tile.hpp"

namespace mj423 {

// mj/common/tables.c:35-42: zig-zag scan position -> natural index.
__constant__ uint32_t kZigzagNat[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                       12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                       35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                       58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};


template <int MODE, int TW, int THREADS, int FLAGS = kDefaultFlags>
__global__ void __launch_bounds__(THREADS, (lds_waves(kBatchLds<MODE, TW, THREADS, FLAGS>, THREADS)))
    decode_kernel(const DecodeParams p) {
    static_assert(production_flags<FLAGS>(), "decode_kernel: production flags only");
    using T = Tile<MODE, TW, THREADS>;
    __shared__ __attribute__((aligned(16))) uint8_t lds[kBatchLds<MODE, TW, THREADS, FLAGS>];
    const int tid = threadIdx.x;
    u32x4 v[T::CHUNKS];
    // one tile per workgroup
    uint32_t t = blockIdx.x;
    if (p.fgroup == kFgroupXcd) {  // workgroups b and b+8 share an XCD:
        // give each XCD a contiguous range (grid = 8 * per workgroups, the last few idle)
        const uint32_t per = (p.ntiles + 7) / 8;
        t = (blockIdx.x % 8) * per + blockIdx.x / 8;
        if (t >= p.ntiles) return;
    } else if (p.fgroup > 1) {  // frame-interleaved order (uniform branch on a kernel argument)
        const uint32_t G = p.fgroup, group = G * p.tiles_per_frame, fg = t / group, i = t % group;
        const uint32_t nf = p.ntiles / p.tiles_per_frame, gs = min(G, nf - fg * G);
        t = (fg * G + i % gs) * p.tiles_per_frame + i / gs;
    }
    const TileCoord c = tile_coord<MODE>(p, t);
    stage_load<MODE, TW, THREADS, FLAGS>(p, c, tid, v);
    stage_store<MODE, TW, THREADS, FLAGS>(lds, tid, v);
    __syncthreads();
    decode_tile_idct<MODE, TW, THREADS, FLAGS, true>(p, c, lds, lds, tid);
    __syncthreads();
    decode_tile_csc<MODE, TW, THREADS, FLAGS>(p, c, lds, tid);
}

// Stream decode with on-GPU P-frame accumulation.  Workgroup
// (x, y) walks tile x of every frame of segment y (a run of frames starting at an
// I-frame, or at frame 0 continuing from p.state).  The tile's absolute quantized
// coefficients stay in LDS from frame to frame: an I-frame's staging chunk replaces
// them, a P-frame's chunk (its deltas) is added mod 2^16 -- lossless_decode.c:90-92,
// 121-122 in the quantized domain.  P-frames therefore cost the same HBM bytes as
// I-frames and no accumulated plane is written back (except the optional end state).

template <int MODE, int TW, int THREADS, int FLAGS = kDefaultFlags>
__global__ void __launch_bounds__(THREADS, (lds_waves(kGopLds<MODE, TW, THREADS, FLAGS>, THREADS)))
    decode_gop_kernel(const DecodeParams p) {
    static_assert(production_flags<FLAGS>(), "decode_gop_kernel: production flags only");
    using T = Tile<MODE, TW, THREADS>;
    constexpr bool LDSQT = (FLAGS & kGopLdsQt) != 0;
    __shared__ __attribute__((aligned(16))) uint8_t lds[kGopLds<MODE, TW, THREADS, FLAGS>];
    constexpr bool S8 = (FLAGS & kGopState8) != 0;
    constexpr int SB = kGopStateBytes<MODE, TW, THREADS, FLAGS>;
    uint8_t* state = lds;          // quantized coefficient slots, persistent
    uint8_t* planes = lds + SB;    // uint8 plane tiles, per frame
    uint32_t* lds_qt = reinterpret_cast<uint32_t*>(lds + SB + T::PLANE_BYTES);  // LDSQT only
    uint32_t wide8 = 0;  // S8: biased values seen (a high byte set = a value outside int8)
    // S8: this lane's chunk k as 8 bytes of its slot's row
    auto st8 = [&](int k, int t) { return state + coef_off8(T::SLOTS_PER_CHUNK * k + (t >> 3), t & 7); };
    const int tid0 = threadIdx.x;
    const int tid = tid0;
    if (LDSQT && tid < 16)  // ordered before the first IDCT by the first staging barrier
        reinterpret_cast<uint4*>(lds_qt)[tid] = reinterpret_cast<const uint4*>(p.qt_dev)[tid];
    const uint32_t tiles_per_frame = p.tiles_per_frame;
    // Workgroup order: tile-major inside a segment, so the resident workgroups walk the same
    // frames together.  (Measured alternatives, round 2: a contiguous tile range per
    // XCD -1 %; consecutive workgroups on consecutive segments of one tile -5 %; groups of 4
    // or 8 segments interleaved like the batch kernel's frame groups -1 % / -5 %.)
    uint32_t tx, sy;
    if (!gop_job(p, tx, sy)) return;  // (whole workgroup, before any barrier)
    uint32_t* const jflag = p.jobflag ? p.jobflag + ((size_t)sy * tiles_per_frame + tx) : nullptr;
    if constexpr ((FLAGS & kGopFixup) != 0) {  // exact re-run of the jobs the optimistic form flagged
        if (jflag == nullptr || __builtin_amdgcn_readfirstlane(*jflag) == 0) return;
        if (p.reruns && threadIdx.x == 0) atomicAdd(p.reruns, 1ull);  // a vector atomic
    }
    uint32_t esc = 0;  // kIdctW16Esc: a block of this lane failed the int16 width test
    if constexpr ((FLAGS & kGopJitter) != 0) {
        // Workgroups that start together stay in step: every resident workgroup loads, then
        // transforms, then stores in the same few microseconds, so HBM sees alternating read and
        // write bursts.  A hashed start delay of up to two frame-halves spreads the phases
        // (in the probe +1.5 ... +7 %, through the library flat: opt-in).
        const uint32_t h = ((tx * 0x9E3779B1u) ^ (sy * 0x85EBCA77u)) >> 30;  // 0..3
        for (uint32_t i = 0; i < (h > 2 ? 2 : h); i++) __builtin_amdgcn_s_sleep(127);
    }
    const uint32_t f0 = p.seg_start[sy], f1 = p.seg_start[sy + 1];
    // Chunk k of this lane in the state buffers ([Y | Cb | Cr] per frame).
    const TileCoord cs = tile_coord<MODE>(p, tx);  // frame-0 coordinates: no frame offset
    auto st_off = [&](int k) -> int64_t {
        const int run = T::chunk_run(k);
        const int col = T::SLOTS_PER_CHUNK * k + (tid >> 3) - T::run_first_slot(run);
        const int colc = col < cs.run_len(run) ? col : 0;
        const int64_t o = cs.run_off(run) + colc * 64 + (tid & 7) * 8;
        return run < 2 ? o : run == 2 ? o - p.cb_off + p.st_cb_off : o - p.cr_off + p.st_cr_off;
    };
    if (p.ftype[f0] != 0) {  // the segment continues a GOP: seed the slots from p.state
        u32x4 v[T::CHUNKS];
#pragma unroll
        for (int k = 0; k < T::CHUNKS; k++) v[k] = *reinterpret_cast<const u32x4*>(p.state + st_off(k));
        if constexpr (S8) {
#pragma unroll
            for (int k = 0; k < T::CHUNKS; k++) *reinterpret_cast<uint2*>(st8(k, tid)) = pack8(v[k], wide8);
        } else {
            stage_store<MODE, TW, THREADS, kDefaultFlags>(state, tid, v);
        }
    }
    // Frame loop.  kGopPrefetch: frame f+1's loads are issued after frame f's IDCT, so they
    // are in flight during its CSC (the IDCT's registers are dead by then).
    constexpr bool EARLY = (FLAGS & kGopEarly) != 0;
    constexpr bool PREFETCH = (FLAGS & (kGopPrefetch | kGopEarly)) != 0;
    u32x4 v[T::CHUNKS];
    TileCoord c;
    // kStaticStores: the next frame's type is loaded with its coefficients (before this frame's
    // stores), so reading it never waits for the stores either.
    constexpr bool STATIC = (FLAGS & kStaticStores) != 0;
    uint32_t ft = f0 < f1 ? p.ftype[f0] : 0u;
    if (PREFETCH && f0 < f1) {
        c = tile_coord<MODE>(p, f0 * tiles_per_frame + tx);
        stage_load<MODE, TW, THREADS, FLAGS>(p, c, tid0, v);
        // vmcnt counts loads and stores in issue order.  With these loads still outstanding at the loop
        // header, the compiler's wait counts there (merged over both edges) are the ones this entry edge
        // needs, so on the back edge every frame waits until its predecessor's stores have completed.
        // Draining this edge instead (the back edge then waits for the prefetched loads only) measured
        // neutral to 4 % slower (profiles/r03/wait/): with HBM saturated, stores left in flight buy
        // nothing, and the drain paces the workgroups.
    }
    for (uint32_t f = f0; f < f1; f++) {
        // Lane-derived addresses are recomputed every frame (a few VALU ops) instead of
        // being hoisted out of the loop and kept live across the IDCT (~+40 VGPRs).
        int tid = tid0;
        asm volatile("" : "+v"(tid));
        if constexpr ((FLAGS & kGopFair) != 0) {
            const uint32_t left = f1 - f;  // uniform
            if (left >= 18) __builtin_amdgcn_s_setprio(3);
            else if (left >= 12) __builtin_amdgcn_s_setprio(2);
            else if (left >= 6) __builtin_amdgcn_s_setprio(1);
            else __builtin_amdgcn_s_setprio(0);
        }
        if (!PREFETCH) {
            c = tile_coord<MODE>(p, f * tiles_per_frame + tx);
            stage_load<MODE, TW, THREADS, FLAGS>(p, c, tid, v);
        }
        if (!STATIC || !PREFETCH) ft = p.ftype[f];  // (with a prefetch under kStaticStores: loaded with it)
        if constexpr (S8) {  // biased int8 state: P adds its deltas to the biased values, I adds the bias
            if (__builtin_amdgcn_readfirstlane(ft) != 0) {
#pragma unroll
                for (int k = 0; k < T::CHUNKS; k++) {
                    const u32x4 o = unpack8_biased(*reinterpret_cast<const uint2*>(st8(k, tid))), d = v[k];
                    const u32x4 n = {add_u16x2(o.x, d.x), add_u16x2(o.y, d.y), add_u16x2(o.z, d.z), add_u16x2(o.w, d.w)};
                    *reinterpret_cast<uint2*>(st8(k, tid)) = pack8_biased(n, wide8);
                }
            } else {
#pragma unroll
                for (int k = 0; k < T::CHUNKS; k++) *reinterpret_cast<uint2*>(st8(k, tid)) = pack8(v[k], wide8);
            }
        } else {
            if (__builtin_amdgcn_readfirstlane(ft) != 0) {  // P: accumulate deltas onto the state (each chunk has one owner lane)
#pragma unroll
                for (int k = 0; k < T::CHUNKS; k++) {
                    const u32x4 o = *reinterpret_cast<const u32x4*>(
                                        state + coef_off(T::SLOTS_PER_CHUNK * k + (tid >> 3), tid & 7)),
                                d = v[k];
                    v[k] = (u32x4){add_u16x2(o.x, d.x), add_u16x2(o.y, d.y), add_u16x2(o.z, d.z), add_u16x2(o.w, d.w)};
                }
            }
            stage_store<MODE, TW, THREADS, kDefaultFlags>(state, tid, v);
        }
        __syncthreads();
        TileCoord cn = c;
        // The next frame's loads are issued on every iteration (stage_load_or_skip: after the last
        // frame of the segment they read nothing), so v is dead between its use above and here.
        const bool last = f + 1 >= f1;
        const uint32_t fn = last ? f : f + 1;
        if (EARLY) {  // v is free again: next frame's loads overlap the IDCT too
            cn = tile_coord<MODE>(p, fn * tiles_per_frame + tx);
            stage_load_or_skip<MODE, TW, THREADS, FLAGS>(p, cn, tid, last, v);
            if (STATIC) ft = p.ftype[fn];
        }
        decode_tile_idct<MODE, TW, THREADS, FLAGS, false>(p, c, state, planes, tid, lds_qt, nullptr, &esc);
        __syncthreads();
        if (!EARLY && PREFETCH) {
            cn = tile_coord<MODE>(p, fn * tiles_per_frame + tx);
            stage_load_or_skip<MODE, TW, THREADS, FLAGS>(p, cn, tid, last, v);
            if (STATIC) ft = p.ftype[fn];
        }
        decode_tile_csc<MODE, TW, THREADS, FLAGS>(p, c, planes, tid);
        // no barrier here: the next frame's staging barrier orders these plane reads
        // before the next IDCT overwrites the planes (state slots and planes are disjoint)
        c = cn;
    }
    // optimistic form: a value outside int8 or a block too wide for the int16 IDCT anywhere in this
    // job marks it (below), and the exact form (kGopFixup) re-runs it, outputs and end state included.
    // A marked job writes no end state, so with one segment state_out may be state_in (the re-run
    // reads state_in again); with several, the launcher hands the kernel a copy of an overlapping
    // state_in (mj423_decode_stream_device): segment 0 reads it while the last segment writes.
    constexpr bool OPTIMISTIC = S8 || (FLAGS & kIdctW16Esc) != 0;
    const uint32_t bad = OPTIMISTIC ? ((S8 ? (wide8 & 0xff00ff00u) : 0u) | esc) : 0u;
    // The barrier makes the last frame's state writes visible to the end-state copy; the job's verdict
    // is OR-reduced through a word of the plane tiles, dead by then (__syncthreads_or would add 256 B
    // of LDS: 4:2:2 would drop from five workgroups per CU to four).
    __syncthreads();
    bool job_bad = false;
    if constexpr (OPTIMISTIC) {
        volatile uint32_t* word = reinterpret_cast<volatile uint32_t*>(planes);
        if (tid == 0) *word = 0u;
        __syncthreads();
        if (bad != 0) *word = 1u;
        __syncthreads();
        job_bad = *word != 0u;
    }
    if (p.state_out && sy + 1 == p.nseg && !job_bad) {  // end state, for a batch that continues this GOP
#pragma unroll
        for (int k = 0; k < T::CHUNKS; k++) {
            const int run = T::chunk_run(k);
            const int col = T::SLOTS_PER_CHUNK * k + (tid >> 3) - T::run_first_slot(run);
            if (col < cs.run_len(run)) {
                u32x4 o;
                if constexpr (S8) {
                    const u32x4 u = unpack8_biased(*reinterpret_cast<const uint2*>(st8(k, tid)));
                    const uint32_t nb = 0xff80ff80u;
                    o = (u32x4){add_u16x2(u.x, nb), add_u16x2(u.y, nb), add_u16x2(u.z, nb), add_u16x2(u.w, nb)};
                } else {
                    o = *reinterpret_cast<const u32x4*>(state + coef_off(T::SLOTS_PER_CHUNK * k + (tid >> 3), tid & 7));
                }
                *reinterpret_cast<u32x4*>(p.state_out + st_off(k)) = o;
            }
        }
    }
    if constexpr (OPTIMISTIC) {
        if (job_bad && tid == 0 && jflag) *jflag = 1u;
    }
    if constexpr ((FLAGS & kGopFixup) != 0) {
        // every wave read the mark before the first barrier: clear it for the next launch
        if (tid == 0) *jflag = 0u;
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
    auto load = [&](int r, uint32_t (&dr)[4]) {
        const uint4 q = src[r];
        dr[0] = qt ? dequant_pair(q.x, qt[4 * r + 0]) : q.x;
        dr[1] = qt ? dequant_pair(q.y, qt[4 * r + 1]) : q.y;
        dr[2] = qt ? dequant_pair(q.z, qt[4 * r + 2]) : q.z;
        dr[3] = qt ? dequant_pair(q.w, qt[4 * r + 3]) : q.w;
    };
    uint32_t o[8][2];
    idct8x8_auto(load, o, true);
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

// One 8x8 block for the reference's per-block symbols, on host-mapped memory, with a
// completion word: op 0 = idct() of one dequantized block (lane 0), op 1 = ycbcr_to_rgb() of
// one 4:4:4 block (a lane per pixel).  The wave's results are made visible system-wide
// before lane 0 stores `seq` into *done, so the host can spin on that word instead of
// waiting for the stream (a synchronisation costs more than the whole call).
__global__ void __launch_bounds__(64) dropin_block_kernel(int op, const uint8_t* __restrict__ in,
                                                          uint8_t* __restrict__ out, uint32_t* done, uint32_t seq) {
    const uint32_t t = threadIdx.x;
    if (op == 0) {
        if (t == 0) {
            const uint4* src = reinterpret_cast<const uint4*>(in);
            uint32_t d[8][4];
#pragma unroll
            for (int r = 0; r < 8; r++) {
                const uint4 q = src[r];
                d[r][0] = q.x;
                d[r][1] = q.y;
                d[r][2] = q.z;
                d[r][3] = q.w;
            }
            uint32_t o[8][2];
            idct8x8(d, o);
            uint2* dst = reinterpret_cast<uint2*>(out);
#pragma unroll
            for (int r = 0; r < 8; r++) dst[r] = make_uint2(o[r][0], o[r][1]);
        }
    } else {
        reinterpret_cast<uint32_t*>(out)[t] = bgra(in[t], chroma_terms(in[64 + t], in[128 + t]));
    }
    __threadfence_system();
    if (t == 0) __hip_atomic_store(done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// The ycbcr_to_rgb() calls queued by the deferred per-block symbols (mj423_dropin.cpp), all
// of one flush in one launch: 16 lanes per call, each converting 4 pixels of one block row
// (ycbcr_to_rgb.c:26-49, the 4:4:4 dot-product form) and writing them as one 16-B store.
__global__ void __launch_bounds__(256) dropin_csc_kernel(const uint8_t* __restrict__ col,
                                                         const DropinCsc* __restrict__ calls, uint32_t n,
                                                         uint32_t* __restrict__ rgb) {
    const uint32_t g = blockIdx.x * 256 + threadIdx.x, ci = g >> 4, l = g & 15;
    if (ci >= n) return;
    const DropinCsc c = calls[ci];
    const uint32_t row = l >> 1, x = (l & 1) * 4, o = row * 8 + x;
    const uint32_t yq = *reinterpret_cast<const uint32_t*>(col + (size_t)c.sy * 64 + o);
    const uint32_t cb4 = *reinterpret_cast<const uint32_t*>(col + (size_t)c.scb * 64 + o);
    const uint32_t cr4 = *reinterpret_cast<const uint32_t*>(col + (size_t)c.scr * 64 + o);
    const CscConst444 k = csc444_consts();
    const u32x4 v = {bgra444<0>(yq, cb4, cr4, k), bgra444<1>(yq, cb4, cr4, k), bgra444<2>(yq, cb4, cr4, k),
                     bgra444<3>(yq, cb4, cr4, k)};
    *reinterpret_cast<u32x4*>(rgb + c.off + (uint64_t)row * c.pitch + x) = v;
}

// Plain 16-B copy, used for small host<->device tables through host-mapped memory (see
// mj423_gpu_frontend.cpp: small hipMemcpyAsync calls could block the host for ~8 ms).
__global__ void __launch_bounds__(256) copy16_kernel(const uint4* __restrict__ src, uint4* __restrict__ dst, uint64_t n) {
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) dst[i] = src[i];
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

// ---------------------------------------------------------------------------------
// Sparse -> dense coefficient planes for the streaming decoder: one 256-lane workgroup
// per 256-block segment of one (frame, plane) task, one lane per block.  The segment's
// 32 KiB of planes is built in LDS (zero, then each lane scatters its entries) and
// written out with coalesced 16-B stores; dense tasks are a straight copy.  Cost is
// HBM-side only (entries read once, planes written once); what it saves is PCIe.
__global__ void __launch_bounds__(256) expand_kernel(const ExpandParams p) {
    __shared__ __attribute__((aligned(16))) uint32_t lds[256 * 32];
    __shared__ uint32_t wave_sum[4];
    const uint32_t seg = blockIdx.x, task = blockIdx.y, tid = threadIdx.x;
    const uint32_t b0 = seg * 256;
    const uint32_t nb = min(256u, p.nblk - b0);
    const uint32_t f = task / 3, plane = task % 3;
    u32x4* out = reinterpret_cast<u32x4*>(p.out + f * p.coef_pf + ((uint64_t)plane * p.nblk + b0) * 64);
    const uint32_t* task_base = reinterpret_cast<const uint32_t*>(p.xfer);
    const uint32_t* task_mode = reinterpret_cast<const uint32_t*>(p.xfer + p.off_mode);
    const uint32_t* ent = reinterpret_cast<const uint32_t*>(p.xfer + p.entries_off) + task_base[task];
    if (task_mode[task] != 0) {  // dense task: the plane's coefficients verbatim
        const u32x4* src = reinterpret_cast<const u32x4*>(ent) + (uint64_t)b0 * 8;
        for (uint32_t i = tid; i < nb * 8; i += 256) __builtin_nontemporal_store(src[i], out + i);
        return;
    }
    u32x4* l4 = reinterpret_cast<u32x4*>(lds);
#pragma unroll
    for (int i = 0; i < 8; i++) l4[i * 256 + tid] = (u32x4){0u, 0u, 0u, 0u};
    // exclusive scan of the per-block counts over the workgroup
    const uint32_t cnt = tid < nb ? p.xfer[p.off_counts + (uint64_t)task * p.nblk + b0 + tid] : 0u;
    uint32_t incl = cnt;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const uint32_t o = __shfl_up(incl, d, 64);
        if ((tid & 63) >= (uint32_t)d) incl += o;
    }
    if ((tid & 63) == 63) wave_sum[tid >> 6] = incl;
    __syncthreads();  // also orders the zeroing before the scatter
    uint32_t before = 0;
    for (uint32_t w = 0; w < (tid >> 6); w++) before += wave_sum[w];
    const uint32_t* seg_off = reinterpret_cast<const uint32_t*>(p.xfer + p.off_seg) + (uint64_t)task * (p.nseg + 1);
    const uint32_t* e = ent + seg_off[seg] + before + incl - cnt;
    uint16_t* blk = reinterpret_cast<uint16_t*>(lds) + tid * 64;
    for (uint32_t i = 0; i < cnt; i++) {
        const uint32_t v = e[i];
        blk[v >> 16] = (uint16_t)v;
    }
    __syncthreads();
    for (uint32_t i = tid; i < nb * 8; i += 256) __builtin_nontemporal_store(l4[i], out + i);
}

// ---------------------------------------------------------------------------------
// GPU entropy front end: the walk of lossless_decode.c:82-134 (quantized domain, SURVEY
// §8 A5) for one (frame, plane) bitstream per WAVE.  A stream is bit-serial, but an .mpg
// holds 3 independent streams per frame and -- with P-frames coded as deltas and
// accumulated later by decode_gop_kernel -- no frame's streams depend on the previous
// frame, so a batch of F frames is 3F independent serial jobs.
//
// The serial walk runs on the scalar unit (window, symbol fields, branches: all
// wave-uniform).  The 64 lanes are its register files: the stream arrives 256 bytes at a
// time as one dword per lane (one vector load, byte-swapped and end-masked in parallel)
// and is read back with v_readlane; the zig-zag table sits one entry per lane; decoded
// coefficients are collected one per lane with v_writelane and stored 64 at a time.  So
// the loop issues no memory instruction per symbol, and the only waits are one per 256
// stream bytes, on a load issued 256 bytes earlier.  Bytes at or past the stream's end
// read as zero, like the bounded host reader.
__global__ void __launch_bounds__(64) entropy_kernel(const EntropyParams p) {
    const uint32_t t = blockIdx.x;
    if (t >= p.ntasks) return;
    if (p.tchg && p.tchg[t] != p.unsettled) return;  // settled by the many-lanes front end
    const uint32_t lane = threadIdx.x;
    const EntropyTask task = p.tasks[t];
    int16_t* out = p.out + (uint64_t)task.frame * p.coef_pf + (uint64_t)task.plane * p.nblk * 64;
    if (p.tchg) {  // the emit pass left this plane untouched: clear it (this wave writes only what the stream sets)
        for (uint64_t i = lane; i < (uint64_t)p.nblk * 8; i += 64) reinterpret_cast<uint4*>(out)[i] = make_uint4(0, 0, 0, 0);
        __threadfence();  // the zeros complete before the coefficient stores below
    }
    const bool P = task.ptype != 0;
    const uint64_t end = task.byte_off + task.nbytes;  // first byte that reads as zero
    const uint32_t zz = kZigzagNat[lane];              // lane k: natural index of zig-zag position k
    asm volatile("" ::"v"(zz));  // land the table before the loop (no per-symbol vmcnt waits on it)
    const uint64_t last_dw = p.bytes_len & ~3ull;       // in-bounds address for lanes past the end
    // This lane's dword of the 256-B chunk at c (raw; branch-free so the load stays in
    // flight until the chunk is consumed) and the mask of its bytes inside the stream.
    auto load_chunk = [&](uint64_t c, uint32_t& m) -> uint32_t {
        const uint64_t a = c + 4 * lane;
        const uint64_t valid = a < end ? end - a : 0;
        m = valid >= 4 ? 0xffffffffu : (1u << (8 * (uint32_t)valid)) - 1u;
        return *reinterpret_cast<const uint32_t*>(p.bytes + (a < end ? a : last_dw));
    };
    const uint64_t chunk0 = task.byte_off & ~255ull;
    uint64_t chunk = chunk0;
    uint32_t cur_m, nxt_m;
    uint32_t cur = load_chunk(chunk, cur_m);
    uint32_t nxt = load_chunk(chunk + 256, nxt_m);
    cur = __builtin_bswap32(cur & cur_m);  // big-endian order, swapped once per chunk on the VALU
    const uint32_t li0 = (uint32_t)((task.byte_off & 255) >> 2);
    uint32_t li = li0;  // next dword of `cur`
    uint64_t win = 0;                                      // MSB-first bit window
    uint32_t n = 0;                                        // valid bits in win
    auto refill = [&]() {
        if (n <= 32) {
            win |= (uint64_t)(uint32_t)__builtin_amdgcn_readlane(cur, li) << (32 - n);  // readlane is int: no sign extension
            n += 32;
            if (++li == 64) {
                cur = __builtin_bswap32(nxt & nxt_m);  // the one wait per 256 stream bytes, on a load 256 bytes old
                chunk += 256;
                nxt = load_chunk(chunk + 256, nxt_m);
                li = 0;
            }
        }
    };
    refill();
    refill();
    {
        const uint32_t skip = (uint32_t)(task.byte_off & 3) * 8;
        win <<= skip;
        n -= skip;
    }
    // output batch: lane k holds the k-th pending (plane position, value)
    uint32_t bpos = 0, bval = 0;
    uint32_t cnt = 0;
    // (readfirstlane: the asm operands below must be SGPRs)
    uint32_t nblk = (uint32_t)__builtin_amdgcn_readfirstlane((int)p.nblk);
    uint32_t Pm = (uint32_t)__builtin_amdgcn_readfirstlane(P ? 1 : 0);
    uint32_t blk = 0, b64 = 0, idx = 1, st = 0;  // b64 = 64 * blk; st: 0 = a DC symbol is next, 1 = AC
    uint32_t dc = 0;                             // I-frame DC running sum (int16, sign-extended)
    // Termination does not depend on the data: every symbol consumes >= 4 bits, bytes past
    // the end read as zero (DC size 0 + EOB: 12 bits per block), and every pass of the outer
    // loop below switches a chunk, flushes a full batch or finishes.  The pass count is
    // still capped (status 2 if ever reached).
    const uint32_t cap = (uint32_t)__builtin_amdgcn_readfirstlane((int)(task.nbytes / 256u + 2u * p.nblk + 64u));
    uint32_t passes = 0;
    // The symbol loop in scalar-unit assembly.  One wave issues at most one instruction
    // per 4 cycles, so the cost is the instruction count on the path plus the stalls on
    // VALU results: an AC coefficient takes 28 (fields by s_bfe, the HUFF_EXTEND offset
    // 1 - 2^size selected on the amplitude's top bit, the batch counter kept in M0 -- the
    // v_writelane lane select), the zig-zag v_readlane is issued before the VLI work that
    // hides its latency, DC and AC states are separate code paths so no symbol tests a
    // state flag, and nothing is counted per symbol (bits consumed are derived from the
    // read position at the end).  It runs until a refill needs a new 256-B chunk,
    // the output batch is full, or the plane is done; the C++ loop around it switches
    // chunks and flushes the batch.  Window in s[80:81] (hi = s81).
    // lossless_decode.c: DC :86-96 (size 4 bits + VLI; I prefix-sums, P the delta), AC
    // :100-129 (run 4 + size 4 + VLI; run 15 size 0 = ZRL, size 0 = EOB, a coefficient
    // at index + run, past 63 skipped and the block ends), HUFF_EXTEND :204.
    auto rfl = [](uint32_t x) -> uint32_t { return (uint32_t)__builtin_amdgcn_readfirstlane((int)x); };
    while (blk < nblk && passes < cap) {
        passes++;
        // the asm's state operands must be SGPRs: pin them (no-ops when already scalar)
        n = rfl(n), li = rfl(li), blk = rfl(blk), b64 = rfl(b64), idx = rfl(idx), st = rfl(st), dc = rfl(dc);
        cnt = rfl(cnt), nblk = rfl(nblk), Pm = rfl(Pm);
        win = ((uint64_t)rfl((uint32_t)(win >> 32)) << 32) | rfl((uint32_t)win);
        asm volatile(
            "s_mov_b32 s95, m0\n\t"
            "s_mov_b32 m0, %[cnt]\n\t"
            "s_mov_b64 s[80:81], %[win]\n\t"
            "s_cmp_eq_u32 %[st], 0\n\t"
            "s_cbranch_scc1 L_dc_%=\n\t"
            "s_branch L_ac_%=\n"
            // refills, out of line (about one symbol in three): the next dword of the chunk
            "L_rac_%=:\n\t"
            "s_cmp_eq_u32 %[li], 64\n\t"
            "s_cbranch_scc1 L_xac_%=\n\t"
            "v_readlane_b32 s92, %[cur], %[li]\n\t"
            "s_mov_b32 s93, 0\n\t"
            "s_sub_u32 s94, 32, %[n]\n\t"
            "s_lshl_b64 s[92:93], s[92:93], s94\n\t"
            "s_or_b64 s[80:81], s[80:81], s[92:93]\n\t"
            "s_add_u32 %[n], %[n], 32\n\t"
            "s_add_u32 %[li], %[li], 1\n\t"
            "s_branch L_hac_%=\n"
            "L_rac2_%=:\n\t"
            "s_cmp_eq_u32 %[li], 64\n\t"
            "s_cbranch_scc1 L_xac_%=\n\t"
            "v_readlane_b32 s92, %[cur], %[li]\n\t"
            "s_mov_b32 s93, 0\n\t"
            "s_sub_u32 s94, 32, %[n]\n\t"
            "s_lshl_b64 s[92:93], s[92:93], s94\n\t"
            "s_or_b64 s[80:81], s[80:81], s[92:93]\n\t"
            "s_add_u32 %[n], %[n], 32\n\t"
            "s_add_u32 %[li], %[li], 1\n\t"
            "s_branch L_hac2_%=\n"
            "L_rdc_%=:\n\t"
            "s_cmp_eq_u32 %[li], 64\n\t"
            "s_cbranch_scc1 L_xdc_%=\n\t"
            "v_readlane_b32 s92, %[cur], %[li]\n\t"
            "s_mov_b32 s93, 0\n\t"
            "s_sub_u32 s94, 32, %[n]\n\t"
            "s_lshl_b64 s[92:93], s[92:93], s94\n\t"
            "s_or_b64 s[80:81], s[80:81], s[92:93]\n\t"
            "s_add_u32 %[n], %[n], 32\n\t"
            "s_add_u32 %[li], %[li], 1\n\t"
            "s_branch L_hdc_%=\n"
            // ---- DC symbol (block start)
            "L_dc_%=:\n\t"
            "s_cmp_le_u32 %[n], 32\n\t"
            "s_cbranch_scc1 L_rdc_%=\n"
            "L_hdc_%=:\n\t"
            "s_lshr_b32 s91, s81, 28\n\t"               // size
            "s_lshl_b64 s[80:81], s[80:81], 4\n\t"
            "s_sub_u32 %[n], %[n], 4\n\t"
            "s_lshl_b32 s96, 1, s91\n\t"
            "s_sub_u32 s96, 1, s96\n\t"                // 1 - 2^size (0 when size = 0)
            "s_lshr_b32 s92, s81, 1\n\t"                // v = top `size` bits (0 when size = 0)
            "s_sub_u32 s93, 31, s91\n\t"
            "s_lshr_b32 s92, s92, s93\n\t"
            "s_cmp_gt_i32 s81, -1\n\t"                  // top bit 0: negative amplitude
            "s_cselect_b32 s96, s96, 0\n\t"
            "s_add_u32 s92, s92, s96\n\t"               // e
            "s_lshl_b64 s[80:81], s[80:81], s91\n\t"
            "s_sub_u32 %[n], %[n], s91\n\t"
            "s_add_u32 %[dc], %[dc], s92\n\t"
            "s_sext_i32_i16 %[dc], %[dc]\n\t"
            "s_cmp_eq_u32 %[P], 0\n\t"
            "s_cselect_b32 s92, %[dc], s92\n\t"         // I: the running sum; P: the delta
            "s_mov_b32 %[idx], 1\n\t"
            "s_and_b32 s93, s92, 0xffff\n\t"            // SCC = value != 0
            "s_cbranch_scc0 L_ac_%=\n\t"
            "v_writelane_b32 %[bpos], %[b64], m0\n\t"
            "v_writelane_b32 %[bval], s92, m0\n\t"
            "s_add_u32 m0, m0, 1\n\t"
            "s_cmp_eq_u32 m0, 64\n\t"
            "s_cbranch_scc1 L_xac_%=\n"
            // ---- AC symbol
            "L_ac_%=:\n\t"
            "s_cmp_le_u32 %[n], 32\n\t"
            "s_cbranch_scc1 L_rac_%=\n"
            "L_hac_%=:\n\t"
            "s_bfe_u32 s91, s81, 0x40018\n\t"           // size = bits 27:24
            "s_bfe_u32 s94, s81, 0x4001c\n\t"           // run  = bits 31:28
            "s_lshl_b64 s[80:81], s[80:81], 8\n\t"
            "s_sub_u32 %[n], %[n], 8\n\t"
            "s_cmp_eq_u32 s91, 0\n\t"
            "s_cbranch_scc1 L_zero_%=\n\t"
            "s_add_u32 %[idx], %[idx], s94\n\t"
            "s_min_u32 s97, %[idx], 63\n\t"            // a lane select inside the wave (idx is unused past 63)
            "v_readlane_b32 s93, %[zz], s97\n\t"      // early: its latency hides under the VLI work
            "s_lshl_b32 s96, 1, s91\n\t"
            "s_sub_u32 s96, 1, s96\n\t"                // 1 - 2^size
            "s_sub_u32 s97, 32, s91\n\t"
            "s_lshr_b32 s92, s81, s97\n\t"
            "s_cmp_gt_i32 s81, -1\n\t"
            "s_cselect_b32 s96, s96, 0\n\t"
            "s_add_u32 s92, s92, s96\n\t"
            "s_lshl_b64 s[80:81], s[80:81], s91\n\t"
            "s_sub_u32 %[n], %[n], s91\n\t"
            "s_cmp_gt_u32 %[idx], 62\n\t"
            "s_cbranch_scc1 L_last_%=\n\t"
            "s_add_u32 s94, %[b64], s93\n\t"
            "v_writelane_b32 %[bpos], s94, m0\n\t"
            "v_writelane_b32 %[bval], s92, m0\n\t"
            "s_add_u32 m0, m0, 1\n\t"
            "s_add_u32 %[idx], %[idx], 1\n\t"
            "s_cmp_eq_u32 m0, 64\n\t"
            "s_cbranch_scc1 L_xac_%=\n"
            // ---- the same AC code once more, so the loop-back branch is taken every other
            //      symbol (a taken branch costs about five instructions here: -5 % per launch;
            //      moving EOB -> DC onto fall-through paths too measured +6 %, kept out)
            "L_ac2_%=:\n\t"
            "s_cmp_le_u32 %[n], 32\n\t"
            "s_cbranch_scc1 L_rac2_%=\n"
            "L_hac2_%=:\n\t"
            "s_bfe_u32 s91, s81, 0x40018\n\t"           // size = bits 27:24
            "s_bfe_u32 s94, s81, 0x4001c\n\t"           // run  = bits 31:28
            "s_lshl_b64 s[80:81], s[80:81], 8\n\t"
            "s_sub_u32 %[n], %[n], 8\n\t"
            "s_cmp_eq_u32 s91, 0\n\t"
            "s_cbranch_scc1 L_zero_%=\n\t"
            "s_add_u32 %[idx], %[idx], s94\n\t"
            "s_min_u32 s97, %[idx], 63\n\t"            // a lane select inside the wave (idx is unused past 63)
            "v_readlane_b32 s93, %[zz], s97\n\t"      // early: its latency hides under the VLI work
            "s_lshl_b32 s96, 1, s91\n\t"
            "s_sub_u32 s96, 1, s96\n\t"                // 1 - 2^size
            "s_sub_u32 s97, 32, s91\n\t"
            "s_lshr_b32 s92, s81, s97\n\t"
            "s_cmp_gt_i32 s81, -1\n\t"
            "s_cselect_b32 s96, s96, 0\n\t"
            "s_add_u32 s92, s92, s96\n\t"
            "s_lshl_b64 s[80:81], s[80:81], s91\n\t"
            "s_sub_u32 %[n], %[n], s91\n\t"
            "s_cmp_gt_u32 %[idx], 62\n\t"
            "s_cbranch_scc1 L_last_%=\n\t"
            "s_add_u32 s94, %[b64], s93\n\t"
            "v_writelane_b32 %[bpos], s94, m0\n\t"
            "v_writelane_b32 %[bval], s92, m0\n\t"
            "s_add_u32 m0, m0, 1\n\t"
            "s_add_u32 %[idx], %[idx], 1\n\t"
            "s_cmp_eq_u32 m0, 64\n\t"
            "s_cbranch_scc0 L_ac_%=\n\t"
            "s_branch L_xac_%=\n"
            // index 63: write, then the block ends; past 63: no write (UB in the reference)
            "L_last_%=:\n\t"
            "s_cmp_gt_u32 %[idx], 63\n\t"
            "s_cbranch_scc1 L_eob_%=\n\t"
            "s_add_u32 s94, %[b64], s93\n\t"          // s93 = zz[63], read above
            "v_writelane_b32 %[bpos], s94, m0\n\t"
            "v_writelane_b32 %[bval], s92, m0\n\t"
            "s_add_u32 m0, m0, 1\n\t"
            "s_branch L_eob_%=\n"
            "L_zero_%=:\n\t"                              // size 0: ZRL (run 15) or EOB
            "s_cmp_eq_u32 s94, 15\n\t"
            "s_cbranch_scc0 L_eob_%=\n\t"
            "s_add_u32 %[idx], %[idx], 16\n\t"
            "s_min_u32 %[idx], %[idx], 64\n\t"       // a ZRL run past index 63 stays at 64 (lossless_decode.c:107-110 + the cap of every other walk)
            "s_branch L_ac_%=\n"
            "L_eob_%=:\n\t"
            "s_add_u32 %[blk], %[blk], 1\n\t"
            "s_add_u32 %[b64], %[b64], 64\n\t"
            "s_cmp_eq_u32 m0, 64\n\t"
            "s_cbranch_scc1 L_xdc_%=\n\t"
            "s_cmp_ge_u32 %[blk], %[nblk]\n\t"
            "s_cbranch_scc0 L_dc_%=\n"
            "L_xdc_%=:\n\t"                               // exit, a DC symbol next
            "s_mov_b32 %[st], 0\n\t"
            "s_branch L_out_%=\n"
            "L_xac_%=:\n\t"                               // exit, an AC symbol next
            "s_mov_b32 %[st], 1\n"
            "L_out_%=:\n\t"
            "s_mov_b64 %[win], s[80:81]\n\t"
            "s_mov_b32 %[cnt], m0\n\t"
            "s_mov_b32 m0, s95"
            : [win] "+s"(win), [n] "+s"(n), [li] "+s"(li), [blk] "+s"(blk), [b64] "+s"(b64), [idx] "+s"(idx),
              [st] "+s"(st), [dc] "+s"(dc), [cnt] "+s"(cnt), [bpos] "+v"(bpos), [bval] "+v"(bval),
              [nblk] "+s"(nblk), [P] "+s"(Pm)  // read-only; in/out keeps them in SGPRs
            : [cur] "v"(cur), [zz] "v"(zz)
            : "s80", "s81", "s91", "s92", "s93", "s94", "s95", "s96", "s97", "scc");
        if (cnt == 64) {  // batch full: one store per lane
            out[bpos] = (int16_t)bval;
            cnt = 0;
        }
        if (n <= 32 && li == 64) {  // chunk exhausted: the one wait per 256 stream bytes
            cur = __builtin_bswap32(nxt & nxt_m);
            chunk += 256;
            nxt = load_chunk(chunk + 256, nxt_m);
            li = 0;
        }
    }
    if (lane < cnt) out[bpos] = (int16_t)bval;
    // bits consumed = dwords moved into the window * 32 - bits still in it - the start skip
    const uint32_t dwords = (uint32_t)((chunk - chunk0) >> 2) + li - li0;
    const uint32_t used = 32u * dwords - n - (uint32_t)(task.byte_off & 3) * 8u;
    if (lane == 0) p.status[t] = blk < p.nblk ? 2u : (used > 8u * task.nbytes ? 1u : 0u);
}

}  // namespace mj423

// ------------------------------------------------------------------ launchers
extern "C" hipError_t mj423_launch_decode(const mj423::DecodeParams* p, uint32_t nframes, int chroma,
                                          hipStream_t stream) {
    const uint64_t tiles = (uint64_t)nframes * p->tiles_per_frame;
    if (tiles == 0) return hipSuccess;
    if (tiles > 0x7fffffffull) return hipErrorInvalidValue;
    // kFgroupXcd maps workgroup b to tile (b % 8) * per + b / 8: a bijection on 8 * per workgroups
    const dim3 grid((uint32_t)(p->fgroup == mj423::kFgroupXcd ? 8 * ((tiles + 7) / 8) : tiles));
    using namespace mj423;
    switch (chroma) {
    case 420: hipLaunchKernelGGL((decode_kernel<420, kTw420, kThreads420>), grid, dim3(kThreads420), 0, stream, *p); break;
    case 422: hipLaunchKernelGGL((decode_kernel<422, kTw422, kThreads422>), grid, dim3(kThreads422), 0, stream, *p); break;
    case 444: hipLaunchKernelGGL((decode_kernel<444, kTw444, kThreads444>), grid, dim3(kThreads444), 0, stream, *p); break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

namespace mj423 {
// Stream-kernel variants: quant tables in LDS for every mode; next frame's loads in flight
// during the CSC (4:2:0, ~120 VGPRs) or during IDCT + CSC (4:2:2 / 4:4:4).  Same-process probe
// (round-2 probe) vs the round-1 variants: 4K 4:2:0 -4.6 %, 1080p 4:2:0 -2.5 %,
// 8K 4:2:2 -9 %, 1080p 4:4:4 -5 %, 640x480 4:4:4 -5 % per launch.  Round 2, loads at the top of
// each frame instead (profiles/r02/stream/): 4K +0.5 %, 1080p -1.2 %, 8K 4:2:2 -1.8 %,
// 640x480 4:4:4 -5 %, 1080p 4:4:4 -1 %: kept.
// Round 3: the stream kernel keeps the int32-workspace IDCT and the int32 CSC.  Same-process
// A/B with warmed clocks (profiles/r03/ab/): the int16-workspace IDCT gains
// nothing there even without its width test (640x480 4:4:4 0.571 vs 0.568, 1080p 0.638 vs
// 0.640, 4K 0.638 vs 0.634), the test costs 2-11 % (one LDS round trip and a dependent chain
// in front of every frame's transform), and the 16-bit CSC loses 1-2 % at 1080p and 4K: each
// frame's chain is latency-bound, not VALU-bound.  The batch kernel takes both (+2.5-11 %).
// Round 3, later: the next frame's loads are issued on every iteration (stage_load_or_skip), so the
// prefetch registers are dead through the IDCT (4:2:0: 90 VGPRs instead of 112).  Same-process A/B
// against the conditional prefetch (profiles/r03/opt/run3/): 1080p 4:2:0 +3.7 %, 4K +1.1 %, 8K 4:2:2
// +4.9 %, 1080p 4:4:4 +2.9 %, 640x480 4:4:4 -0.5 %.
constexpr int kGopFlags420 = kDefaultFlags | kGopPrefetch | kGopLdsQt | kIdctI32 | kCscI32;
constexpr int kGopFlags422 = kDefaultFlags | kGopEarly | kGopLdsQt | kIdctI32 | kCscI32;
constexpr int kGopFlags444 = kDefaultFlags | kGopEarly | kGopLdsQt | kIdctI32 | kCscI32;
template <int MODE, int TW, int THREADS, int FLAGS>
static void launch_gop2(const DecodeParams* p, dim3 grid, bool static_stores, hipStream_t stream) {
    if (static_stores)
        hipLaunchKernelGGL((decode_gop_kernel<MODE, TW, THREADS, FLAGS | kStaticStores>), grid, dim3(THREADS), 0, stream, *p);
    else
        hipLaunchKernelGGL((decode_gop_kernel<MODE, TW, THREADS, FLAGS>), grid, dim3(THREADS), 0, stream, *p);
}
template <int MODE, int TW, int THREADS, int FLAGS>
static void launch_gop(const DecodeParams* p, dim3 grid, bool static_stores, bool jitter, bool fair, hipStream_t stream) {
    if (jitter)
        launch_gop2<MODE, TW, THREADS, FLAGS | kGopJitter>(p, grid, static_stores, stream);
    else if (fair)
        launch_gop2<MODE, TW, THREADS, FLAGS | kGopFair>(p, grid, static_stores, stream);
    else
        launch_gop2<MODE, TW, THREADS, FLAGS>(p, grid, static_stores, stream);
}
// Workgroups of the exact stream kernel one CU holds at once (its LDS decides).
template <int MODE, int TW, int THREADS, int FLAGS>
constexpr uint32_t gop_wg_per_cu() {
    return (160u * 1024u) / (uint32_t)kGopLds<MODE, TW, THREADS, FLAGS>;
}

// Optimistic stream kernel (round 3), 4:2:2 only: the accumulated state as biased
// int8 in LDS (16 KiB instead of 32: five workgroups per CU instead of three), the int16-workspace
// IDCT with no fall-back branch, the 16-bit CSC and the quant table through scalar loads.  A job
// (segment, tile) in which a value leaves int8 or a block fails the IDCT's width test is marked in
// p.jobflag; the exact kernel then re-runs exactly those jobs (kGopFixup) over the same outputs and
// end state, so the results are the exact kernel's in every case.  Same-process probe
// (profiles/r03/opt/): 8K 4:2:2 0.694 vs 0.668 of 8 TB/s (+3.9 %), the re-run pass
// 7 us when nothing is marked.  At 4:2:0 / 4:4:4 the same form at six workgroups per CU measured
// -1 ... -4 % (4:2:0, 640x480 4:4:4) and +2 % (1080p 4:4:4) -- less than the re-run pass costs.
constexpr int kGopOpt422 = kDefaultFlags | kStaticStores | kGopState8 | kIdctW16Esc | kGopPrefetch | kGopSmemQt;
template <int MODE, int TW, int THREADS, int OPT, int EXACT>
static void launch_gop_opt(const DecodeParams* p, dim3 grid, bool fair, hipStream_t stream) {
    if (fair)
        hipLaunchKernelGGL((decode_gop_kernel<MODE, TW, THREADS, OPT | kGopFair>), grid, dim3(THREADS), 0, stream, *p);
    else
        hipLaunchKernelGGL((decode_gop_kernel<MODE, TW, THREADS, OPT>), grid, dim3(THREADS), 0, stream, *p);
    hipLaunchKernelGGL((decode_gop_kernel<MODE, TW, THREADS, EXACT | kStaticStores | kGopFixup>), grid, dim3(THREADS), 0,
                       stream, *p);
}
}  // namespace mj423


// The fixed-store-count form (kStaticStores) needs 16-B aligned rows, a width that is a
// multiple of 4 pixels and a frame smaller than the 32-bit buffer range; anything else takes
// the branching form (same results).
extern "C" int mj423_gop_static_stores(const mj423::DecodeParams* p) {
    static const bool off = getenv("MJ423_GOP_STATIC") && atoi(getenv("MJ423_GOP_STATIC")) == 0;  // A/B switch
    if (off) return 0;
    return p->aligned16 && (p->width & 3u) == 0 && (uint64_t)p->height * p->out_pitch * 4u < 0x80000000ull;
}

// The optimistic form runs for 4:2:2 when the caller supplies the job marks (p->jobflag, zeroed,
// one uint32 per job) and the fixed-store-count form applies; MJ423_GOP_OPT=0 turns it off (A/B).
extern "C" int mj423_gop_optimistic(const mj423::DecodeParams* p, int chroma) {
    static const bool off = getenv("MJ423_GOP_OPT") && atoi(getenv("MJ423_GOP_OPT")) == 0;
    return !off && chroma == 422 && p->jobflag != nullptr && mj423_gop_static_stores(p);
}

// Workgroup order of the stream kernel: MJ423_GOP_ORDER = tile (default) | eighths | xcd (A/B).
// XCD eighths measured box-dependent (profiles/r02/stream2 run13/14): on one box +1.7 % (4K) to
// +8 % (640x480 4:4:4) over tile order, on another -0.7 % (4K), -0.5 % (1080p), equal (8K 4:2:2),
// -3 % (640x480 4:4:4) through the product library -- tile order stays the default.
// Start jitter (kGopJitter): off by default, MJ423_GOP_JITTER=1 turns it on (A/B switch).  The
// probe (its own hipMalloc'd buffers) gains 1.5-7 % with it on two boxes; through the product
// library (bench.py --mode stream, profiles/r02/stream2 run16) c3 +0.3 %, c2 -0.5 %, c5 +0.1 %,
// c1 -4 % (a single-round grid pays the delay outright).
static bool gop_jitter_default() {
    static const bool on = getenv("MJ423_GOP_JITTER") && atoi(getenv("MJ423_GOP_JITTER")) == 1;
    return on;
}

// Wave priority by frames left (kGopFair) when the grid is at most three rounds of resident
// workgroups.  The SQ issues from the oldest waves first, so of the workgroups that start together
// on a CU the oldest runs ahead and the last one finishes alone, its load, transform and store
// phases no longer overlapped by anyone else's (phase traces, profiles/r03/fair/: in a one-round
// 640x480 grid the first frames of a job take ~3x the last ones).  Priority 3 ... 0 by frames left
// keeps them abreast.  Same-process probe by grid size (profiles/r03/fair/rounds/, 1080p 4:4:4, 1 024
// resident workgroups): 1 round +10.7 %, 1.5 rounds +6.2 %, 2 +4.6 %, 3 +2.9 %, 5 -0.6 %; 640x480
// 4:4:4 (0.95 rounds) +11 %; 1080p 4:2:0 at 1.6 rounds +3.2 %, at 3.45 rounds -1.8 %; 4K (13.7
// rounds) +1.3 %.  MJ423_GOP_FAIR=0 / 1 forces it off / on (A/B switch).
static bool gop_fair(uint64_t jobs, uint64_t tiles_per_frame, uint32_t wg_per_cu) {
    static const int force = getenv("MJ423_GOP_FAIR") ? atoi(getenv("MJ423_GOP_FAIR")) : -1;
    if (force >= 0) return force != 0;
    static std::atomic<int> cus[64];  // CU count per device, 0 = not yet asked (launches may come from several threads)
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return false;
    int n = cus[dev].load(std::memory_order_relaxed);
    if (n == 0) {
        if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) return false;
        cus[dev].store(n, std::memory_order_relaxed);
    }
    // also when one frame's tiles fill the resident workgroups: then the resident jobs belong to one
    // or two GOP segments and walk their frames together, as in a short grid (4K 4:2:0 at 13.7 rounds
    // +1.1 ... +1.6 % in three same-process runs, 8K 4:2:2 +2 ... +3 %, optimistic 8K 4:2:2 +1.2 %;
    // where several segments share the resident set -- 1080p 4:2:0 at 3.45 rounds, 1080p 4:4:4 at 5 --
    // -1.8 % and -0.6 %)
    const uint64_t slots = (uint64_t)n * wg_per_cu;
    return jobs <= 3ull * slots || tiles_per_frame >= slots;
}

static uint32_t gop_order_default() {
    static const uint32_t o = [] {
        const char* e = getenv("MJ423_GOP_ORDER");
        if (e && strcmp(e, "eighths") == 0) return mj423::kGopOrderEighths;
        if (e && strcmp(e, "xcd") == 0) return mj423::kFgroupXcd;
        return 0u;
    }();
    return o;
}

extern "C" hipError_t mj423_launch_decode_gop(const mj423::DecodeParams* pp, uint32_t nseg, int chroma,
                                              hipStream_t stream) {
    const uint64_t tiles = pp->tiles_per_frame;
    if (tiles == 0 || nseg == 0) return hipSuccess;
    if (tiles > 0x7fffffffull || nseg > 65535) return hipErrorInvalidValue;
    mj423::DecodeParams q = *pp;
    q.nseg = nseg;  // the kernel reads p.nseg (end-state write, job bounds): keep it equal to the grid's
    q.gop_order = gop_order_default();
    const uint64_t n1 = q.gop_order == mj423::kGopOrderEighths ? 8 * ((tiles + 7) / 8) * nseg
                        : q.gop_order == mj423::kFgroupXcd   ? 8 * ((tiles * nseg + 7) / 8)
                                                             : 0;
    if (n1 > 0x7fffffffull) return hipErrorInvalidValue;
    const dim3 grid = n1 ? dim3((uint32_t)n1) : dim3((uint32_t)tiles, nseg);
    const mj423::DecodeParams* p = &q;
    const bool st = mj423_gop_static_stores(p) != 0;
    const bool jt = gop_jitter_default();
    using namespace mj423;
    if (!jt && mj423_gop_optimistic(p, chroma)) {
        launch_gop_opt<422, kGop422[0], kGop422[1], kGopOpt422, kGopFlags422>(
            p, grid, gop_fair(tiles * nseg, tiles, gop_wg_per_cu<422, kGop422[0], kGop422[1], kGopOpt422>()), stream);
        return hipGetLastError();
    }
    const uint64_t jobs = tiles * nseg;
    switch (chroma) {
    case 420:
        launch_gop<420, kGop420[0], kGop420[1], kGopFlags420>(
            p, grid, st, jt, gop_fair(jobs, tiles, gop_wg_per_cu<420, kGop420[0], kGop420[1], kGopFlags420>()), stream);
        break;
    case 422:
        launch_gop<422, kGop422[0], kGop422[1], kGopFlags422>(
            p, grid, st, jt, gop_fair(jobs, tiles, gop_wg_per_cu<422, kGop422[0], kGop422[1], kGopFlags422>()), stream);
        break;
    case 444:
        launch_gop<444, kGop444[0], kGop444[1], kGopFlags444>(
            p, grid, st, jt, gop_fair(jobs, tiles, gop_wg_per_cu<444, kGop444[0], kGop444[1], kGopFlags444>()), stream);
        break;
    default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
}

extern "C" hipError_t mj423_launch_expand(const mj423::ExpandParams* p, hipStream_t stream) {
    if (p->ntask == 0 || p->nblk == 0) return hipSuccess;
    if (p->ntask > 65535) return hipErrorInvalidValue;
    hipLaunchKernelGGL(mj423::expand_kernel, dim3(p->nseg, p->ntask), dim3(256), 0, stream, *p);
    return hipGetLastError();
}

extern "C" hipError_t mj423_launch_entropy(const mj423::EntropyParams* p, hipStream_t stream) {
    if (p->ntasks == 0) return hipSuccess;
    hipLaunchKernelGGL(mj423::entropy_kernel, dim3(p->ntasks), dim3(64), 0, stream, *p);
    return hipGetLastError();
}

extern "C" int mj423_tile_max_mcus(int chroma) {
    switch (chroma) {
    case 420: return mj423::kTw420;
    case 422: return mj423::kTw422;
    case 444: return mj423::kTw444;
    default: return 0;
    }
}

// Workgroup order of the batch kernel.  Workgroup b runs on XCD b % 8 (each XCD has its own
// L2).  Frame-major order hands every XCD every eighth tile of a frame; frame-interleaving
// 4 or 8 frames (the round-1 order) gives each XCD a run of tiles inside one frame; the
// XCD-contiguous order gives each XCD one contiguous eighth of the whole batch (a run of
// whole frames).  Same-process probe (profiles/r01/probe_xcd_order.txt) vs
// the frame-interleaved order: 4:2:0 4K +1 / +4.5 / +6 % (three boxes), 1080p +0.7 /
// +1.5 %, 4:2:2 8K +5 %, 4:4:4 1080p +5 %, 640x480 equal.
extern "C" uint32_t mj423_batch_fgroup(int chroma, uint32_t tiles_per_frame) {
    (void)chroma;
    (void)tiles_per_frame;
    return mj423::kFgroupXcd;
}

extern "C" int mj423_gop_tile_max_mcus(int chroma) {
    switch (chroma) {
    case 420: return mj423::kGop420[0];
    case 422: return mj423::kGop422[0];
    case 444: return mj423::kGop444[0];
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

extern "C" hipError_t mj423_launch_dropin_block(int op, const uint8_t* in, uint8_t* out, uint32_t* done, uint32_t seq,
                                                 hipStream_t stream) {
    hipLaunchKernelGGL(mj423::dropin_block_kernel, dim3(1), dim3(64), 0, stream, op, in, out, done, seq);
    return hipGetLastError();
}

extern "C" hipError_t mj423_launch_dropin_csc(const uint8_t* col, const mj423::DropinCsc* calls, uint32_t n,
                                              uint32_t* rgb, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    if (n > (0xffffffffu >> 4)) return hipErrorInvalidValue;
    hipLaunchKernelGGL(mj423::dropin_csc_kernel, dim3((n + 15) / 16), dim3(256), 0, stream, col, calls, n, rgb);
    return hipGetLastError();
}

extern "C" hipError_t mj423_launch_copy16(const void* src, void* dst, uint64_t bytes, hipStream_t stream) {
    const uint64_t n = (bytes + 15) / 16;
    if (n == 0) return hipSuccess;
    const uint32_t grid = (uint32_t)std::min<uint64_t>((n + 255) / 256, 1024);
    hipLaunchKernelGGL(mj423::copy16_kernel, dim3(grid), dim3(256), 0, stream, (const uint4*)src, (uint4*)dst, n);
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
