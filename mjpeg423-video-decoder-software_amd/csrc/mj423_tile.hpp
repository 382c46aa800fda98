// mj423_tile.hpp -- device building blocks of the fused decode kernels (gfx950, wave64):
// tile geometry, the staging loads, the IDCT and CSC passes of one tile, and the
// production flag set that selects among their forms.  The kernels themselves
// (decode_kernel, decode_gop_kernel) and their launchers are in mj423_kernels.hip.
//
// Only production flags exist here.  Forms that were measured and dropped (ablations,
// phase traces, lock-step and priority probes, cache-policy asm variants, the persistent
// batch body) live in git history; DESIGN.md's appendix lists them with their results.
//
// Reference (paths under core0/software/common/libs/mjpeg423/):
//   per-frame body      decoder/mjpeg423_decoder.c:109-124
//   dequant             decoder/lossless_decode.c:89-129
//   idct                decoder/idct.c:22-181
//   ycbcr_to_rgb        decoder/ycbcr_to_rgb.c:26-49
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "mj423_idct.hpp"
#include "mj423_kernels.h"

namespace mj423 {

// Chroma geometry of one MCU.
template <int MODE>
struct Mcu;
template <>
struct Mcu<420> {  // 16x16: 4 Y (2x2) + Cb + Cr
    static constexpr int MW = 16, MH = 16, SX = 2, SY = 2, YPER = 4;
};
template <>
struct Mcu<422> {  // 16x8: 2 Y (2x1) + Cb + Cr
    static constexpr int MW = 16, MH = 8, SX = 2, SY = 1, YPER = 2;
};
template <>
struct Mcu<444> {  // 8x8: Y + Cb + Cr
    static constexpr int MW = 8, MH = 8, SX = 1, SY = 1, YPER = 1;
};

// One workgroup of THREADS lanes decodes a tile of up to TW MCUs of one MCU row.
// Block "slots" (one LDS block each, one IDCT lane each) hold the tile's runs back to
// back: 4:2:0 = Y block row 0 [0,2TW) | Y block row 1 [2TW,4TW) | Cb [4TW,5TW) | Cr [5TW,6TW);
// 4:2:2 = Y [0,2TW) | Cb | Cr;  4:4:4 = Y [0,TW) | Cb | Cr.
template <int MODE, int TW, int THREADS>
struct Tile {
    using M = Mcu<MODE>;
    static constexpr int NSLOT = (M::YPER + 2) * TW;
    static constexpr int YW = TW * M::MW;  // Y plane tile width (px)
    static constexpr int CW = YW / M::SX;  // chroma plane tile width (px)
    static constexpr int CH = 8;           // chroma rows per MCU row, every mode
    static constexpr int PLANE_BYTES = M::MH * YW + 2 * CH * CW;
    static constexpr int COEF_BYTES = NSLOT * 128;
    static constexpr int LDS_BYTES = COEF_BYTES > PLANE_BYTES ? COEF_BYTES : PLANE_BYTES;
    static constexpr int SLOTS_PER_CHUNK = THREADS / 8;  // 8 lanes stage one block (8 rows of 16 B)
    static constexpr int CHUNKS = NSLOT / SLOTS_PER_CHUNK;
    static constexpr int YRUN = MODE == 420 ? 2 * TW : M::YPER * TW;  // blocks per luma run

    // Runs: 0,1 = Y block rows (1 only in 4:2:0), 2 = Cb, 3 = Cr; each starts at a fixed slot.
    static constexpr int run_first_slot(int run) {
        return MODE == 420 ? (run == 0 ? 0 : run == 1 ? 2 * TW : run == 2 ? 4 * TW : 5 * TW)
                           : (run <= 1 ? 0 : run == 2 ? YRUN : YRUN + TW);
    }
    static constexpr int slot_run_c(int s) {
        return MODE == 420 ? (s < 2 * TW ? 0 : s < 4 * TW ? 1 : s < 5 * TW ? 2 : 3)
                           : (s < YRUN ? 0 : s < YRUN + TW ? 2 : 3);
    }
    __device__ static __forceinline__ int slot_run(int s) { return slot_run_c(s); }
    // Staging chunk k of a thread covers slots [k*SLOTS_PER_CHUNK, (k+1)*SLOTS_PER_CHUNK): static run.
    static constexpr int chunk_run(int k) { return slot_run_c(k * SLOTS_PER_CHUNK); }

    static_assert(THREADS % 64 == 0 && NSLOT <= THREADS, "one IDCT lane per slot");
    static_assert(NSLOT % SLOTS_PER_CHUNK == 0, "whole staging chunks");
    static_assert((2 * TW) % SLOTS_PER_CHUNK == 0 && TW % SLOTS_PER_CHUNK == 0, "runs align to staging chunks");
    static_assert((M::YPER * TW) % 64 == 0, "luma/chroma boundary on a wave boundary (uniform quant table)");
    static_assert((TW * M::MW / 4 * CH) % THREADS == 0, "whole CSC iterations");
};

// LDS position of row r of slot s: rows are XOR-swizzled by the slot so that the
// per-lane ds_read_b128 of "row r of my block" spreads over the banks.
__device__ __forceinline__ int coef_off(int s, int r) { return s * 128 + ((r ^ (s & 7)) << 4); }

// Two int16 lanes added mod 2^16 (v_pk_add_u16).  Written on whole scalars: per-element
// assignment into an ext-vector inside the unrolled chunk loop was miscompiled.
__device__ __forceinline__ uint32_t add_u16x2(uint32_t a, uint32_t b) {
    return __builtin_bit_cast(uint32_t, __builtin_bit_cast(u16x2, a) + __builtin_bit_cast(u16x2, b));
}

// kGopState8: a block's accumulated quantized coefficients as 8 rows of 8 bytes, each value
// stored as Q + 128 (offset binary).  Rows swizzled by slot >> 2 so that a wave's 8-byte
// row reads (one lane per slot) and writes (8 lanes per slot) hit distinct banks.
__device__ __forceinline__ int coef_off8(int s, int r) { return s * 64 + (((r ^ (s >> 2)) & 7) << 3); }
// 8 int16 (4 packed pairs) -> 8 biased bytes; `acc` collects the biased values, whose high
// byte is non-zero for any value outside [-128, 127] (then the state does not fit int8).
__device__ __forceinline__ uint2 pack8(const u32x4& v, uint32_t& acc) {
    const uint32_t b = 0x00800080u;
    const uint32_t x = add_u16x2(v.x, b), y = add_u16x2(v.y, b), z = add_u16x2(v.z, b), w = add_u16x2(v.w, b);
    acc |= x | y | z | w;
    return make_uint2(__builtin_amdgcn_perm(y, x, 0x06040200u), __builtin_amdgcn_perm(w, z, 0x06040200u));
}
// The same for values that already carry the +128 bias.
__device__ __forceinline__ uint2 pack8_biased(const u32x4& v, uint32_t& acc) {
    acc |= v.x | v.y | v.z | v.w;
    return make_uint2(__builtin_amdgcn_perm(v.y, v.x, 0x06040200u), __builtin_amdgcn_perm(v.w, v.z, 0x06040200u));
}
// 8 biased bytes -> 8 int16 (4 packed pairs) with the bias still on (+128 each).
__device__ __forceinline__ u32x4 unpack8_biased(uint2 q) {
    return (u32x4){__builtin_amdgcn_perm(0u, q.x, 0x0c010c00u), __builtin_amdgcn_perm(0u, q.x, 0x0c030c02u),
                   __builtin_amdgcn_perm(0u, q.y, 0x0c010c00u), __builtin_amdgcn_perm(0u, q.y, 0x0c030c02u)};
}

// Production tile shapes (MCUs per tile, lanes per workgroup), chosen by same-process A/B.
// (-DMJ423_BATCH_SHAPE420=tw,threads etc. override them for A/B builds, tools/build_variant.sh.)
#ifndef MJ423_BATCH_SHAPE420
#define MJ423_BATCH_SHAPE420 32, 256
#endif
#ifndef MJ423_BATCH_SHAPE422
#define MJ423_BATCH_SHAPE422 64, 256
#endif
#ifndef MJ423_BATCH_SHAPE444
#define MJ423_BATCH_SHAPE444 64, 256
#endif
constexpr int kBatch420[2] = {MJ423_BATCH_SHAPE420}, kBatch422[2] = {MJ423_BATCH_SHAPE422},
              kBatch444[2] = {MJ423_BATCH_SHAPE444};
constexpr int kTw420 = kBatch420[0], kThreads420 = kBatch420[1];
constexpr int kTw422 = kBatch422[0], kThreads422 = kBatch422[1];
constexpr int kTw444 = kBatch444[0], kThreads444 = kBatch444[1];
// Stream (GOP) kernel shapes: its LDS holds the persistent coefficient state next to the
// plane tiles, so it gets its own shapes (override with -DMJ423_GOP_SHAPE420=tw,threads
// for A/B builds, tools/build_variant.sh).
#ifndef MJ423_GOP_SHAPE420
#define MJ423_GOP_SHAPE420 32, 256
#endif
#ifndef MJ423_GOP_SHAPE422
#define MJ423_GOP_SHAPE422 64, 256
#endif
#ifndef MJ423_GOP_SHAPE444
#define MJ423_GOP_SHAPE444 64, 256
#endif
constexpr int kGop420[2] = {MJ423_GOP_SHAPE420}, kGop422[2] = {MJ423_GOP_SHAPE422}, kGop444[2] = {MJ423_GOP_SHAPE444};

// Production flags: the forms of the shared building blocks the launchers in mj423_kernels.hip
// instantiate (bit values are stable: they appear in the kernels' symbol names and profiles).
enum : int {
    kNtLoad = 1,            // coefficient loads non-temporal
    kNtStore = 2,           // BGRA stores non-temporal
    kGopPrefetch = 2048,    // stream kernel: next frame's loads in flight during this frame's CSC
    kGopEarly = 4096,       // stream kernel: ... issued before this frame's IDCT (in flight during IDCT + CSC)
    kGopLdsQt = 8192,       // stream kernel: dequantization tables in LDS (one uniform ds_read_b128 per row)
    kStaticStores = 32768,  // CSC: a fixed number of buffer stores per frame, invalid pixels dropped by
                            // the buffer range check (no branches around stores; see decode_tile_csc)
    kGopFixup = 1 << 21,    // stream kernel: run only the jobs p.jobflag marks, and clear their marks
    kGopJitter = 1 << 23,   // stream kernel: per-workgroup start delay of 0 / 1 / 2 x ~3.4 us (opt-in, MJ423_GOP_JITTER=1)
    kGopSmemQt = 1 << 25,   // stream kernel: dequantization table rows read by scalar loads (SGPRs, no VGPRs)
    kIdctI32 = 1 << 26,     // always the int32-workspace IDCT (the stream kernel's choice)
    kCscI32 = 1 << 27,      // 4:2:x CSC in the int32 form (bgra16 per pixel; the stream kernel's choice)
    kGopState8 = 1 << 29,   // stream kernel: the state in LDS as biased int8, 64 B per block (optimistic form)
    kIdctW16Esc = 1 << 30,  // int16-workspace IDCT always; a lane whose block fails the width test raises its escape
                            // (the optimistic stream kernel: the job is flagged and re-run by the exact form)
    kGopFair = (int)(1u << 31),  // stream kernel: wave priority by frames left in the job, so that the workgroups
                                 // sharing a CU progress together (the arbiter favours old waves)
    kDefaultFlags = kNtLoad | kNtStore
};
constexpr int kProductionFlags = kNtLoad | kNtStore | kGopPrefetch | kGopEarly | kGopLdsQt | kStaticStores |
                                 kGopFixup | kGopJitter | kGopSmemQt | kIdctI32 | kCscI32 | kGopState8 |
                                 kIdctW16Esc | kGopFair;
// Every kernel instantiation checks its flag word against the production set.
template <int FLAGS>
constexpr bool production_flags() {
    return (FLAGS & ~kProductionFlags) == 0;
}

template <typename V>
__device__ __forceinline__ V load16(const V* p, bool nt) {
    return nt ? __builtin_nontemporal_load(p) : *p;
}
template <typename V>
__device__ __forceinline__ void store16(V* p, V v, bool nt) {
    if (nt)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

// Where a tile's four block runs start (int16 elements from p.coef) and how long they are.
struct TileCoord {
    uint32_t f, my, mx0;
    int tw;    // MCUs in this tile = blocks in each chroma run
    int ylen;  // blocks in each luma run
    int64_t off0, off1, off2, off3;
    __device__ __forceinline__ int64_t run_off(int run) const {  // run must be a compile-time constant
        return run == 0 ? off0 : run == 1 ? off1 : run == 2 ? off2 : off3;
    }
    __device__ __forceinline__ int run_len(int run) const { return run < 2 ? ylen : tw; }
};

template <int MODE>
__device__ __forceinline__ TileCoord tile_coord(const DecodeParams& p, uint32_t t) {
    TileCoord c;
    const uint32_t ti = t % p.tiles_per_frame;
    c.f = t / p.tiles_per_frame;
    const int64_t fbase = (int64_t)c.f * (int64_t)p.plane_fstride;
    int64_t coff;
    if (MODE == 420) {  // strip of tw MCUs inside MCU row my
        c.my = ti / p.tiles_per_row;
        c.mx0 = (ti % p.tiles_per_row) * p.tw;
        c.tw = (int)min(p.tw, p.mcu_cols - c.mx0);
        c.off0 = fbase + ((int64_t)(2 * c.my) * p.y_bw + 2 * c.mx0) * 64;
        c.off1 = c.off0 + (int64_t)p.y_bw * 64;
        c.ylen = 2 * c.tw;
        coff = fbase + ((int64_t)c.my * p.c_bw + c.mx0) * 64;
    } else {  // raster run of tw MCUs starting at MCU m0 (kept in mx0), possibly wrapping rows
        constexpr int YPER = MODE == 422 ? 2 : 1;
        c.my = 0;
        c.mx0 = ti * p.tw;
        c.tw = (int)min(p.tw, p.mcus_per_frame - c.mx0);
        c.off0 = c.off1 = fbase + (int64_t)YPER * c.mx0 * 64;
        c.ylen = YPER * c.tw;
        coff = fbase + (int64_t)c.mx0 * 64;
    }
    c.off2 = coff + p.cb_off;
    c.off3 = coff + p.cr_off;
    return c;
}

// Stage, part 1: issue this lane's 16-B loads of the tile (HBM -> VGPRs).
// Chunk k of thread t is (slot k*THREADS/8 + t/8, row t%8): a wave reads 1 KiB contiguous.
// Slots past the end of a short (edge) tile re-read block 0 of their run -- the same
// cache lines the wave already fetches -- so the code stays branch-free and moves no
// extra HBM bytes; those slots are never computed.
template <int MODE, int TW, int THREADS, int FLAGS>
__device__ __forceinline__ void stage_load(const DecodeParams& p, const TileCoord& c, int tid,
                                           u32x4 (&v)[Tile<MODE, TW, THREADS>::CHUNKS]) {
    using T = Tile<MODE, TW, THREADS>;
#pragma unroll
    for (int k = 0; k < T::CHUNKS; k++) {
        const int run = T::chunk_run(k);
        const int col = T::SLOTS_PER_CHUNK * k + (tid >> 3) - T::run_first_slot(run);
        const int colc = col < c.run_len(run) ? col : 0;
        v[k] = load16(reinterpret_cast<const u32x4*>(p.coef + c.run_off(run) + colc * 64 + (tid & 7) * 8),
                      (FLAGS & kNtLoad) != 0);
    }
}

// The same loads as raw buffer loads, one buffer resource per block run, issued on every path:
// with `skip` (wave-uniform) every offset lies past the resource's range, so the hardware returns
// zeros and reads nothing.  The stream kernel's prefetch uses it so that v is written on every
// path through the frame loop: a prefetch behind `if (f + 1 < f1)` left the compiler unable to
// prove v dead during the IDCT (the loop may continue without the branch, as far as it knows), so
// v's 16-24 VGPRs stayed live across the transform -- at six waves per SIMD 20-32 registers spilled.
template <int MODE, int TW, int THREADS, int FLAGS>
__device__ __forceinline__ void stage_load_or_skip(const DecodeParams& p, const TileCoord& c, int tid, bool skip,
                                                   u32x4 (&v)[Tile<MODE, TW, THREADS>::CHUNKS]) {
    using T = Tile<MODE, TW, THREADS>;
    constexpr int aux = (FLAGS & kNtLoad) ? 2 : 0;  // nt
    // each resource starts at its run (a few KiB are read from it): 0x80000000 is past every range
    const uint32_t lane_off = (uint32_t)(tid & 7) * 16u;
#pragma unroll
    for (int k = 0; k < T::CHUNKS; k++) {
        const int run = T::chunk_run(k);
        const int col = T::SLOTS_PER_CHUNK * k + (tid >> 3) - T::run_first_slot(run);
        const int colc = col < c.run_len(run) ? col : 0;
        const __amdgpu_buffer_rsrc_t r =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<int16_t*>(p.coef + c.run_off(run)), 0, 0x7fffffff, 0x00020000);
        const uint32_t off = skip ? 0x80000000u : (uint32_t)colc * 128u + lane_off;
        v[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, aux));
    }
}

// Stage, part 2: VGPRs -> LDS coefficient slots.
template <int MODE, int TW, int THREADS, int FLAGS>
__device__ __forceinline__ void stage_store(uint8_t* lds, int tid, const u32x4 (&v)[Tile<MODE, TW, THREADS>::CHUNKS]) {
    using T = Tile<MODE, TW, THREADS>;
#pragma unroll
    for (int k = 0; k < T::CHUNKS; k++)
        *reinterpret_cast<u32x4*>(lds + coef_off(T::SLOTS_PER_CHUNK * k + (tid >> 3), tid & 7)) = v[k];
}

// Row r of a wave-uniform dequantization table in global memory, read through the constant
// address space so the compiler emits scalar loads (SGPR results; the table is never written).
__device__ __forceinline__ uint4 qt_row_smem(const uint32_t* base, int r) {
    typedef const __attribute__((address_space(4))) uint32_t cu32;
    cu32* c = (cu32*)base;
    return make_uint4(c[4 * r + 0], c[4 * r + 1], c[4 * r + 2], c[4 * r + 3]);
}

// IDCT of one staged tile: quantized blocks in LDS slots at `coef`, a barrier passed.
// The uint8 plane tiles go to `planes`; with ALIAS they overlay `coef` (the slots are
// dead once every lane holds its block in registers: barrier below).  The caller
// places a barrier between this and decode_tile_csc().
template <int MODE, int TW, int THREADS, int FLAGS, bool ALIAS>
__device__ __forceinline__ void decode_tile_idct(const DecodeParams& p, const TileCoord& c, const uint8_t* coef,
                                                 uint8_t* planes, int tid, const uint32_t* lds_qt = nullptr,
                                                 const uint32_t* qregs = nullptr, uint32_t* esc = nullptr) {
    using L = Mcu<MODE>;
    using T = Tile<MODE, TW, THREADS>;
    // ---- IDCT: one lane per slot; the wave's plane class (Y or chroma) is uniform,
    //      so its dequantization table is read through SGPRs.
    const int s = tid;
    const int run = T::slot_run(s);
    const int col = s - (run == 0 ? T::run_first_slot(0) : run == 1 ? T::run_first_slot(1)
                                  : run == 2 ? T::run_first_slot(2) : T::run_first_slot(3));
    const bool active = s < T::NSLOT && col < c.run_len(run);
    if (ALIAS && T::NSLOT % 64 == 0 && __builtin_amdgcn_readfirstlane(s) >= T::NSLOT) {
        // whole waves without a block (4:2:0 / 4:4:4: the 4th wave): only the barrier.  Taking
        // this wave-uniform exit keeps d out of their registers -- inside a frame loop the
        // "undefined" d of the branch below was carried as extra copies (~20 VGPRs)
        __syncthreads();
        return;
    }
    const int wave_chroma = __builtin_amdgcn_readfirstlane(run >= 2 ? 1 : 0);
    // ALIAS == false (stream kernel, a frame loop): read the device copy through one
    // computed pointer, so only this wave's 32-dword table occupies SGPRs (selecting
    // between the two kernel-argument tables kept both live: 64 SGPRs, spilled).
    // kGopLdsQt: the stream kernel's LDS copy, read with one uniform ds_read_b128 per row
    // (a global read through qt_dev is a vector load with L2 latency every frame).
    const uint32_t* qt = (FLAGS & kGopLdsQt) ? lds_qt + 32 * wave_chroma
                         : ALIAS            ? p.qt[wave_chroma]
                                            : p.qt_dev + 32 * wave_chroma;
    // Row r of this lane's block, dequantized: (int16)(Q * q) two coefficients at a time.
    auto row = [&](int r, uint32_t (&dr)[4]) {
        uint4 q;
        if constexpr ((FLAGS & kGopState8) != 0) {  // biased bytes -> int16: Q = byte - 128
            const u32x4 u = unpack8_biased(*reinterpret_cast<const uint2*>(coef + coef_off8(s, r)));
            const uint32_t nb = 0xff80ff80u;  // -128 in both halves
            q = make_uint4(add_u16x2(u.x, nb), add_u16x2(u.y, nb), add_u16x2(u.z, nb), add_u16x2(u.w, nb));
        } else {
            q = *reinterpret_cast<const uint4*>(coef + coef_off(s, r));
        }
        // qregs: the wave's table already in SGPRs (a local array, fully unrolled)
        const uint4 t = qregs ? make_uint4(qregs[4 * r + 0], qregs[4 * r + 1], qregs[4 * r + 2], qregs[4 * r + 3])
                        : (FLAGS & kGopSmemQt) ? qt_row_smem(p.qt_dev + 32 * wave_chroma, r)
                        : (FLAGS & kGopLdsQt) ? *reinterpret_cast<const uint4*>(qt + 4 * r)
                                              : make_uint4(qt[4 * r + 0], qt[4 * r + 1], qt[4 * r + 2], qt[4 * r + 3]);
        dr[0] = dequant_pair(q.x, t.x);
        dr[1] = dequant_pair(q.y, t.y);
        dr[2] = dequant_pair(q.z, t.z);
        dr[3] = dequant_pair(q.w, t.w);
    };
    uint8_t* yplane = planes;
    uint8_t* cbplane = planes + L::MH * T::YW;
    uint8_t* crplane = cbplane + T::CH * T::CW;
    // One complete pass: the block into registers, (ALIAS) the barrier after which its slot may
    // become plane tiles, the transform, the 8 LDS rows of bytes.  FORM: 0 = int16 workspace,
    // 1 = int32 workspace, 3 = int16 workspace with the escape (no fall-back branch).
    auto pass = [&](auto form) {
        constexpr int FORM = decltype(form)::value;
        uint32_t d[8][4];
        if (s >= T::NSLOT) {  // lanes without a block: leave d undefined (no zero-fill movs; never used)
#pragma unroll
            for (int r = 0; r < 8; r++) asm("" : "=v"(d[r][0]), "=v"(d[r][1]), "=v"(d[r][2]), "=v"(d[r][3]));
        } else {
#pragma unroll
            for (int r = 0; r < 8; r++) row(r, d[r]);
        }
        if (ALIAS) __syncthreads();  // every coefficient is in registers: the slots may become plane tiles
        if (active) {
            uint32_t o[8][2];
            if constexpr (FORM == 1) {
                idct8x8(d, o);
            } else if constexpr (FORM == 3) {
                // kIdctW16Esc: the width test on the registers already loaded, no branch -- a
                // block over the bound only raises the escape (its job is re-run exactly)
                int32_t e[4] = {0, 0, 0, 0};
#pragma unroll
                for (int r = 0; r < 8; r++)
#pragma unroll
                    for (int k = 0; k < 4; k++) e[k] = sdot2_sat(d[r][k], e[k]);
                if (max(max(e[0], e[1]), max(e[2], e[3])) > kWs16Energy) *esc = 1u;
                idct8x8_w16(d, o);
            } else {
                idct8x8_w16(d, o);
            }
            uint8_t* dstp = run < 2 ? yplane + (run * 8) * T::YW + col * 8 : (run == 2 ? cbplane : crplane) + col * 8;
            const int pitch = run < 2 ? T::YW : T::CW;
#pragma unroll
            for (int r = 0; r < 8; r++) *reinterpret_cast<uint2*>(dstp + r * pitch) = make_uint2(o[r][0], o[r][1]);
        }
    };
    using F16 = std::integral_constant<int, 0>;
    using F32 = std::integral_constant<int, 1>;
    if constexpr ((FLAGS & kIdctI32) != 0) return pass(F32{});
    if constexpr ((FLAGS & kIdctW16Esc) != 0) return pass(std::integral_constant<int, 3>{});
    // The int16-workspace IDCT unless a block of this wave is too wide for it (mj423_idct.hpp).
    // The test is a pass of its own over the LDS rows (8 ds_read_b128 + the dequantization +
    // 32 saturating dot products, the registers dropped again), so each branch below is a
    // complete, separate pass: deciding on a block already held in registers made the register
    // allocator keep ~25-30 VGPRs more than either transform needs alone (spills at 6 waves per
    // SIMD).
    bool wide = false;
    if (active) {
        int32_t e[4] = {0, 0, 0, 0};
#pragma unroll
        for (int r = 0; r < 8; r++) {
            uint32_t dr[4];
            row(r, dr);
#pragma unroll
            for (int k = 0; k < 4; k++) e[k] = sdot2_sat(dr[k], e[k]);
        }
        wide = max(max(e[0], e[1]), max(e[2], e[3])) > kWs16Energy;
    }
    if (__builtin_amdgcn_ballot_w64(wide) == 0)
        pass(F16{});
    else
        pass(F32{});
}

// CSC of one tile whose uint8 plane tiles are in LDS at `planes` (a barrier passed).
template <int MODE, int TW, int THREADS, int FLAGS>
__device__ __forceinline__ void decode_tile_csc(const DecodeParams& p, const TileCoord& c, const uint8_t* planes,
                                                int tid) {
    using L = Mcu<MODE>;
    using T = Tile<MODE, TW, THREADS>;
    const int tw = c.tw;
    const uint32_t f = c.f, my = c.my, mx0 = c.mx0;
    const uint8_t* yplane = planes;
    const uint8_t* cbplane = planes + L::MH * T::YW;
    const uint8_t* crplane = cbplane + T::CH * T::CW;

    // ---- CSC: a lane takes 4 horizontally adjacent pixels of every luma row that
    //      shares one chroma row (2 rows in 4:2:0), computes the chroma terms once,
    //      and writes 16 B per row: a wave stores 1 KiB of contiguous BGRA.
    constexpr int QPR = T::YW / 4;          // quads per tile row
    constexpr int JOBS = QPR * T::CH;       // (quad, chroma row) pairs
    constexpr int ITERS = JOBS / THREADS;
    static_assert(JOBS % THREADS == 0, "whole CSC iterations");
    constexpr int QPM = L::MW / 4;          // quads per MCU row
    const int qcols = tw * QPM;             // quads present in this tile
    const uint32_t x_tile = mx0 * L::MW, y_tile = my * L::MH;  // 4:2:0 strips
    uint32_t* outf = p.out + (size_t)f * p.out_fstride;
    const CscConst444 k444 = csc444_consts();  // 4:4:4 per-pixel sums; 4:2:x the chroma terms' offsets
    // kStaticStores (stream kernel): every lane issues the same, compile-time number of store
    // instructions per frame -- pixels outside the frame (edge tiles, the coded rows below a
    // 1080-row frame, a ragged right edge) get a byte offset past the buffer's num_records and
    // the hardware range check drops them.  With no branch around a store, the compiler knows
    // how many stores follow the next frame's prefetched loads and waits for those loads with
    // vmcnt(#stores) instead of vmcnt(0): the frame loop never waits for its own stores to
    // drain to HBM (gfx9 counts loads and stores in one in-order vmcnt).
    constexpr bool STATIC = (FLAGS & kStaticStores) != 0;
    // (unused, and dropped by the compiler, without kStaticStores; the host selects that path
    // only for frames of < 2 GiB, rows * pitch * 4 bytes, with 16-B aligned rows and a width
    // that is a multiple of 4 pixels: one 16-B store per lane and row)
    const uint32_t nrec = (uint32_t)((uint64_t)p.height * p.out_pitch * 4u);
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(outf, 0, (int)nrec, 0x00020000);
    const uint32_t oob = nrec;  // the first byte past the frame: out of range, and no 32-bit wrap in the check
    constexpr int UNROLL = STATIC ? ITERS : 1;
#pragma unroll UNROLL
    for (int it = 0; it < ITERS; it++) {
        const int job = it * THREADS + tid;
        const int qc = job % QPR, cy = job / QPR;
        const bool qvalid = qc < qcols;
        if (!STATIC && !qvalid) continue;
        ChromaT ct[2];  // 4:2:x: the two chroma samples of this quad, each shared by a pixel pair
        ChromaTerms ct32[2];  // (kCscI32 only)
        uint32_t cb4 = 0, cr4 = 0;
        if (MODE == 444) {  // per-pixel dot products below (bgra444)
            cb4 = *reinterpret_cast<const uint32_t*>(cbplane + cy * T::CW + qc * 4);
            cr4 = *reinterpret_cast<const uint32_t*>(crplane + cy * T::CW + qc * 4);
        } else if (L::SX == 2) {
            const uint32_t cb2 = *reinterpret_cast<const uint16_t*>(cbplane + cy * T::CW + qc * 2);
            const uint32_t cr2 = *reinterpret_cast<const uint16_t*>(crplane + cy * T::CW + qc * 2);
            if (FLAGS & kCscI32) {
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    const ChromaTerms t = chroma_terms((cb2 >> (8 * i)) & 0xff, (cr2 >> (8 * i)) & 0xff);
                    ct32[i] = t;
                }
            } else {
                ct[0] = chroma_t(__builtin_amdgcn_perm(cr2, cb2, 0x0c040c00u), k444);  // {Cb0, Cr0}
                ct[1] = chroma_t(__builtin_amdgcn_perm(cr2, cb2, 0x0c050c01u), k444);  // {Cb1, Cr1}
            }
        }
        uint32_t gx, gy0;
        if (MODE == 420) {
            gx = x_tile + qc * 4;
            gy0 = y_tile;
        } else {  // raster run: MCU m0 + qc / QPM, at (m % mcu_cols, m / mcu_cols)
            const uint32_t m = mx0 + (uint32_t)(qc / QPM);
            uint32_t row = __umulhi(m, p.cols_magic);  // floor(m / mcu_cols) or one less
            uint32_t col = m - row * p.mcu_cols;
            if (col >= p.mcu_cols) {
                col -= p.mcu_cols;
                row++;
            }
            gx = col * L::MW + (qc % QPM) * 4;
            gy0 = row * L::MH;
        }
#pragma unroll
        for (int sub = 0; sub < L::SY; sub++) {
            const int ry = cy * L::SY + sub;
            const uint32_t gy = gy0 + ry;
            if (!STATIC && gy >= p.height) continue;
            const uint32_t yq = *reinterpret_cast<const uint32_t*>(yplane + ry * T::YW + qc * 4);
            uint32_t px[4];
            if (MODE == 444) {
                px[0] = bgra444<0>(yq, cb4, cr4, k444);
                px[1] = bgra444<1>(yq, cb4, cr4, k444);
                px[2] = bgra444<2>(yq, cb4, cr4, k444);
                px[3] = bgra444<3>(yq, cb4, cr4, k444);
            } else if (FLAGS & kCscI32) {
                px[0] = bgra16(y16<0>(yq), ct32[0]);
                px[1] = bgra16(y16<1>(yq), ct32[0]);
                px[2] = bgra16(y16<2>(yq), ct32[1]);
                px[3] = bgra16(y16<3>(yq), ct32[1]);
            } else {
                bgra_pair(__builtin_amdgcn_perm(0u, yq, 0x0c010c00u), ct[0], px[0], px[1]);  // {Y0, Y1}
                bgra_pair(__builtin_amdgcn_perm(0u, yq, 0x0c030c02u), ct[1], px[2], px[3]);  // {Y2, Y3}
            }
            if constexpr (STATIC) {
                // coded MCUs past the displayed width (1080p: none; 200 px: 208 coded) are not
                // written: with width % 4 == 0, gx < width means the whole quad is inside
                const bool ok = qvalid && gy < p.height && gx < p.width;
                const uint32_t off = (gy * p.out_pitch + gx) * 4u;
                constexpr int aux = (FLAGS & kNtStore) ? 2 : 0;  // nt
                const u32x4 v4 = {px[0], px[1], px[2], px[3]};
                __builtin_amdgcn_raw_buffer_store_b128(v4, orsrc, ok ? off : oob, 0, aux);
                continue;
            }
            uint32_t* dst = outf + (size_t)gy * p.out_pitch + gx;
            if (p.aligned16 && gx + 4 <= p.width) {
                const u32x4 v4 = {px[0], px[1], px[2], px[3]};
                store16(reinterpret_cast<u32x4*>(dst), v4, (FLAGS & kNtStore) != 0);
            } else {
#pragma unroll
                for (int i = 0; i < 4; i++)
                    if (gx + i < p.width) dst[i] = px[i];
            }
        }
    }
}

// Waves per SIMD that the LDS of one workgroup allows (160 KiB per CU, at most 8 per SIMD),
// given to the compiler as the register budget (__launch_bounds__' second argument = minimum
// waves per SIMD).  Without it the scheduler may trade occupancy for ILP on its own: with the
// two IDCT forms in one function it chose 109-124 VGPRs for the batch kernel (4 waves per
// SIMD) where LDS allows 6.
constexpr int lds_waves(int lds_bytes, int threads) {
    const int wg = (160 * 1024) / lds_bytes;
    const int w = wg * threads / 256;
    return w < 1 ? 1 : w > 8 ? 8 : w;
}
template <int MODE, int TW, int THREADS, int FLAGS>
constexpr int kBatchLds = Tile<MODE, TW, THREADS>::LDS_BYTES;
template <int MODE, int TW, int THREADS, int FLAGS>
constexpr int kGopStateBytes = (FLAGS & kGopState8) ? Tile<MODE, TW, THREADS>::NSLOT * 64 : Tile<MODE, TW, THREADS>::COEF_BYTES;
template <int MODE, int TW, int THREADS, int FLAGS>
constexpr int kGopLds = kGopStateBytes<MODE, TW, THREADS, FLAGS> + Tile<MODE, TW, THREADS>::PLANE_BYTES + ((FLAGS & kGopLdsQt) ? 256 : 0);


// Stream-kernel job of this workgroup: (tile tx, segment sy).  p.gop_order == kGopOrderEighths (1-D
// grid of 8 * ceil(T / 8) * nseg): workgroups b and b + 8 share an XCD, and XCD b % 8
// walks the (b % 8)-th contiguous eighth of the tiles of segment 0, then of segment 1, ... -- so
// each XCD keeps to one band of the frame.  p.gop_order == kFgroupXcd: the
// (segment, tile) jobs in segment-major order are cut into eight contiguous ranges, workgroup b
// taking job (b % 8) * per + b / 8 -- workgroups b and b + 8 share an XCD, so each XCD walks
// whole segments tile after tile (the batch kernel's XCD-contiguous order); false = no job.
__device__ __forceinline__ bool gop_job(const DecodeParams& p, uint32_t& tx, uint32_t& sy) {
    if (p.gop_order == kGopOrderEighths) {  // XCD x takes the x-th contiguous eighth of every segment's tiles
        const uint32_t T = p.tiles_per_frame, E = (T + 7) / 8, i = blockIdx.x / 8;
        sy = i / E;
        tx = (blockIdx.x % 8) * E + i % E;
        return sy < p.nseg && tx < T;
    }
    if (p.gop_order != kFgroupXcd) {
        tx = blockIdx.x;
        sy = blockIdx.y;
        return true;
    }
    const uint32_t jobs = p.tiles_per_frame * p.nseg, per = (jobs + 7) / 8;
    const uint32_t j = (blockIdx.x % 8) * per + blockIdx.x / 8;
    sy = j / p.tiles_per_frame;
    tx = j - sy * p.tiles_per_frame;
    return j < jobs;
}

}  // namespace mj423
