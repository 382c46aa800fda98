// mj423_fused.hip -- the whole-GPU .mpg decode in one pass over the pixels (mj423_mpg_decode_gpu):
// entropy decode of every block, P-frame accumulation, dequantization, 8x8 IDCT and YCbCr->BGRA
// fused, from the frames' bitstream bytes in HBM and a block index.
//
// The many-lanes front end (mj423_entropy.hip) finds where every block of every (frame, plane)
// bitstream starts: its index pass leaves each block's coded length in bits (2 B) and, per tile of
// kFuseTw blocks, the tile's first bit and its DC predictor (8 B).  Here one workgroup walks one
// tile of kFuseTw MCUs through the frames of a GOP segment, like decode_gop_kernel<444>, but
// instead of staging dense int16 planes it decodes the tile's blocks itself -- wave w holds plane
// w, lane c block c: a wave prefix sum of the lengths gives every lane its block's first bit, a
// second one (I-frames) turns the DC differences into DC values -- straight into the LDS slots
// that hold the tile's accumulated coefficients.  No dense plane is written or read: per frame
// the kernel reads the bitstream (~0.3 MB at 1080p) and the index (~0.2 MB) and writes the BGRA
// frame (8.3 MB), where the two-pass form wrote and re-read 12.4 MB of int16 planes.
//
// The slots hold DEQUANTIZED coefficients, column-major: the block decoder multiplies each coefficient
// by its quantizer as it stores it (P-frames: adds e * q to the slot mod 2^16 -- (sum e) * q == sum (e * q)
// mod 2^16, SURVEY §8 A5, so the accumulated state equals the reference's dequantized DCAC plane), and
// row c of a slot is column c of the block with its rows in the order 0,4,2,6,1,3,5,7: the four int16
// pairs (x0,x4), (x2,x6), (x1,x3), (x5,x7) the column pass's dot products take.  So the transform reads
// its operands straight from LDS -- no dequantization and no repacking in it (fused_tile_idct).
//
// Reference: lossless_decode.c:82-134 (symbols, I DC prediction, P accumulation 90-92 and 121-122),
// idct.c:22-181, ycbcr_to_rgb.c:26-49, the frame loop mjpeg423_decoder.c:109-124.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "mj423_bits.hpp"
#include "mj423_entropy.h"
#include "mj423_tile.hpp"

// MJ423_FUSED_ABLATE=1|2|3 (measurement builds only, tools/build_variant.sh): leave out the IDCT, the
// CSC or the block decode, to time the rest (the output is then wrong)
#ifndef MJ423_FUSED_ABLATE
#define MJ423_FUSED_ABLATE 0
#endif


namespace mj423 {
namespace {

using FT = Tile<444, (int)kFuseTw, 256>;
constexpr int kFusedLds = FT::COEF_BYTES + FT::PLANE_BYTES + 512;  // slots | planes | symbol tables
// decode_gop_kernel<444>'s CSC; the IDCT is fused_tile_idct below: the int16-workspace transform behind the
// exact width test -- this kernel is bound by VALU work, not by memory (MJ423_FUSED_IDCT32=1: the int32 form,
// A/B)
constexpr int kFusedFlags = kNtStore;
constexpr int kFusedFlags32 = kNtStore | kIdctI32;

// Position of row r inside a column row of a slot: rows 0,4,2,6,1,3,5,7 (the pass-1 operand pairs).
__device__ __forceinline__ uint32_t col_pos(uint32_t r) { return (0x73615240u >> (4 * r)) & 7u; }

// Inclusive prefix sum over the wave (64 lanes) by DPP: row_shr 1, 2, 4, 8 inside each row of 16 lanes
// (bound_ctrl: lanes without a source add 0), then row_bcast:15 and row_bcast:31 carry the rows' totals.
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);  // row_shr:1
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);  // row_shr:2
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);  // row_shr:4
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);  // row_shr:8
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
    v += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
    return v;
}

// (uint16)(a) * (uint16)(q) + c: the dequantized coefficient (int16)(e * q) (lossless_decode.c:95,125)
// added to c mod 2^16 -- v_mad_u32_u16, the low 16 bits of each operand.
__device__ __forceinline__ uint32_t mad_u16(uint32_t a, uint32_t q, uint32_t c) {
    uint32_t d;
    asm("v_mad_u32_u16 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(q), "v"(c));
    return d;
}

// Block `col` of plane `plane` in the tile, frame f, in three steps so that the loads of frame
// f + 1 can be in flight while frame f is transformed (PRE):
//   fetch  : the index entries (the tile's DC predictor; this block's first bit and the next one's)
//   locate : the block's first three dwords
//   decode : the block into this lane's LDS slot (rows XOR-swizzled like every staged block,
//            coef_off); I-frames replace the slot's contents, P-frames add their deltas mod 2^16.
// Wave-uniform: plane, f.  Lanes without a block (past a short last tile) take part in the scans
// with zeros.
struct BlockAt {
    uint32_t len;       // this block's coded length in bits (0: no block; at most 65535)
    uint32_t dc0;       // the tile's DC predictor (I-frames)
    uint64_t bit;       // (fetch) this block's first bit, absolute in the uploaded bytes
    const uint32_t* dw; // (locate) the dword holding that bit (clamped into the upload)
    uint32_t rdmax;     // (locate) dwords readable from dw
    uint32_t v0, v1;    // (locate) the two dwords holding the block's start, as loaded
    uint32_t v2;        // (locate) the dword after them (the reader's first refill)
};

__device__ __forceinline__ void fetch_block(const FusedParams& fp, uint32_t f, uint32_t plane, uint32_t tx,
                                            uint32_t col, bool has, BlockAt& b) {
    const uint32_t fp3 = __builtin_amdgcn_readfirstlane(f * 3 + plane);  // (wave-uniform: scalar loads)
    MJ423_BOUND(fp3, fp.lim.tasks, "tasks (fused)");
    MJ423_BOUND((uint64_t)fp3 * fp.tiles_pp + tx, fp.lim.tiles, "tiles (fused)");
    if (has) MJ423_BOUND((uint64_t)fp3 * (fp.nblk + 1) + tx * kFuseTw + col + 1, fp.lim.bpos, "bpos (fused)");
    const uint64_t byte_off = fp.tasks[fp3].byte_off;
    b.dc0 = fp.tiles[(uint64_t)fp3 * fp.tiles_pp + tx].y;
    const uint32_t* bp = fp.bpos + (uint64_t)fp3 * (fp.nblk + 1) + tx * kFuseTw + col;
    const uint32_t p0 = has ? bp[0] : 0u, p1 = has ? bp[1] : 0u;
    b.bit = byte_off * 8 + p0;
    // The length bounds the block's AC loop.  Capped: a block can run on past index 63 with ZRL
    // symbols indefinitely, but only its first ~67 symbols (<= 23 bits each) can place a coefficient
    // (each advances the index, a ZRL by 16), so a cap far above that changes nothing; the next
    // block's position comes from the index, not from this one's length.  (p1 < p0 only in a plane
    // whose index walk failed: its status fails the call.)
    b.len = p1 < p0 ? 0u : min(p1 - p0, 65535u);
}

__device__ __forceinline__ void locate_block(const FusedParams& fp, BlockAt& b) {
    const uint64_t dw_max = (fp.bytes_len + 60) / 4, rd = min(b.bit >> 5, dw_max);
    MJ423_BOUND(dw_max, fp.lim.bytes_dw, "bytes (fused)");
    b.dw = reinterpret_cast<const uint32_t*>(fp.bytes) + rd;
    b.rdmax = (uint32_t)min<uint64_t>(dw_max - rd, 0xffffffffu);
    b.v0 = b.dw[0];
    b.v1 = b.dw[min(1u, b.rdmax)];
    b.v2 = b.dw[min(2u, b.rdmax)];
}

// tab: the wave's symbol table (Y or chroma, in LDS): entry k = (byte offset of zig-zag position k in a
// slot, before the slot's swizzle) << 16 | its quantizer.  swz16: this slot's row swizzle, (slot & 7) << 4.
// The reader takes the block's bits as they are: a block the index placed inside its stream never
// consumes a bit past the stream's end (a stream whose blocks would fails the whole call, status 1), so
// no stream-end mask is applied.  A refill's dword is loaded one refill ahead.
// Returns whether the slot may have changed: always for an I-frame; for a P-frame only if the block
// carries a non-zero DC difference or any coefficient (an EOB-only block leaves its state, and so its
// pixels, as they were -- the common case of static content).
__device__ __forceinline__ bool decode_block(const BlockAt& b, bool has, bool P, uint8_t* slot, uint32_t swz16,
                                             const uint32_t* tab) {
    const uint32_t sh = (uint32_t)b.bit & 31u;
    uint64_t win = (((uint64_t)__builtin_bswap32(b.v0) << 32) | __builtin_bswap32(b.v1)) << sh;
    uint32_t n = 64 - sh, nxt = b.v2, rd = 3;  // rd: the next dword to load, from b.dw
    // DC: SIZE(4) + VLI, >= 33 bits in the window (lossless_decode.c:86-96)
    const uint32_t hi0 = (uint32_t)(win >> 32), dsz = hi0 >> 28;
    const uint32_t dv = __builtin_amdgcn_ubfe(hi0, 28u - dsz, dsz);
    win <<= 4 + dsz;
    n -= 4 + dsz;
    const int32_t diff = has ? huff_extend(dv, dsz) : 0;
    // I: DC prediction inside the plane from the tile's predictor
    const uint32_t dcv = P ? (uint32_t)diff : b.dc0 + wave_incl_sum((uint32_t)diff);
    if (!P) {
#pragma unroll
        for (int k = 0; k < 8; k++) reinterpret_cast<uint4*>(slot)[k] = make_uint4(0u, 0u, 0u, 0u);
    }
    if (!has) return false;
    bool changed = !P || diff != 0;
    uint16_t* d0 = reinterpret_cast<uint16_t*>(slot + swz16);  // column 0, row 0
    *d0 = (uint16_t)mad_u16(dcv, tab[0], P ? (uint32_t)*d0 : 0u);
    // AC: RUN(4) SIZE(4) + VLI; SIZE 0: RUN 15 = ZRL, else EOB; a coefficient at index >= 63 ends
    // the block (lossless_decode.c:100-129).  A valid block ends exactly at its indexed length;
    // the length also bounds the walk of a damaged one.  One symbol per iteration from the window's top
    // 32 bits (>= 33 valid after the refill; a symbol takes <= 23).
    uint32_t idx = 1, used = 4 + dsz;
    while (used < b.len) {
        if (n <= 32) {
            win |= (uint64_t)__builtin_bswap32(nxt) << (32 - n);
            n += 32;
            nxt = b.dw[min(rd, b.rdmax)];
            rd++;
        }
        const uint32_t hi = (uint32_t)(win >> 32), run = hi >> 28, size = __builtin_amdgcn_ubfe(hi, 24u, 4u);
        const uint32_t vli = __builtin_amdgcn_ubfe(hi, 24u - size, size);  // (size 0: 0)
        const uint32_t tot = 8 + size;
        win <<= tot;
        n -= tot;
        used += tot;
        const bool zero = size == 0;
        if (zero && run != 15) break;  // EOB
        const uint32_t ni = min(idx + (zero ? 16u : run), 64u);  // ZRL: 16 zeros; else the coefficient's index
        if (!zero && ni <= 63) {
            const uint32_t e = tab[ni];
            uint16_t* a = reinterpret_cast<uint16_t*>(slot + ((e >> 16) ^ swz16));
            *a = (uint16_t)mad_u16((uint32_t)huff_extend(vli, size), e, P ? (uint32_t)*a : 0u);
            changed = true;
        }
        if (!zero && ni >= 63) break;
        idx = zero ? ni : ni + 1;
    }
    return changed;
}

// The 8x8 IDCT of the lane's block from its column-major dequantized slot (w[c] = the four operand pairs
// of column c; idct.c:39-109 pass 1, :115-180 pass 2): mj423_idct.hpp's int16-workspace transform
// (idct8x8_w16) and int32 transform (idct8x8) with their pass-1 operands read directly.
__device__ __forceinline__ void idct_cols_w16(const uint32_t (&w)[8][4], uint32_t (&out)[8][2]) {
    uint32_t ws[8][4];  // row r: {ws[r][0], ws[r][4]}, {ws[r][2], ws[r][6]}, {ws[r][1], ws[r][3]}, {ws[r][5], ws[r][7]}
    const uint32_t rnd = 1u << 10;
    auto column = [&](int c, uint32_t y[8]) {  // hi16(y[n]) = DESCALE(., 11) of row n (idct8x8_w16)
        const Sums8 t = sums8(w[c][0], w[c][1], w[c][2], w[c][3], rnd);
        y[0] = (t.s0 + t.o1) << 5;
        y[7] = (t.s0 - t.o1) << 5;
        y[1] = (t.s1 + t.o3) << 5;
        y[6] = (t.s1 - t.o3) << 5;
        y[2] = (t.s2 + t.o5) << 5;
        y[5] = (t.s2 - t.o5) << 5;
        y[3] = (t.s3 + t.o7) << 5;
        y[4] = (t.s3 - t.o7) << 5;
    };
    constexpr int kPairCols[4][2] = {{0, 4}, {2, 6}, {1, 3}, {5, 7}};
#pragma unroll
    for (int q = 0; q < 4; q++) {
        uint32_t ya[8], yb[8];
        column(kPairCols[q][0], ya);
        column(kPairCols[q][1], yb);
#pragma unroll
        for (int r = 0; r < 8; r++) ws[r][q] = pair_hi(ya[r], yb[r]);
    }
    const uint32_t rnd2 = 1u << 17;  // DESCALE(., 18) rounding
#pragma unroll
    for (int r = 0; r < 8; r++) {  // pass 2: rows, NORMALIZE to [0,255] (idct.c:115-180, :20)
        const Sums8 t = sums8(ws[r][0], ws[r][1], ws[r][2], ws[r][3], rnd2);
        const int32_t y0 = (int32_t)(t.s0 + t.o1), y7 = (int32_t)(t.s0 - t.o1);
        const int32_t y1 = (int32_t)(t.s1 + t.o3), y6 = (int32_t)(t.s1 - t.o3);
        const int32_t y2 = (int32_t)(t.s2 + t.o5), y5 = (int32_t)(t.s2 - t.o5);
        const int32_t y3 = (int32_t)(t.s3 + t.o7), y4 = (int32_t)(t.s3 - t.o7);
        out[r][0] = ashr_pk_u8_hi<18>(ashr_pk_u8<18>(y0, y1), y2, y3);
        out[r][1] = ashr_pk_u8_hi<18>(ashr_pk_u8<18>(y4, y5), y6, y7);
    }
}
__device__ __forceinline__ void idct_cols_i32(const uint32_t (&w)[8][4], uint32_t (&out)[8][2]) {
    int32_t ws[8][8];  // ws[n][c], scaled by 2^PASS1_BITS
    const uint32_t rnd = 1u << 10;
#pragma unroll
    for (int c = 0; c < 8; c++) {
        int32_t y[8];
        pass1_column(w[c][0], w[c][1], w[c][2], w[c][3], rnd, y);
#pragma unroll
        for (int n = 0; n < 8; n++) ws[n][c] = y[n];
    }
#pragma unroll
    for (int r = 0; r < 8; r++) {
        int32_t y[8];
        butterfly8<2>(ws[r], y);
        out[r][0] = ashr_pk_u8_hi<18>(ashr_pk_u8<18>(y[0], y[1]), y[2], y[3]);
        out[r][1] = ashr_pk_u8_hi<18>(ashr_pk_u8<18>(y[4], y[5]), y[6], y[7]);
    }
}

// IDCT of one tile: lane s transforms slot s into the uint8 plane tiles (decode_tile_idct's layout).  The
// int16-workspace form unless a block of the wave fails the exact width test (mj423_idct.hpp kWs16Energy;
// per column: ||column||^2 <= 8 388 183 bounds every workspace value of that column inside int16), each
// form a complete pass of its own that loads its own registers (a decision on a block already in registers
// cost ~25-30 VGPRs, decode_tile_idct).  Wave 3 holds no block.
// `redo`: this lane's block changed since the wave last transformed it.  A wave none of whose blocks
// changed keeps last frame's plane tiles (the IDCT of the same coefficients), so it skips the transform.
template <int FLAGS>
__device__ __forceinline__ void fused_tile_idct(const TileCoord& c, const uint8_t* coef, uint8_t* planes, int tid,
                                                bool redo) {
    const int s = tid;
    if (__builtin_amdgcn_readfirstlane(s) >= FT::NSLOT || __builtin_amdgcn_ballot_w64(redo) == 0) return;
    const int run = FT::slot_run(s);
    const int col = s - (run <= 1 ? 0 : run == 2 ? FT::run_first_slot(2) : FT::run_first_slot(3));
    const bool active = col < c.run_len(run);
    const uint8_t* base = coef + s * 128;
    const int swz = s & 7;
    auto load = [&](uint32_t (&w)[8][4]) {
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint4 v = *reinterpret_cast<const uint4*>(base + ((k ^ swz) << 4));
            w[k][0] = v.x;
            w[k][1] = v.y;
            w[k][2] = v.z;
            w[k][3] = v.w;
        }
    };
    uint8_t* dstp = run < 2 ? planes + col * 8 : planes + (run == 2 ? 8 * FT::YW : 8 * FT::YW + FT::CH * FT::CW) + col * 8;
    constexpr int pitch = FT::YW;  // = FT::CW at 4:4:4
    auto pass = [&](auto form) {
        uint32_t w[8][4];
        load(w);
        if (!active) return;
        uint32_t o[8][2];
        if constexpr (decltype(form)::value == 1)
            idct_cols_i32(w, o);
        else
            idct_cols_w16(w, o);
#pragma unroll
        for (int r = 0; r < 8; r++) *reinterpret_cast<uint2*>(dstp + r * pitch) = make_uint2(o[r][0], o[r][1]);
    };
    using F16 = std::integral_constant<int, 0>;
    using F32 = std::integral_constant<int, 1>;
    if constexpr ((FLAGS & kIdctI32) != 0) return pass(F32{});
    bool wide = false;
    if (active) {
        int32_t m = 0;
#pragma unroll
        for (int k = 0; k < 8; k++) {
            const uint4 v = *reinterpret_cast<const uint4*>(base + ((k ^ swz) << 4));
            m = max(m, sdot2_sat(v.w, sdot2_sat(v.z, sdot2_sat(v.y, sdot2_sat(v.x, 0)))));
        }
        wide = m > kWs16Energy;
    }
    if (__builtin_amdgcn_ballot_w64(wide) == 0)
        pass(F16{});
    else
        pass(F32{});
}

// CSC of one tile with the fixed-store-count form (decode_tile_csc<444>'s arithmetic and stores, kStaticStores):
// lane t converts quad (t & 127) of tile rows (t >> 7) + 2 it, it = 0..3.  Where each quad lands in a frame --
// the raster position of its MCU, or past the buffer's range when it lies outside the coded region -- is
// the same in every frame of the segment, so it is worked out once per workgroup (csc_plan), not per frame.
constexpr int kCscIters = (FT::YW / 4) * FT::CH / 256;  // 4
static_assert(kCscIters * 256 == (FT::YW / 4) * FT::CH && FT::YW / 4 == 128, "fused CSC: 128 quads per tile row");
__device__ __forceinline__ void csc_plan(const DecodeParams& p, const TileCoord& c0, int tid, uint32_t (&off)[kCscIters],
                                         uint32_t& nrec) {
    nrec = (uint32_t)((uint64_t)p.height * p.out_pitch * 4u);
    const uint32_t qc = (uint32_t)tid & 127u;  // quad in the tile row; MCU qc / 2 of the tile
    const uint32_t m = c0.mx0 + qc / 2;       // raster MCU index
    uint32_t row = __umulhi(m, p.cols_magic), col = m - row * p.mcu_cols;
    if (col >= p.mcu_cols) {
        col -= p.mcu_cols;
        row++;
    }
    const uint32_t gx = col * 8 + (qc % 2) * 4;
    const bool qvalid = (int)qc < c0.tw * 2;
#pragma unroll
    for (int it = 0; it < kCscIters; it++) {
        const uint32_t gy = row * 8 + 2 * it + ((uint32_t)tid >> 7);
        // with width % 4 == 0 (kStaticStores' condition), gx < width means the whole quad is inside
        off[it] = qvalid && gy < p.height && gx < p.width ? (gy * p.out_pitch + gx) * 4u : nrec;
    }
}
template <int FLAGS>
__device__ __forceinline__ void fused_tile_csc(const DecodeParams& p, uint32_t f, const uint8_t* planes, int tid,
                                               const uint32_t (&off)[kCscIters], uint32_t nrec) {
    const CscConst444 k444 = csc444_consts();
    uint32_t* outf = p.out + (size_t)f * p.out_fstride;
    const __amdgpu_buffer_rsrc_t orsrc = __builtin_amdgcn_make_buffer_rsrc(outf, 0, (int)nrec, 0x00020000);
    constexpr int aux = (FLAGS & kNtStore) ? 2 : 0;  // nt
    const uint32_t lo = ((uint32_t)tid >> 7) * FT::YW + ((uint32_t)tid & 127u) * 4;
#pragma unroll
    for (int it = 0; it < kCscIters; it++) {
        const uint32_t a = lo + 2 * it * FT::YW;  // tile row (tid >> 7) + 2 it, quad (tid & 127)
        const uint32_t yq = *reinterpret_cast<const uint32_t*>(planes + a);
        const uint32_t cb4 = *reinterpret_cast<const uint32_t*>(planes + 8 * FT::YW + a);
        const uint32_t cr4 = *reinterpret_cast<const uint32_t*>(planes + 8 * FT::YW + FT::CH * FT::CW + a);
        const u32x4 v4 = {bgra444<0>(yq, cb4, cr4, k444), bgra444<1>(yq, cb4, cr4, k444), bgra444<2>(yq, cb4, cr4, k444),
                          bgra444<3>(yq, cb4, cr4, k444)};
        __builtin_amdgcn_raw_buffer_store_b128(v4, orsrc, off[it], 0, aux);
    }
}

// PRE: frame f + 1's index entries are loaded before frame f's IDCT and its first dwords before
// frame f's CSC, so the dependent loads of a frame's decode are in flight during the previous
// frame's transform (MJ423_FUSED_PREFETCH=0 turns it off, A/B).
template <int FLAGS, bool PRE>
__global__ void __launch_bounds__(256, (lds_waves(kFusedLds, 256))) mpg_fused_kernel(const FusedParams fp) {
    static_assert(production_flags<FLAGS>(), "mpg_fused_kernel: production flags only");
    const DecodeParams& p = fp.d;
    __shared__ __attribute__((aligned(16))) uint8_t lds[kFusedLds];
    uint8_t* state = lds;                  // the tile's accumulated dequantized coefficients, one column-major slot per block
    uint8_t* planes = lds + FT::COEF_BYTES;  // uint8 plane tiles, per frame
    uint32_t* tabs = reinterpret_cast<uint32_t*>(lds + FT::COEF_BYTES + FT::PLANE_BYTES);  // [Y | chroma][zig-zag k]
    const int tid = threadIdx.x;
    if (tid < 128) {  // entry = slot byte offset of natural position kZz[k] << 16 | its quantizer (p.qt_dev, natural order)
        const uint32_t n = kZz[tid & 63], cls = (uint32_t)tid >> 6;
        const uint32_t q = reinterpret_cast<const uint16_t*>(p.qt_dev)[cls * 64 + n];
        tabs[tid] = ((((n & 7u) << 4) | (col_pos(n >> 3) << 1)) << 16) | q;
    }
    uint32_t tx, sy;
    if (!gop_job(p, tx, sy)) return;  // (whole workgroup, before any barrier)
    // (the segment table is the host's; clamped to the launch's frames, so no table can move an access outside them)
    MJ423_BOUND(sy + 1, fp.lim.seg_start, "seg_start (fused)");
    const uint32_t nf = p.ntiles / p.tiles_per_frame, f1 = min(p.seg_start[sy + 1], nf), f0 = min(p.seg_start[sy], f1);
    if (f1 > f0) MJ423_BOUND(f1 - 1, fp.lim.ftype, "ftype (fused)");
    const TileCoord cs = tile_coord<444>(p, tx);  // frame-0 coordinates (state offsets)
    auto st_off = [&](int k) -> int64_t {         // staging chunk k of this lane in the state buffers
        const int run = FT::chunk_run(k);
        const int c = FT::SLOTS_PER_CHUNK * k + (tid >> 3) - FT::run_first_slot(run);
        const int64_t o = cs.run_off(run) + (c < cs.run_len(run) ? c : 0) * 64 + (tid & 7) * 8;
        return run < 2 ? o : run == 2 ? o - p.cb_off + p.st_cb_off : o - p.cr_off + p.st_cr_off;
    };
    if (f0 < f1 && p.ftype[f0] != 0) {  // the segment continues a GOP: seed the slots from p.state
        u32x4 v[FT::CHUNKS];
#ifdef MJ423_BOUNDS_CHECK
        if (!p.state) {
            printf("mj423 bound: fused: a P-frame segment start without state (segment %u, frame %u)\n", sy, f0);
            __builtin_trap();
        }
#endif
#pragma unroll
        for (int k = 0; k < FT::CHUNKS; k++) {
            MJ423_BOUND(st_off(k) + 7, fp.lim.state, "state (fused seed)");
            v[k] = *reinterpret_cast<const u32x4*>(p.state + st_off(k));
        }
        // chunk k of this lane: natural row r of slot sl; the host's seek seed is quantized (dequantized
        // here), a previous window's end state already dequantized
        const uint32_t r = (uint32_t)tid & 7u;
#pragma unroll
        for (int k = 0; k < FT::CHUNKS; k++) {
            const int sl = FT::SLOTS_PER_CHUNK * k + (tid >> 3);
            u32x4 x = v[k];
            if (fp.state_quantized) {
                const uint32_t* q = p.qt_dev + 32 * (FT::chunk_run(k) >= 2 ? 1 : 0) + 4 * r;
                x = (u32x4){dequant_pair(x.x, q[0]), dequant_pair(x.y, q[1]), dequant_pair(x.z, q[2]), dequant_pair(x.w, q[3])};
            }
            uint8_t* b = state + sl * 128 + col_pos(r) * 2;
            const uint32_t xs[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int cc = 0; cc < 8; cc++)
                *reinterpret_cast<uint16_t*>(b + ((cc ^ (sl & 7)) << 4)) = (uint16_t)(xs[cc >> 1] >> (16 * (cc & 1)));
        }
    }
    __syncthreads();  // seed, tables: before the first frame's decode
    // Wave w < 3 decodes and transforms plane w of the tile (slots 64 w .. 64 w + 63, lane = slot); wave 3
    // only converts colour.  (Rotating these roles with the workgroup, in case every CU's fourth SIMD held
    // only idle waves, measured 0.8 % slower: profiles/r06/fused/file_ab_rotate.log.)
    const int vt = tid;  // this lane's slot
    const uint32_t plane = (uint32_t)tid >> 6, col = (uint32_t)tid & 63u;
    const bool has = plane < 3 && (int)col < cs.tw;
    const bool dec = __builtin_amdgcn_readfirstlane(plane) < 3;  // waves 0-2
    constexpr bool STATIC = (FLAGS & kStaticStores) != 0;
    uint32_t csc_off[kCscIters], csc_nrec = 0;
    if (STATIC) csc_plan(p, cs, tid, csc_off, csc_nrec);
    BlockAt b;
    if (PRE && dec && f0 < f1) {
        fetch_block(fp, f0, plane, tx, col, has, b);
        locate_block(fp, b);
    }
    for (uint32_t f = f0; f < f1; f++) {
        const bool P = __builtin_amdgcn_readfirstlane(p.ftype[f]) != 0;
        bool redo = f == f0;  // (the plane tiles hold nothing yet at the segment's first frame)
        if (dec) {
            if (!PRE) {
                fetch_block(fp, f, plane, tx, col, has, b);
                locate_block(fp, b);
            }
#if MJ423_FUSED_ABLATE != 3
            redo |= decode_block(b, has, P, state + vt * 128, ((uint32_t)vt & 7u) << 4, tabs + (plane == 0 ? 0 : 64));
#else
            redo = true;
#endif
        }
        __syncthreads();
        const bool more = f + 1 < f1;
        if (PRE && dec && more) fetch_block(fp, f + 1, plane, tx, col, has, b);
        const TileCoord c = tile_coord<444>(p, f * p.tiles_per_frame + tx);
        MJ423_BOUND((uint64_t)f * p.out_fstride + (uint64_t)p.height * p.out_pitch - 1, fp.lim.out, "out (fused)");
#if MJ423_FUSED_ABLATE != 1
        fused_tile_idct<FLAGS>(c, state, planes, vt, redo);
#endif
        __syncthreads();
        if (PRE && dec && more) locate_block(fp, b);
#if MJ423_FUSED_ABLATE != 2
        if constexpr (STATIC)
            fused_tile_csc<FLAGS>(p, f, planes, tid, csc_off, csc_nrec);
        else
            decode_tile_csc<444, (int)kFuseTw, 256, FLAGS>(p, c, planes, tid);
#endif
        // no barrier: the next frame's decode writes only the slots (read by this frame's IDCT before
        // the barrier above), and its barrier orders these plane reads before the next IDCT
    }
    if (p.state_out && sy + 1 == p.nseg) {  // end state, for the next window of the same GOP
        __syncthreads();
#pragma unroll
        for (int k = 0; k < FT::CHUNKS; k++) {
            const int run = FT::chunk_run(k);
            const int c = FT::SLOTS_PER_CHUNK * k + (tid >> 3) - FT::run_first_slot(run);
            if (c < cs.run_len(run)) MJ423_BOUND(st_off(k) + 7, fp.lim.state, "state_out (fused)");
            if (c < cs.run_len(run)) {  // natural row r of slot sl, dequantized
                const int sl = FT::SLOTS_PER_CHUNK * k + (tid >> 3);
                const uint8_t* b = state + sl * 128 + col_pos((uint32_t)tid & 7u) * 2;
                uint32_t xs[4];
#pragma unroll
                for (int h = 0; h < 4; h++)
                    xs[h] = (uint32_t)*reinterpret_cast<const uint16_t*>(b + (((2 * h) ^ (sl & 7)) << 4)) |
                            ((uint32_t)*reinterpret_cast<const uint16_t*>(b + (((2 * h + 1) ^ (sl & 7)) << 4)) << 16);
                *reinterpret_cast<u32x4*>(p.state_out + st_off(k)) = (u32x4){xs[0], xs[1], xs[2], xs[3]};
            }
        }
    }
}

}  // namespace
}  // namespace mj423

extern "C" int mj423_gop_static_stores(const mj423::DecodeParams* p);

extern "C" hipError_t mj423_launch_mpg_fused(const mj423::FusedParams* p, hipStream_t stream) {
    const uint32_t tiles = p->d.tiles_per_frame, nseg = p->d.nseg;
    if (tiles == 0 || nseg == 0) return hipSuccess;
    if (nseg > 65535 || p->d.tw != mj423::kFuseTw) return hipErrorInvalidValue;
    const dim3 grid(tiles, nseg);
    using namespace mj423;
    const bool pre = !(getenv("MJ423_FUSED_PREFETCH") && atoi(getenv("MJ423_FUSED_PREFETCH")) == 0);
    const bool i32 = getenv("MJ423_FUSED_IDCT32") && atoi(getenv("MJ423_FUSED_IDCT32")) == 1;
    const bool st = mj423_gop_static_stores(&p->d) != 0;
    if (i32) {
        if (st)
            hipLaunchKernelGGL((mpg_fused_kernel<kFusedFlags32 | kStaticStores, true>), grid, dim3(256), 0, stream, *p);
        else
            hipLaunchKernelGGL((mpg_fused_kernel<kFusedFlags32, true>), grid, dim3(256), 0, stream, *p);
    } else if (st && pre) {
        hipLaunchKernelGGL((mpg_fused_kernel<kFusedFlags | kStaticStores, true>), grid, dim3(256), 0, stream, *p);
    } else if (st) {
        hipLaunchKernelGGL((mpg_fused_kernel<kFusedFlags | kStaticStores, false>), grid, dim3(256), 0, stream, *p);
    } else if (pre) {
        hipLaunchKernelGGL((mpg_fused_kernel<kFusedFlags, true>), grid, dim3(256), 0, stream, *p);
    } else {
        hipLaunchKernelGGL((mpg_fused_kernel<kFusedFlags, false>), grid, dim3(256), 0, stream, *p);
    }
    return hipGetLastError();
}
