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
constexpr int kFusedLds = FT::COEF_BYTES + FT::PLANE_BYTES + 256 + 64;  // slots | planes | quant tables | zig-zag
// decode_gop_kernel<444>'s forms, except the IDCT: the int16-workspace transform behind the exact
// width test (the batch kernel's, mj423_idct.hpp) -- this kernel is bound by VALU work, not by
// memory (MJ423_FUSED_IDCT32=1: the int32 form, A/B)
constexpr int kFusedFlags = kNtStore | kGopLdsQt;
constexpr int kFusedFlags32 = kNtStore | kGopLdsQt | kIdctI32;

__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t v) {
    const uint32_t lane = threadIdx.x & 63;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(v, o);
        if (lane >= (uint32_t)o) v += t;
    }
    return v;
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
    uint64_t byte_off;  // the plane bitstream's first byte
    uint32_t nbytes;
    uint32_t len;       // this block's coded length in bits (0: no block; at most 65535)
    uint2 te;           // the tile's {first bit, DC before it}
    uint32_t pos;       // this block's first bit in the plane's bitstream
    uint32_t v0, v1;    // (locate) the two dwords holding it, as loaded
    uint32_t v2;        // (locate) the dword after them (the reader's first refill)
};

__device__ __forceinline__ void fetch_block(const FusedParams& fp, uint32_t f, uint32_t plane, uint32_t tx,
                                            uint32_t col, bool has, BlockAt& b) {
    const uint32_t fp3 = f * 3 + plane;
    MJ423_BOUND(fp3, fp.lim.tasks, "tasks (fused)");
    MJ423_BOUND((uint64_t)fp3 * fp.tiles_pp + tx, fp.lim.tiles, "tiles (fused)");
    if (has) MJ423_BOUND((uint64_t)fp3 * (fp.nblk + 1) + tx * kFuseTw + col + 1, fp.lim.bpos, "bpos (fused)");
    const EntropyTask t = fp.tasks[fp3];
    b.byte_off = t.byte_off;
    b.nbytes = t.nbytes;
    b.te = fp.tiles[(uint64_t)fp3 * fp.tiles_pp + tx];
    const uint32_t* bp = fp.bpos + (uint64_t)fp3 * (fp.nblk + 1) + tx * kFuseTw + col;
    const uint32_t p0 = has ? bp[0] : 0u, p1 = has ? bp[1] : 0u;
    b.pos = p0;
    // The length bounds the block's AC loop.  Capped: a block can run on past index 63 with ZRL
    // symbols indefinitely, but only its first ~67 symbols (<= 23 bits each) can place a coefficient
    // (each advances the index, a ZRL by 16), so a cap far above that changes nothing; the next
    // block's position comes from the index, not from this one's length.  (p1 < p0 only in a plane
    // whose index walk failed: its status fails the call.)
    b.len = p1 < p0 ? 0u : min(p1 - p0, 65535u);
}

__device__ __forceinline__ void locate_block(const FusedParams& fp, BlockAt& b) {
    const uint64_t rd = (b.byte_off * 8 + b.pos) >> 5, dw_max = (fp.bytes_len + 60) / 4;
    MJ423_BOUND(dw_max, fp.lim.bytes_dw, "bytes (fused)");
    const uint32_t* dw = reinterpret_cast<const uint32_t*>(fp.bytes);
    b.v0 = dw[rd < dw_max ? rd : dw_max];
    b.v1 = dw[rd + 1 < dw_max ? rd + 1 : dw_max];
    b.v2 = dw[rd + 2 < dw_max ? rd + 2 : dw_max];
}

__device__ __forceinline__ void decode_block(const FusedParams& fp, const BlockAt& b, bool has, bool P, uint8_t* slot,
                                             uint32_t swz, const uint8_t* zz) {
    Reader r;
    r.dw = reinterpret_cast<const uint32_t*>(fp.bytes);
    r.end = b.byte_off + b.nbytes;
    r.dw_max = (fp.bytes_len + 60) / 4;
    const uint64_t begin = b.byte_off * 8 + b.pos;
    {  // Reader::init on the dwords loaded by locate_block (the same masking at the stream's end)
        r.rd = begin >> 5;
        const uint32_t sh = (uint32_t)(begin & 31);
        r.win = (((uint64_t)r.fix(r.rd, b.v0) << 32) | r.fix(r.rd + 1, b.v1)) << sh;
        r.n = 64 - sh;
        r.rd += 2;
        r.nxt = b.v2;  // (raw, as Reader::refill expects when prefetching)
    }
    // >= 33 bits in the window: the DC symbol takes <= 19
    const uint32_t dsz = r.take(4);
    const int32_t diff = has ? huff_extend(r.take(dsz), dsz) : 0;
    // I: DC prediction inside the plane (lossless_decode.c:86-96) from the tile's predictor
    const uint32_t dcv = P ? (uint32_t)diff : b.te.y + wave_incl_sum((uint32_t)diff);
    auto at = [&](uint32_t n) { return reinterpret_cast<int16_t*>(slot + ((((n >> 3) ^ swz) & 7u) << 4) + (n & 7u) * 2); };
    if (!P) {
#pragma unroll
        for (int k = 0; k < 8; k++) reinterpret_cast<uint4*>(slot)[k] = make_uint4(0u, 0u, 0u, 0u);
    }
    if (!has) return;
    int16_t* d0 = at(0);
    *d0 = (int16_t)(P ? (uint32_t)(uint16_t)*d0 + dcv : dcv);
    // AC: RUN(4) SIZE(4) + VLI; SIZE 0: RUN 15 = ZRL, else EOB; a coefficient at index >= 63 ends
    // the block (lossless_decode.c:100-129).  A valid block ends exactly at its indexed length;
    // the length also bounds the walk of a damaged one.
    // One symbol per iteration from the window's top 32 bits (>= 33 valid after the refill; a symbol
    // takes <= 23): the header byte, the VLI after it, one shift of the window; `used` counts the
    // block's bits so far.
    uint32_t idx = 1, used = 4 + dsz;
    const uint64_t dw_max = r.dw_max;
    while (used < b.len) {
        // refill without the stream-end mask: a block the index placed inside its stream never
        // consumes a bit past the stream's end (a stream whose blocks run past it fails the call)
        if (r.n <= 32) {
            r.win |= (uint64_t)__builtin_bswap32(r.nxt) << (32 - r.n);
            r.n += 32;
            ++r.rd;
            r.nxt = r.dw[r.rd < dw_max ? r.rd : dw_max];
        }
        const uint32_t hi = (uint32_t)(r.win >> 32), run = hi >> 28, size = (hi >> 24) & 15u;
        const uint32_t vli = (uint32_t)((uint64_t)(hi << 8) >> (32 - size));  // (size 0: 0)
        const uint32_t tot = 8 + size;
        r.win <<= tot;
        r.n -= tot;
        used += tot;
        if (size == 0) {
            if (run != 15) break;  // EOB
            idx = min(idx + 16, 64u);
            continue;
        }
        idx = min(idx + run, 64u);
        const int32_t v = huff_extend(vli, size);
        if (idx <= 63) {
            int16_t* a = at(zz[idx]);
            *a = (int16_t)(P ? (uint32_t)(uint16_t)*a + (uint32_t)v : (uint32_t)v);
        }
        if (idx >= 63) break;
        idx++;
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
    uint8_t* state = lds;                  // the tile's accumulated quantized coefficients, one slot per block
    uint8_t* planes = lds + FT::COEF_BYTES;  // uint8 plane tiles, per frame
    uint32_t* lds_qt = reinterpret_cast<uint32_t*>(lds + FT::COEF_BYTES + FT::PLANE_BYTES);
    uint8_t* zz = lds + FT::COEF_BYTES + FT::PLANE_BYTES + 256;
    const int tid = threadIdx.x;
    if (tid < 16) reinterpret_cast<uint4*>(lds_qt)[tid] = reinterpret_cast<const uint4*>(p.qt_dev)[tid];
    if (tid < 64) zz[tid] = kZz[tid];
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
        stage_store<444, (int)kFuseTw, 256, kDefaultFlags>(state, tid, v);
    }
    __syncthreads();  // seed, tables: before the first frame's decode
    const uint32_t plane = (uint32_t)tid >> 6, col = (uint32_t)tid & 63u;  // wave = plane (wave 3: no block)
    const bool has = plane < 3 && (int)col < cs.tw;
    const bool dec = __builtin_amdgcn_readfirstlane(plane) < 3;  // waves 0-2
    BlockAt b;
    if (PRE && dec && f0 < f1) {
        fetch_block(fp, f0, plane, tx, col, has, b);
        locate_block(fp, b);
    }
    for (uint32_t f = f0; f < f1; f++) {
        const bool P = __builtin_amdgcn_readfirstlane(p.ftype[f]) != 0;
        if (dec) {
            if (!PRE) {
                fetch_block(fp, f, plane, tx, col, has, b);
                locate_block(fp, b);
            }
#if MJ423_FUSED_ABLATE != 3
            decode_block(fp, b, has, P, state + tid * 128, (uint32_t)tid & 7u, zz);
#endif
        }
        __syncthreads();
        const bool more = f + 1 < f1;
        if (PRE && dec && more) fetch_block(fp, f + 1, plane, tx, col, has, b);
        const TileCoord c = tile_coord<444>(p, f * p.tiles_per_frame + tx);
        MJ423_BOUND((uint64_t)f * p.out_fstride + (uint64_t)p.height * p.out_pitch - 1, fp.lim.out, "out (fused)");
#if MJ423_FUSED_ABLATE != 1
        decode_tile_idct<444, (int)kFuseTw, 256, FLAGS, false>(p, c, state, planes, tid, lds_qt, nullptr, nullptr);
#endif
        __syncthreads();
        if (PRE && dec && more) locate_block(fp, b);
#if MJ423_FUSED_ABLATE != 2
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
            if (c < cs.run_len(run))
                *reinterpret_cast<u32x4*>(p.state_out + st_off(k)) =
                    *reinterpret_cast<const u32x4*>(state + coef_off(FT::SLOTS_PER_CHUNK * k + (tid >> 3), tid & 7));
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
