// mj423_bits.hpp -- the bitstream reader shared by the GPU entropy front end (mj423_entropy.hip)
// and the fused .mpg decode kernel (mj423_fused.hip).  Format: lossless_decode.c:82-134,204-246
// (MSB-first fields, VLI amplitudes with HUFF_EXTEND).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mj423 {
namespace {

// zig-zag scan position -> natural index (mj/common/tables.c:35-42)
__constant__ uint8_t kZz[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

typedef uint32_t v4u32 __attribute__((ext_vector_type(4)));

// Packed state: bits 0-31 position (bits from the stream's first byte), bit 32 mode
// (0 = a DC symbol is next, 1 = AC), bits 33-39 zig-zag index (AC only; 0 when DC).
__device__ __forceinline__ uint64_t pack(uint32_t pos, uint32_t ac, uint32_t idx) {
    return (uint64_t)pos | ((uint64_t)ac << 32) | ((uint64_t)(ac ? idx : 0) << 33);
}

// MSB-first reader of one stream, bytes at or past `end` reading as zero.
// Staged window: a lane's dwords [w0, w0 + kWin) copied to its own LDS slot by independent loads
// before the walk, so the walk's refills -- a dependent chain of global loads otherwise -- read LDS.
#ifndef MJ423_ENTPAR_SUB_BYTES  // (mj423_entropy.h: the subsequence length)
#define MJ423_ENTPAR_SUB_BYTES 64
#endif
#ifndef MJ423_ENTPAR_WIN_PAD  // dwords of the window beyond the subsequence's own (A/B)
#define MJ423_ENTPAR_WIN_PAD 8
#endif
constexpr uint32_t kWin = MJ423_ENTPAR_SUB_BYTES / 4 + MJ423_ENTPAR_WIN_PAD;  // 768 bits at 64-B subsequences: one plus the symbols straddling its ends
// A pointer into LDS as such: reads through it are ds_read.  (A generic pointer selected against a
// global one compiled to a flat load in the walk's refill -- a dependent chain through the slower
// flat path on every 32 bits.)
typedef __attribute__((address_space(3))) uint32_t lds_u32;
// Refills are software-pipelined (MJ423_READER_PREFETCH, default on): the dword after the window
// is loaded one refill ahead and only masked and byte-swapped when it is shifted in, so the load's
// latency (LDS or global) overlaps the symbols decoded meanwhile instead of sitting on the walk's
// dependent chain at every 32 bits.
#ifndef MJ423_READER_PREFETCH
#define MJ423_READER_PREFETCH 1
#endif
struct Reader {
    const uint32_t* dw;
    uint64_t end;      // absolute byte index of the stream's end
    uint64_t dw_max;   // last dword index inside the upload buffer
    uint64_t rd;       // next dword to shift in
    uint64_t win;      // next bits, MSB first
    uint32_t n;        // valid bits in win
    uint32_t nxt = 0;  // dword rd as loaded (raw; with `lds`: fixed), when prefetching
    const lds_u32* lw = nullptr;  // staged window (LDS), dwords [w0, w0 + kWin) already fixed, when `lds`
    uint64_t w0 = 0;
    uint32_t wd = 0;   // (lds) rd - w0, kept in 32 bits for the window-only refill
    bool lds = false;  // (not `lw != nullptr`: a slot at LDS offset 0 compares equal to the null pointer)
    __device__ __forceinline__ uint32_t raw(uint64_t i) const { return dw[i < dw_max ? i : dw_max]; }
    // dword i masked and byte-swapped: from the staged window when it holds i
    __device__ __forceinline__ uint32_t fixed(uint64_t i) const {
        const uint64_t d = i - w0;  // (wraps for i < w0: outside the window)
        if (lds && d < kWin) return lw[d];
        return fix(i, raw(i));
    }
    __device__ __forceinline__ uint32_t fix(uint64_t i, uint32_t v) const {  // bytes at or past `end` read as zero; MSB first
        const uint64_t a = 4 * i;
        const uint32_t m = a + 4 <= end ? 0xffffffffu : a >= end ? 0u : (1u << (8 * (uint32_t)(end - a))) - 1u;
        return __builtin_bswap32(v & m);
    }
    __device__ __forceinline__ uint32_t load(uint64_t i) const { return fixed(i); }
    __device__ __forceinline__ void init(uint64_t absbit) {
        rd = absbit >> 5;
        const uint32_t sh = (uint32_t)(absbit & 31);
        win = (((uint64_t)load(rd) << 32) | load(rd + 1)) << sh;
        n = 64 - sh;
        rd += 2;
        wd = (uint32_t)(rd - w0);
        if (lds)
            nxt = fixed(rd);
        else if (MJ423_READER_PREFETCH)
            nxt = raw(rd);
    }
    __device__ __forceinline__ void refill() {
        if (n <= 32) {
            if (lds && MJ423_READER_PREFETCH) {
                win |= (uint64_t)nxt << (32 - n);
                ++wd;
                nxt = fixed(++rd);
            } else if (MJ423_READER_PREFETCH) {
                win |= (uint64_t)fix(rd, nxt) << (32 - n);
                nxt = raw(++rd);
            } else {
                win |= (uint64_t)load(rd++) << (32 - n);
            }
            n += 32;
        }
    }
    // The same for a walk that never leaves its staged window (the synchronisation walk: it ends at
    // the first symbol boundary past its subsequence, <= kSubBits + 23 bits from a start inside it,
    // plus the dword read ahead -- inside the window's kWin * 32 - 32 bits).  One LDS read per refill,
    // issued a refill ahead; no global path to merge with, so nothing makes the wave wait for it early.
    // The window's dwords were masked and byte-swapped when staged: a refill is one shift and an OR.
    __device__ __forceinline__ void refill_lds() {
        if (n <= 32) {
            win |= (uint64_t)nxt << (32 - n);
            ++rd;
            const uint32_t d = ++wd;
#ifdef MJ423_DEBUG_WINDOW
            if (d >= kWin) printf("refill_lds past the window: d=%u rd=%llu w0=%llu n=%u\n", d,
                                  (unsigned long long)rd, (unsigned long long)w0, n);
#endif
            nxt = lw[d < kWin ? d : kWin - 1];
            n += 32;
        }
    }
    __device__ __forceinline__ uint32_t take(uint32_t k) {  // k in [0, 24]; k == 0 gives 0
        const uint32_t v = (uint32_t)((win >> (63 - k)) >> 1);
        win <<= k;
        n -= k;
        return v;
    }
    __device__ __forceinline__ uint64_t abspos() const { return rd * 32 - n; }
};

__device__ __forceinline__ int32_t huff_extend(uint32_t v, uint32_t size) {  // size 0 -> 0
    return v < ((1u << size) >> 1) ? (int32_t)v - (1 << size) + 1 : (int32_t)v;
}

}  // namespace
}  // namespace mj423
