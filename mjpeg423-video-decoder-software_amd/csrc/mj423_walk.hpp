// mj423_walk.hpp -- the entropy front end's block walk, host side:
// the serial decode of one plane's bitstream, lossless_decode.c:82-134, with pluggable
// output (dense planes, or the sparse transfer form of the streaming decoder).
//
// Bitstream (lossless_decode.c:204-246): per block a DC symbol SIZE(4) + VLI(SIZE), then
// AC symbols RUN(4) SIZE(4) + VLI(SIZE) until EOB (SIZE 0, RUN != 15) or index 63;
// RUN 15 / SIZE 0 is ZRL (16 zeros).  VLI amplitudes decode as HUFF_EXTEND (:204).
#pragma once

#include <cstddef>
#include <cstdint>
#include <cstring>

namespace mj423fe {

// mj/common/tables.c:35-42: zig-zag scan position -> natural index.
inline constexpr uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                                        12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                                        35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                                        58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

// MSB-first reader.  Equivalent to the reference's 32-bit bitbuffer + update_buffer
// (lossless_decode.c:139-162): both expose the next bits of the stream at the top of
// the window; a symbol needs at most 4+4+15 = 23 bits, and a refill keeps at least 25.
// The unbounded form (end == nullptr) never reads more than 4 bytes past the consumed
// position -- no further ahead than the reference -- so it is as safe as the reference.
struct Bits {
    const uint8_t* p;
    const uint8_t* end;  // nullptr: unbounded, like the reference
    uint64_t win = 0;
    int n = 0;  // valid bits at the top of win
    bool over = false;

    // Bounded stream with >= 8 readable bytes at p: one unaligned big-endian load and no
    // branch; afterwards n is in [56, 63].  Whole bytes that fit go in; the bits of the
    // partial byte also land in `win` but are re-ORed with the same values next time.
    inline void refill_fast() {
        uint64_t v;
        std::memcpy(&v, p, 8);
        win |= __builtin_bswap64(v) >> n;
        p += (63 - n) >> 3;
        n |= 56;
    }
    inline void refill() {
        if (n > 24) return;
        if (end && end - p >= 8) {
            refill_fast();
            return;
        }
        while (n <= 24) {  // byte by byte: stream tail, or the unbounded reference-compatible form
            uint64_t b = 0;
            if (!end || p < end)
                b = *p;
            else
                over = true;
            ++p;
            win |= b << (56 - n);
            n += 8;
        }
    }
    template <bool BOUNDED>
    inline void refill_any() {
        if (BOUNDED && end - p >= 8)
            refill_fast();
        else
            refill();
    }
    inline void skip(int k) {  // k in [0, 24]; caller guarantees n >= k
        win <<= k;
        n -= k;
    }
    inline uint32_t take(int k) {  // k in [1, 24]
        const uint32_t v = (uint32_t)(win >> (64 - k));
        skip(k);
        return v;
    }
    inline uint32_t take0(int k) {  // k in [0, 24]; k == 0 gives 0
        const uint32_t v = (uint32_t)((win >> (63 - k)) >> 1);
        skip(k);
        return v;
    }
    size_t bytes_used(const uint8_t* start) const { return ((size_t)(p - start) * 8 - (size_t)n + 7) / 8; }
};

// HUFF_EXTEND (lossless_decode.c:204): a size-bit VLI amplitude -> signed value; size 0 -> 0.
inline int32_t vli(uint32_t v, int size) {
    return v < ((1u << size) >> 1) ? (int32_t)v - (1 << size) + 1 : (int32_t)v;
}

// One table lookup on the next 12 bits decodes any AC symbol whose RUN/SIZE header and
// amplitude fit in them (SIZE <= 4: |e| <= 15, nearly every symbol of real and synthetic
// streams): entry = value (int16, bits 0-15) | run << 16 | length << 20 | kind << 26.
enum : uint32_t { kAcCoef = 0, kAcEob = 1, kAcZrl = 2, kAcLong = 3 };
struct AcTable {
    uint32_t e[4096];
    constexpr AcTable() : e() {
        for (uint32_t i = 0; i < 4096; i++) {
            const uint32_t run = i >> 8, size = (i >> 4) & 15;
            if (size == 0) {
                e[i] = (8u << 20) | ((run == 15 ? kAcZrl : kAcEob) << 26);
            } else if (size <= 4) {
                const uint32_t v = (i & 15) >> (4 - size);
                const int32_t val = v < (1u << (size - 1)) ? (int32_t)v - (1 << size) + 1 : (int32_t)v;
                e[i] = (uint32_t)(uint16_t)val | (run << 16) | ((8 + size) << 20) | (kAcCoef << 26);
            } else {
                e[i] = kAcLong << 26;
            }
        }
    }
};
inline constexpr AcTable kAcTable{};

// The walk over `nblocks` blocks.  Sink: begin(blk), dc(e), ac(natural index, e), end(blk).
// BOUNDED: `b.end` is set (every product call); false only for the reference-compatible
// unbounded lossless_decode() symbol.
template <bool BOUNDED, class Sink>
inline void walk_blocks(Bits& b, int nblocks, Sink& s) {
    for (int blk = 0; blk < nblocks; blk++) {
        s.begin(blk);
        if (b.n < 19) b.refill_any<BOUNDED>();  // DC: at most 4 + 15 bits
        // DC: SIZE(4) + VLI (input_DC :210-224)
        const int dsize = (int)b.take(4);
        s.dc(vli(b.take0(dsize), dsize));
        for (int index = 1;;) {  // AC: RUN(4) SIZE(4) + VLI (input_AC :227-246)
            if (b.n < 23) b.refill_any<BOUNDED>();  // AC: at most 4 + 4 + 15 bits
            const uint32_t t = kAcTable.e[b.win >> 52];
            const uint32_t kind = t >> 26;
            int32_t e;
            if (kind == kAcCoef) {
                b.skip((int)(t >> 20) & 31);
                index += (int)(t >> 16) & 15;
                e = (int16_t)t;
            } else if (kind == kAcEob) {
                b.skip(8);
                break;  // EOB (:111-114)
            } else if (kind == kAcZrl) {
                b.skip(8);
                index += 16;  // ZRL (:107-110)
                continue;
            } else {  // SIZE 5..15
                index += (int)b.take(4);
                const int size = (int)b.take(4);
                e = vli(b.take(size), size);
            }
            if (index <= 63) s.ac(kZigzag[index], e);  // past 63 is UB in the reference: no write
            if (index >= 63) break;
            index++;
        }
        s.end(blk);
    }
}

// Dense output (lossless_decode.c:90-126).  QD: quantized domain, no
// dequantization; P: add onto the plane instead of setting (DC differential per frame).
template <bool QD, bool P>
struct DenseSink {
    int16_t* dst;
    const int16_t* quant;
    int16_t* pe = nullptr;
    int16_t cur = 0;
    inline void begin(int blk) { pe = dst + (size_t)blk * 64; }
    inline void dc(int32_t e) {
        if (P) {
            pe[0] = (int16_t)(pe[0] + (QD ? e : e * quant[0]));  // :90-92
        } else {
            cur = (int16_t)(cur + e);  // :93-96, int16 running sum
            pe[0] = (int16_t)(QD ? cur : cur * quant[0]);
        }
    }
    inline void ac(int k, int32_t e) {
        const int32_t v = QD ? e : e * quant[k];
        pe[k] = (int16_t)(P ? pe[k] + v : v);  // :121-126
    }
    inline void end(int) {}
};

// Sparse transfer form for the streaming decoder: counts[b] = coefficients the stream
// sets in block b; one uint32 per coefficient, natural index << 16 | (uint16)value
// (I-frames: absolute value, DC prefix-summed and omitted when 0; P-frames: the delta
// lossless_decode would add); seg_off[s] = entries before block 256*s.
template <bool P>
struct SparseSink {
    uint8_t* counts;
    uint32_t* seg_off;
    uint32_t* ent;
    size_t n = 0, n0 = 0;
    int16_t cur = 0;
    inline void begin(int blk) {
        if ((blk & 255) == 0) seg_off[blk >> 8] = (uint32_t)n;
        n0 = n;
    }
    inline void dc(int32_t e) {
        if (P) {  // branch-free: the slot is overwritten when the value is 0
            ent[n] = (uint32_t)(uint16_t)e;
            n += e != 0;
        } else {
            cur = (int16_t)(cur + e);
            ent[n] = (uint32_t)(uint16_t)cur;
            n += cur != 0;
        }
    }
    inline void ac(int k, int32_t e) { ent[n++] = ((uint32_t)k << 16) | (uint16_t)e; }
    inline void end(int blk) { counts[blk] = (uint8_t)(n - n0); }
};

// Dense walk; returns the bytes consumed (bits taken, rounded up).
template <bool QD>
inline size_t walk(int nblocks, const uint8_t* bs, const uint8_t* end, int16_t* dst, const int16_t* quant, bool P,
                   bool* overrun) {
    Bits b{bs, end};
    if (!P) std::memset(dst, 0, (size_t)nblocks * 64 * sizeof(int16_t));  // :77-78
    auto go = [&](auto sink) {
        if (end)
            walk_blocks<true>(b, nblocks, sink);
        else
            walk_blocks<false>(b, nblocks, sink);
    };
    if (P)
        go(DenseSink<QD, true>{dst, quant});
    else
        go(DenseSink<QD, false>{dst, quant});
    if (overrun) *overrun = b.over;
    return b.bytes_used(bs);
}

// Sparse walk of a bounded stream; returns the entry count.  `ent` holds room for
// 64 * nblocks entries (a block sets at most 64; the DC slot is written before it is
// known to be needed, but always below that bound).
inline size_t walk_sparse(int nblocks, const uint8_t* bs, const uint8_t* end, bool P, uint8_t* counts,
                          uint32_t* seg_off, uint32_t* ent, bool* overrun, size_t* used_bytes) {
    Bits b{bs, end};
    size_t n;
    if (P) {
        SparseSink<true> s{counts, seg_off, ent};
        walk_blocks<true>(b, nblocks, s);
        n = s.n;
    } else {
        SparseSink<false> s{counts, seg_off, ent};
        walk_blocks<true>(b, nblocks, s);
        n = s.n;
    }
    seg_off[(nblocks + 255) >> 8] = (uint32_t)n;
    if (overrun) *overrun = b.over;
    *used_bytes = b.bytes_used(bs);
    return n;
}

}  // namespace mj423fe
