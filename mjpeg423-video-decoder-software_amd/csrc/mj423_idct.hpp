// mj423_idct.hpp -- device-side building blocks of the hot path (gfx950, wave64).
//
// One 8x8 block per LANE: the lane holds its 64 dequantized coefficients in
// 32 VGPRs (int16 pairs), runs the column pass into a 64-entry int32
// workspace held in registers, then the row pass, clamps and packs to bytes.
// No transposes, no shuffles, no LDS traffic inside the transform.
//
// Bit-exactness contract: the reference's idct() evaluates
// int32 expressions with two's-complement wrap and arithmetic right shifts.
// Every add/sub/shl below is a ring operation mod 2^32 (done on uint32_t),
// so any algebraically equal arrangement of the butterfly gives the same
// pre-descale sums as the reference, wrap included.  Multiplies use the
// full-rate 24-bit multiplier (v_mul_i32_i24 / v_mad_i32_i24): its operands
// are exact as long as they fit in signed 24 bits, which holds here --
// pass-1 operands are sums of <= 4 int16 (|v| <= 2^17), pass-2 operands are
// sums of <= 4 workspace values, each DESCALE(int32, 11) in [-2^20, 2^20),
// so |v| <= 2^22.  The low 32 bits of the 48-bit product are then exactly
// the reference's wrapped int32 product.
//
// Reference: core0/software/common/libs/mjpeg423/decoder/idct.c:22-181,
//            common/dct_math.h:32-78.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mj423 {

// FIX(c) = round(c * 2^CONST_BITS), CONST_BITS = 13 (dct_math.h:50-64).
constexpr int K0298 = 2446, K0390 = 3196, K0541 = 4433, K0765 = 6270, K0899 = 7373,
              K1175 = 9633, K1501 = 12299, K1847 = 15137, K1961 = 16069, K2053 = 16819,
              K2562 = 20995, K3072 = 25172;

__device__ __forceinline__ uint32_t mul24(int32_t a, int32_t b) { return (uint32_t)__mul24(a, b); }
__device__ __forceinline__ uint32_t mad24(int32_t a, int32_t b, uint32_t c) {
    return (uint32_t)__mul24(a, b) + c;
}

// One 8-point LLM butterfly (idct.c pass 1 :46-105 / pass 2 :121-177) with the
// DESCALE rounding constant folded into the DC term:
//   PASS 1: y = (sum + 2^10) >> 11        (CONST_BITS - PASS1_BITS)
//   PASS 2: y =  sum + 2^17               (the >> 18 happens in the saturating pack)
// Folding is exact: every output is s_i +/- o_j and each s_i carries the DC
// term e0 or e1 exactly once.
template <int PASS>
__device__ __forceinline__ void butterfly8(const int32_t x[8], int32_t y[8]) {
    // even part: rotator sqrt(2)*c6 on (x2, x6) (idct.c:49-55)
    const uint32_t r = mul24(x[2] + x[6], K0541);
    const uint32_t e2 = mad24(x[6], -K1847, r);
    const uint32_t e3 = mad24(x[2], K0765, r);
    // DC/x4 butterfly scaled by 2^13 (idct.c:57-60), rounding constant folded in
    uint32_t x0s;
    if (PASS == 1)
        x0s = ((uint32_t)x[0] << 13) + (1u << 10);
    else
        x0s = ((uint32_t)x[0] + 16u) << 13;  // 16 << 13 == 1 << 17
    const uint32_t e0 = x0s + ((uint32_t)x[4] << 13);
    const uint32_t e1 = mad24(x[4], -8192, x0s);
    const uint32_t s0 = e0 + e3, s3 = e0 - e3, s1 = e1 + e2, s2 = e1 - e2;

    // odd part, inputs x7, x5, x3, x1 (idct.c:68-94)
    const int32_t a = x[7] + x[1], b = x[5] + x[3], c = x[7] + x[3], d = x[5] + x[1];
    const uint32_t z5 = mul24(c + d, K1175);
    const uint32_t pa = mul24(a, -K0899);
    const uint32_t pb = mul24(b, -K2562);
    const uint32_t pc = mad24(c, -K1961, z5);
    const uint32_t pd = mad24(d, -K0390, z5);
    const uint32_t o7 = mad24(x[7], K0298, pa) + pc;
    const uint32_t o5 = mad24(x[5], K2053, pb) + pd;
    const uint32_t o3 = mad24(x[3], K3072, pb) + pc;
    const uint32_t o1 = mad24(x[1], K1501, pa) + pd;

    constexpr int SH = PASS == 1 ? 11 : 0;
    y[0] = (int32_t)(s0 + o1) >> SH;
    y[7] = (int32_t)(s0 - o1) >> SH;
    y[1] = (int32_t)(s1 + o3) >> SH;
    y[6] = (int32_t)(s1 - o3) >> SH;
    y[2] = (int32_t)(s2 + o5) >> SH;
    y[5] = (int32_t)(s2 - o5) >> SH;
    y[3] = (int32_t)(s3 + o7) >> SH;
    y[4] = (int32_t)(s3 - o7) >> SH;
}

__device__ __forceinline__ int32_t lo16(uint32_t v) { return (int32_t)(int16_t)(v & 0xffffu); }
__device__ __forceinline__ int32_t hi16(uint32_t v) { return (int32_t)v >> 16; }
__device__ __forceinline__ uint32_t clamp255(int32_t v) { return (uint32_t)min(max(v, 0), 255); }

// v_ashr_pk_u8_i32 (gfx950): byte0 = sat_u8(a >> sh), byte1 = sat_u8(b >> sh), where
// sat_u8 clamps the signed value to [0, 255].  That is NORMALIZE of idct.c:20 after
// DESCALE, and NORMALIZE_RGB of ycbcr_to_rgb.c:19 (a negative sum shifts to a
// negative value, which saturates to 0 exactly like the `temp < 0` branch).
// Upper 16 bits of the result are not used by callers.
template <int SH>
__device__ __forceinline__ uint32_t ashr_pk_u8(int32_t a, int32_t b) {
    uint32_t r;
    asm("v_ashr_pk_u8_i32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "n"(SH));
    return r;
}
// {lo.byte0, lo.byte1, hi.byte0, hi.byte1}
__device__ __forceinline__ uint32_t join16(uint32_t lo, uint32_t hi) { return __builtin_amdgcn_perm(hi, lo, 0x05040100u); }
// The same pair written into bits 16..31 of `lo`, bits 0..15 kept (VOP3 op_sel on the
// destination): join16(lo, ashr_pk_u8<SH>(a, b)) in one instruction (tools/isa_probe.hip
// checks the semantics on the MI355X).
template <int SH>
__device__ __forceinline__ uint32_t ashr_pk_u8_hi(uint32_t lo, int32_t a, int32_t b) {
    asm("v_ashr_pk_u8_i32 %0, %1, %2, %3 op_sel:[0,0,0,1]" : "+v"(lo) : "v"(a), "v"(b), "n"(SH));
    return lo;
}

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// (int16)(Q * q) for two packed coefficients at once: v_pk_mul_lo_u16 keeps the
// low 16 bits of each product, which is exactly the int16 truncation of
// lossless_decode.c:95,125.
__device__ __forceinline__ uint32_t dequant_pair(uint32_t q, uint32_t t) {
    u16x2 a = __builtin_bit_cast(u16x2, q), b = __builtin_bit_cast(u16x2, t);
    return __builtin_bit_cast(uint32_t, a * b);
}

typedef short s16x2 __attribute__((ext_vector_type(2)));

// D = a.lo*b.lo + a.hi*b.hi + c with int16 x int16 products (v_dot2c_i32_i16); the
// sum wraps mod 2^32 like the reference's int32 arithmetic.
__device__ __forceinline__ uint32_t dot2(uint32_t a, uint32_t b, uint32_t c) {
    return (uint32_t)__builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, b), (int)c, false);
}
__device__ __forceinline__ constexpr uint32_t k2(int lo, int hi) {
    return (uint32_t)(uint16_t)(int16_t)lo | ((uint32_t)(uint16_t)(int16_t)hi << 16);
}

// Pass 1 (columns, idct.c:39-109) of ONE column as int16-pair dot products.
// The LLM butterfly is a chain of ring operations mod 2^32, so each of its sums is
// exactly a fixed integer combination of the eight inputs; pass-1 inputs are int16
// and every combined coefficient fits int16 (|c| <= 11363), so two-term
// v_dot2_i32_i16 evaluates those sums exactly:
//   even  s0,s3 = 8192(x0+x4) +/- (10703 x2 + 4433 x6)    s1,s2 = 8192(x0-x4) +/- (4433 x2 - 10704 x6)
//   odd   o1 = 11363 x1 + 9633 x3 + 6437 x5 + 2260 x7     o3 = 9633 x1 - 2259 x3 - 11362 x5 - 6436 x7
//         o5 = 6437 x1 - 11362 x3 + 2261 x5 + 9633 x7     o7 = 2260 x1 - 6436 x3 + 9633 x5 - 11363 x7
// (coefficients = the products of FIX_* constants along each butterfly path,
// e.g. o1's x1 term is 12299 - 7373 - 3196 + 9633).  DESCALE's 2^10 rides in the
// accumulator.  Pairs: p04 = (x0,x4), p26 = (x2,x6), p13 = (x1,x3), p57 = (x5,x7).
// The constant pairs are pinned in SGPRs (s_mov inside asm, opaque to the compiler) and
// the products issued as VOP3P v_dot2_i32_i16 with the accumulator as a separate source:
// with literal constants the compiler picks the destructive VOP2 v_dot2c form and pays a
// v_mov per accumulator (~8 per column).  Shared even-part products are formed once.
template <uint32_t K>
__device__ __forceinline__ uint32_t sconst() {
    uint32_t s;
    asm("s_mov_b32 %0, %1" : "=s"(s) : "i"(K));
    return s;
}
__device__ __forceinline__ uint32_t dot2s(uint32_t k, uint32_t a) {  // k.lo*a.lo + k.hi*a.hi
    uint32_t d;
    asm("v_dot2_i32_i16 %0, %1, %2, 0" : "=v"(d) : "s"(k), "v"(a));
    return d;
}
__device__ __forceinline__ uint32_t dot2s(uint32_t k, uint32_t a, uint32_t c) {  // ... + c
    uint32_t d;
    asm("v_dot2_i32_i16 %0, %1, %2, %3" : "=v"(d) : "s"(k), "v"(a), "v"(c));
    return d;
}

// The butterfly's even and odd sums of one 8-point transform as int16-pair dot products
// (the constants above; the even sums s_i with the accumulator `rnd` chained in).
struct Sums8 {
    uint32_t s0, s1, s2, s3, o1, o3, o5, o7;
};
__device__ __forceinline__ Sums8 sums8(uint32_t p04, uint32_t p26, uint32_t p13, uint32_t p57, uint32_t rnd) {
    // even: e0 = 8192(x0+x4) + R, e1 = 8192(x0-x4) + R; s0,s3 = e0 +/- (10703 x2 + 4433 x6),
    //       s1,s2 = e1 +/- (4433 x2 - 10704 x6)
    Sums8 t;
    const uint32_t e0 = dot2s(sconst<k2(8192, 8192)>(), p04, rnd);
    const uint32_t e1 = dot2s(sconst<k2(8192, -8192)>(), p04, rnd);
    t.s0 = dot2s(sconst<k2(10703, 4433)>(), p26, e0);
    t.s3 = dot2s(sconst<k2(-10703, -4433)>(), p26, e0);
    t.s1 = dot2s(sconst<k2(4433, -10704)>(), p26, e1);
    t.s2 = dot2s(sconst<k2(-4433, 10704)>(), p26, e1);
    t.o1 = dot2s(sconst<k2(6437, 2260)>(), p57, dot2s(sconst<k2(11363, 9633)>(), p13));
    t.o3 = dot2s(sconst<k2(-11362, -6436)>(), p57, dot2s(sconst<k2(9633, -2259)>(), p13));
    t.o5 = dot2s(sconst<k2(2261, 9633)>(), p57, dot2s(sconst<k2(6437, -11362)>(), p13));
    t.o7 = dot2s(sconst<k2(9633, -11363)>(), p57, dot2s(sconst<k2(2260, -6436)>(), p13));
    return t;
}

__device__ __forceinline__ void pass1_column(uint32_t p04, uint32_t p26, uint32_t p13, uint32_t p57, uint32_t rnd,
                                             int32_t y[8]) {
    const Sums8 t = sums8(p04, p26, p13, p57, rnd);
    const uint32_t s0 = t.s0, s1 = t.s1, s2 = t.s2, s3 = t.s3, o1 = t.o1, o3 = t.o3, o5 = t.o5, o7 = t.o7;
    y[0] = (int32_t)(s0 + o1) >> 11;
    y[7] = (int32_t)(s0 - o1) >> 11;
    y[1] = (int32_t)(s1 + o3) >> 11;
    y[6] = (int32_t)(s1 - o3) >> 11;
    y[2] = (int32_t)(s2 + o5) >> 11;
    y[5] = (int32_t)(s2 - o5) >> 11;
    y[3] = (int32_t)(s3 + o7) >> 11;
    y[4] = (int32_t)(s3 - o7) >> 11;
}

// {lo16(a), lo16(b)} and {hi16(a), hi16(b)}: one column's values from two rows.
__device__ __forceinline__ uint32_t pair_lo(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x05040100u); }
__device__ __forceinline__ uint32_t pair_hi(uint32_t a, uint32_t b) { return __builtin_amdgcn_perm(b, a, 0x07060302u); }

// Full 8x8 inverse DCT of one block held by this lane.
//   d[r][p] : row r, packed int16 pair (col 2p low half, col 2p+1 high half)
//   out[r][0..1] : row r, 8 uint8 pixels packed little-endian
__device__ __forceinline__ void idct8x8(const uint32_t (&d)[8][4], uint32_t (&out)[8][2]) {
    int32_t ws[8][8];  // ws[n][c], scaled by 2^PASS1_BITS
    const uint32_t rnd = 1u << 10;  // DESCALE(., 11) rounding, one VGPR for all columns
#pragma unroll
    for (int p = 0; p < 4; p++) {  // pass 1: columns 2p, 2p+1 (idct.c:39-109)
        int32_t y[8];
        pass1_column(pair_lo(d[0][p], d[4][p]), pair_lo(d[2][p], d[6][p]), pair_lo(d[1][p], d[3][p]),
                     pair_lo(d[5][p], d[7][p]), rnd, y);
#pragma unroll
        for (int n = 0; n < 8; n++) ws[n][2 * p] = y[n];
        pass1_column(pair_hi(d[0][p], d[4][p]), pair_hi(d[2][p], d[6][p]), pair_hi(d[1][p], d[3][p]),
                     pair_hi(d[5][p], d[7][p]), rnd, y);
#pragma unroll
        for (int n = 0; n < 8; n++) ws[n][2 * p + 1] = y[n];
    }
#pragma unroll
    for (int r = 0; r < 8; r++) {  // pass 2: rows, NORMALIZE to [0,255] (idct.c:115-180, :20)
        int32_t y[8];
        butterfly8<2>(ws[r], y);
        out[r][0] = ashr_pk_u8_hi<18>(ashr_pk_u8<18>(y[0], y[1]), y[2], y[3]);
        out[r][1] = ashr_pk_u8_hi<18>(ashr_pk_u8<18>(y[4], y[5]), y[6], y[7]);
    }
}

// ---------------------------------------------------------------- int16 workspace
// The common case: every pass-1 result (workspace value) fits int16.  Then the row pass
// takes int16 pairs too and runs on v_dot2_i32_i16 like the column pass (the same exact
// combined constants; the workspace is the reference's int32 value, so the row sums are
// the reference's mod 2^32), and pass 1 hands its results over packed: with
// y' = (sum << 5), hi16(y') is the low 16 bits of sum >> 11 (DESCALE(., 11)), so one
// v_perm_b32 packs two of them.
//
// When it holds: a workspace value is floor((t + 1024) / 2048) with t = sum_k M[n][k] x[k]
// over one column (M = the combined pass-1 constants); it fits int16 iff
// -2^26 <= t + 1024 < 2^26.  Every row of M has Euclidean norm <= 23170.71, so by
// Cauchy-Schwarz |t| <= 23170.71 * ||column||, and ||column||^2 <= 8 388 183 suffices.
// The test (idct8x8_auto, and decode_tile_idct in mj423_kernels.hip) bounds each column by the
// energy of its column PAIR (the packed register layout): E_p = sum_r x[r][2p]^2 + x[r][2p+1]^2, summed with saturating v_dot2 (a
// full-range block cannot wrap to a small value).  Realistic blocks are far inside
// (a DC of 2040 alone is 4.16 M); the wave takes the int16 path only if every active lane
// passes, otherwise the int32 path above.
constexpr int32_t kWs16Energy = 8388183;

__device__ __forceinline__ int32_t sdot2_sat(uint32_t a, int32_t c) {
    return __builtin_amdgcn_sdot2(__builtin_bit_cast(s16x2, a), __builtin_bit_cast(s16x2, a), c, true);
}
__device__ __forceinline__ void idct8x8_w16(const uint32_t (&d)[8][4], uint32_t (&out)[8][2]) {
    // w[r][0] = {ws[r][0], ws[r][4]}, w[r][1] = {ws[r][2], ws[r][6]}, w[r][2] = {ws[r][1], ws[r][3]},
    // w[r][3] = {ws[r][5], ws[r][7]}: the pairs the row pass multiplies
    uint32_t w[8][4];
    const uint32_t rnd = 1u << 10;
    // column c: p = c / 2, half = c % 2 (the packed pair of that row holds columns 2p, 2p+1)
    auto column = [&](int c, uint32_t y[8]) {
        const int p = c >> 1;
        const bool hi = (c & 1) != 0;
        auto pr = [&](int ra, int rb) { return hi ? pair_hi(d[ra][p], d[rb][p]) : pair_lo(d[ra][p], d[rb][p]); };
        const Sums8 t = sums8(pr(0, 4), pr(2, 6), pr(1, 3), pr(5, 7), rnd);
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
    for (int q = 0; q < 4; q++) {  // pass 1, two columns at a time, packed as the row pass wants them
        uint32_t ya[8], yb[8];
        column(kPairCols[q][0], ya);
        column(kPairCols[q][1], yb);
#pragma unroll
        for (int r = 0; r < 8; r++) w[r][q] = pair_hi(ya[r], yb[r]);
    }
    const uint32_t rnd2 = 1u << 17;  // DESCALE(., 18) rounding
#pragma unroll
    for (int r = 0; r < 8; r++) {  // pass 2: rows, NORMALIZE to [0,255] (idct.c:115-180, :20)
        const Sums8 t = sums8(w[r][0], w[r][1], w[r][2], w[r][3], rnd2);
        const int32_t y0 = (int32_t)(t.s0 + t.o1), y7 = (int32_t)(t.s0 - t.o1);
        const int32_t y1 = (int32_t)(t.s1 + t.o3), y6 = (int32_t)(t.s1 - t.o3);
        const int32_t y2 = (int32_t)(t.s2 + t.o5), y5 = (int32_t)(t.s2 - t.o5);
        const int32_t y3 = (int32_t)(t.s3 + t.o7), y4 = (int32_t)(t.s3 - t.o7);
        out[r][0] = ashr_pk_u8_hi<18>(ashr_pk_u8<18>(y0, y1), y2, y3);
        out[r][1] = ashr_pk_u8_hi<18>(ashr_pk_u8<18>(y4, y5), y6, y7);
    }
}

// The 8x8 IDCT of the lane's block, int16-workspace form when the whole wave allows it.
// `load(r, dr)` produces row r of the dequantized block (four int16 pairs); it is called
// twice per row -- once for the width test, once for the transform -- so that the two
// transforms are separate code paths that each hold only their own registers (a decision
// made on a block already held in registers cost ~25-30 extra VGPRs and spills).
// `valid`: this lane holds a real block (others never veto the int16 form).
template <class Load>
__device__ __forceinline__ void idct8x8_auto(Load&& load, uint32_t (&out)[8][2], bool valid) {
    bool wide = false;
    if (valid) {
        int32_t e[4] = {0, 0, 0, 0};
#pragma unroll
        for (int r = 0; r < 8; r++) {
            uint32_t dr[4];
            load(r, dr);
#pragma unroll
            for (int k = 0; k < 4; k++) e[k] = sdot2_sat(dr[k], e[k]);
        }
        wide = max(max(e[0], e[1]), max(e[2], e[3])) > kWs16Energy;
    }
    if (__builtin_amdgcn_ballot_w64(wide) == 0) {
        uint32_t d[8][4];
#pragma unroll
        for (int r = 0; r < 8; r++) load(r, d[r]);
        idct8x8_w16(d, out);
    } else {
        uint32_t d[8][4];
#pragma unroll
        for (int r = 0; r < 8; r++) load(r, d[r]);
        idct8x8(d, out);
    }
}

// ---------------------------------------------------------------- colour
// ycbcr_to_rgb.c:32-44 computes v = (Y << 14) + k * (C - 128) in Q14 and takes
// NORMALIZE_RGB(v) = sat_u8(v >> 14).  Here everything is scaled by 4:
// v' = (Y << 16) + 4k * (C - 128) = 4v exactly (|v| < 2^23, no overflow), and
// v' >> 16 == v >> 14 (floor division by 2^16 of 4v).  Y << 16 is a byte
// placement (one v_perm_b32), and the pair saturation is one v_ashr_pk_u8_i32.
struct ChromaTerms {
    int32_t r, g, b;  // 4 * (22970 Crr), 4 * (-5638 Cbb - 11700 Crr), 4 * (29032 Cbb)
};
__device__ __forceinline__ ChromaTerms chroma_terms(uint32_t cb, uint32_t cr) {
    const int32_t cbb = (int32_t)cb - 128, crr = (int32_t)cr - 128;
    ChromaTerms t;
    t.r = (int32_t)mul24(crr, 4 * 22970);
    t.g = (int32_t)mad24(cbb, -4 * 5638, mul24(crr, -4 * 11700));
    t.b = (int32_t)mul24(cbb, 4 * 29032);
    return t;
}
// Y sample of byte i of a packed word, shifted to bits [23:16].
template <int I>
__device__ __forceinline__ int32_t y16(uint32_t yq) {
    // selector bytes: 0x0c = zero; byte I of yq goes to byte 2
    return (int32_t)__builtin_amdgcn_perm(0u, yq, 0x0c000c0cu | ((uint32_t)I << 16));
}
__device__ __forceinline__ uint32_t bgra16(int32_t yy, const ChromaTerms& t) {
    // rgb_pixel_t {blue, green, red, alpha = 0} (mjpeg423_types.h:56-61, ycbcr_to_rgb.c:41)
    return ashr_pk_u8_hi<16>(ashr_pk_u8<16>(yy + t.b, yy + t.g), yy + t.r, -1);
}
__device__ __forceinline__ uint32_t bgra(uint32_t y, const ChromaTerms& t) { return bgra16((int32_t)(y << 16), t); }

// 4:4:4 form (no chroma sample is shared, so nothing is gained by precomputing chroma
// terms): the Q14 sums of ycbcr_to_rgb.c:34-44 as int16-pair dot products on
// {Y, C} pairs built with one v_perm each, the -128 offsets folded into the accumulator:
//   B = 16384 Y + 29032 Cb - 29032*128        R = 16384 Y + 22970 Cr - 22970*128
//   G = 16384 Y -  5638 Cb - 11700 Cr + (5638 + 11700)*128
// All |sums| < 2^23; NORMALIZE_RGB = sat_u8(v >> 14) (one v_ashr_pk_u8_i32 per two channels).
struct CscConst444 {
    uint32_t cb, cg, cr;  // accumulator constants, in VGPRs (one SGPR operand per VALU op)
};
__device__ __forceinline__ CscConst444 csc444_consts() {
    CscConst444 k;
    k.cb = (uint32_t)(-29032 * 128);
    k.cg = (uint32_t)((5638 + 11700) * 128);
    k.cr = (uint32_t)(-22970 * 128);
    asm volatile("" : "+v"(k.cb), "+v"(k.cg), "+v"(k.cr));  // materialise once, outside the loops
    return k;
}
// Pixel I of packed bytes yq / cb4 / cr4.
template <int I>
__device__ __forceinline__ uint32_t bgra444(uint32_t yq, uint32_t cb4, uint32_t cr4, const CscConst444& k) {
    constexpr uint32_t sel = (uint32_t)I | 0x0c00u | ((uint32_t)(4 + I) << 16) | 0x0c000000u;  // {Y_I, 0, C_I, 0}
    const uint32_t ycb = __builtin_amdgcn_perm(cb4, yq, sel);
    const uint32_t ycr = __builtin_amdgcn_perm(cr4, yq, sel);
    const int32_t b = (int32_t)dot2s(sconst<k2(16384, 29032)>(), ycb, k.cb);
    const int32_t g = (int32_t)dot2s(sconst<k2(0, -11700)>(), ycr, dot2s(sconst<k2(16384, -5638)>(), ycb, k.cg));
    const int32_t r = (int32_t)dot2s(sconst<k2(16384, 22970)>(), ycr, k.cr);
    return ashr_pk_u8_hi<14>(ashr_pk_u8<14>(b, g), r, -1);
}

// 4:2:2 / 4:2:0 form (a chroma sample shared by 2 or 4 pixels).  ycbcr_to_rgb.c:32-45 takes
// sat_u8(((Y << 14) + k * C') >> 14) per channel; Y << 14 is a multiple of 2^14, so that is
// exactly sat_u8(Y + (k * C' >> 14)): the chroma part of each channel is one small integer
// per chroma SAMPLE --
//   Tb = 29032 Cbb >> 14,  Tg = (-5638 Cbb - 11700 Crr) >> 14,  Tr = 22970 Crr >> 14
// (|T| <= 226, Cbb = Cb - 128, Crr = Cr - 128).  Per pixel, Y + T runs in int16 lanes
// (v_pk_add_u16 wraps mod 2^16, i.e. int16 arithmetic; |Y + T| < 2^15) and
// v_sat_pk_u8_i16 is NORMALIZE_RGB for two channels at once.
struct ChromaT {
    uint32_t bg;  // {Tb, Tg} as an int16 pair
    uint32_t r;   // Tr in the low half
};
// pa = {Cb, Cr} of one sample as a 16-bit pair; the -128 offsets ride in the accumulators.
__device__ __forceinline__ ChromaT chroma_t(uint32_t pa, const CscConst444& k) {
    const int32_t tb = (int32_t)dot2s(sconst<k2(29032, 0)>(), pa, k.cb) >> 14;
    const int32_t tg = (int32_t)dot2s(sconst<k2(-5638, -11700)>(), pa, k.cg) >> 14;
    const int32_t tr = (int32_t)dot2s(sconst<k2(0, 22970)>(), pa, k.cr) >> 14;
    return ChromaT{__builtin_amdgcn_perm((uint32_t)tg, (uint32_t)tb, 0x05040100u), (uint32_t)tr};
}
__device__ __forceinline__ uint32_t sat_pk_u8(uint32_t v) {  // {sat_u8(v.lo16), sat_u8(v.hi16)} in bits 0..15
    uint32_t r;
    asm("v_sat_pk_u8_i16 %0, %1" : "=v"(r) : "v"(v));
    return r;
}
// Two horizontally adjacent pixels sharing one chroma sample: y01 = {Y0, Y1} as 16-bit lanes.
__device__ __forceinline__ void bgra_pair(uint32_t y01, const ChromaT& t, uint32_t& px0, uint32_t& px1) {
    uint32_t bg0, bg1, rr;
    asm("v_pk_add_u16 %0, %1, %2 op_sel:[0,0] op_sel_hi:[0,1]" : "=v"(bg0) : "v"(y01), "v"(t.bg));  // {Y0+Tb, Y0+Tg}
    asm("v_pk_add_u16 %0, %1, %2 op_sel:[1,0] op_sel_hi:[1,1]" : "=v"(bg1) : "v"(y01), "v"(t.bg));  // {Y1+Tb, Y1+Tg}
    asm("v_pk_add_u16 %0, %1, %2 op_sel:[0,0] op_sel_hi:[1,0]" : "=v"(rr) : "v"(y01), "v"(t.r));    // {Y0+Tr, Y1+Tr}
    const uint32_t rs = sat_pk_u8(rr);
    px0 = __builtin_amdgcn_perm(rs, sat_pk_u8(bg0), 0x0c040100u);  // {B0, G0, R0, 0}
    px1 = __builtin_amdgcn_perm(rs, sat_pk_u8(bg1), 0x0c050100u);  // {B1, G1, R1, 0}
}

}  // namespace mj423
