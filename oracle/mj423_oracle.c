/*
 * mj423_oracle.c -- TEST INFRASTRUCTURE ONLY: the CPU restatement used as the
 * checker for the HIP product (see mj423_oracle.h for the pinning story).
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg load it.
 *
 * Written from the reference's behaviour, not its text.  Arithmetic is done in
 * uint32_t so that the int32 wrap-around the reference relies on
 * is defined behaviour here; right shifts are arithmetic on the int32 view.
 * Reference paths are relative to core0/software/common/libs/mjpeg423/.
 */
#include "mj423_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- tables */
/* common/tables.c:13-21 (JPEG Annex K.1) */
const int16_t orc_yquant[64] = {
    16, 11, 10, 16, 24, 40, 51, 61,     12, 12, 14, 19, 26, 58, 60, 55,
    14, 13, 16, 24, 40, 57, 69, 56,     14, 17, 22, 29, 51, 87, 80, 62,
    18, 22, 37, 56, 68, 109, 103, 77,   24, 35, 55, 64, 81, 104, 113, 92,
    49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
/* common/tables.c:24-32 (JPEG Annex K.2) */
const int16_t orc_cquant[64] = {
    17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
    24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
    99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};
/* common/tables.c:35-42: zig-zag scan position -> natural index */
const int32_t orc_zigzag[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

/* ------------------------------------------------------------------ IDCT */
/* common/dct_math.h:50-64: CONST_BITS = 13, PASS1_BITS = 2, FIX(c) = round(c * 2^13). */
enum {
    K0298 = 2446, K0390 = 3196, K0541 = 4433, K0765 = 6270, K0899 = 7373, K1175 = 9633,
    K1501 = 12299, K1847 = 15137, K1961 = 16069, K2053 = 16819, K2562 = 20995, K3072 = 25172
};

/*
 * The 8-point LLM butterfly shared by both passes of decoder/idct.c (pass 1:
 * :46-94, pass 2: :121-167): x[k] is the k-th frequency sample, y[n] the
 * undescaled n-th output.  Every operation is a ring operation mod 2^32, so
 * this equals the reference's int32 evaluation bit for bit, wrap included.
 */
static inline void orc_butterfly8(const uint32_t x[8], uint32_t y[8])
{
    /* even part: rotator sqrt(2)*c6 on (x2, x6), DC/x4 sum/difference scaled by 2^13 */
    uint32_t r = (x[2] + x[6]) * (uint32_t)K0541;
    uint32_t e2 = r - x[6] * (uint32_t)K1847;
    uint32_t e3 = r + x[2] * (uint32_t)K0765;
    uint32_t e0 = (x[0] + x[4]) << 13;
    uint32_t e1 = (x[0] - x[4]) << 13;
    uint32_t s0 = e0 + e3, s3 = e0 - e3, s1 = e1 + e2, s2 = e1 - e2;

    /* odd part (figure 8 of the LLM paper): inputs x7, x5, x3, x1 */
    uint32_t a = x[7] + x[1], b = x[5] + x[3], c = x[7] + x[3], d = x[5] + x[1];
    uint32_t z5 = (c + d) * (uint32_t)K1175;
    uint32_t pa = 0u - a * (uint32_t)K0899;
    uint32_t pb = 0u - b * (uint32_t)K2562;
    uint32_t pc = z5 - c * (uint32_t)K1961;
    uint32_t pd = z5 - d * (uint32_t)K0390;
    uint32_t o7 = x[7] * (uint32_t)K0298 + pa + pc;
    uint32_t o5 = x[5] * (uint32_t)K2053 + pb + pd;
    uint32_t o3 = x[3] * (uint32_t)K3072 + pb + pc;
    uint32_t o1 = x[1] * (uint32_t)K1501 + pa + pd;

    y[0] = s0 + o1; y[7] = s0 - o1;
    y[1] = s1 + o3; y[6] = s1 - o3;
    y[2] = s2 + o5; y[5] = s2 - o5;
    y[3] = s3 + o7; y[4] = s3 - o7;
}

/* DESCALE(x, n) of dct_math.h:48: add 2^(n-1) (wrapping), arithmetic shift by n. */
static inline int32_t orc_descale(uint32_t v, int n)
{
    return (int32_t)(v + (1u << (n - 1))) >> n;
}

void orc_idct_block(const int16_t in[64], uint8_t out[64])
{
    int32_t ws[64];
    uint32_t x[8], y[8];
    /* pass 1: columns -> workspace scaled by 2^PASS1_BITS (idct.c:39-109) */
    for (int c = 0; c < 8; c++) {
        for (int k = 0; k < 8; k++) x[k] = (uint32_t)(int32_t)in[8 * k + c];
        orc_butterfly8(x, y);
        for (int n = 0; n < 8; n++) ws[8 * n + c] = orc_descale(y[n], 13 - 2);
    }
    /* pass 2: rows -> descale by 2^(13+2+3), clamp to [0,255] (idct.c:115-180, NORMALIZE :20) */
    for (int r = 0; r < 8; r++) {
        for (int k = 0; k < 8; k++) x[k] = (uint32_t)ws[8 * r + k];
        orc_butterfly8(x, y);
        for (int n = 0; n < 8; n++) {
            int32_t v = orc_descale(y[n], 13 + 2 + 3);
            out[8 * r + n] = (uint8_t)(v < 0 ? 0 : (v > 255 ? 255 : v));
        }
    }
}

void orc_idct_blocks(size_t n, const int16_t *in, uint8_t *out)
{
    for (size_t b = 0; b < n; b++) orc_idct_block(in + 64 * b, out + 64 * b);
}

/* ------------------------------------------------------------------- CSC */
/* decoder/ycbcr_to_rgb.c:32-44 with NORMALIZE_RGB (:19): negative -> 0, else >>14 capped at 255. */
static inline uint32_t orc_norm_rgb(int32_t v)
{
    if (v < 0) return 0;
    v >>= 14;
    return (uint32_t)(v > 255 ? 255 : v);
}

uint32_t orc_ycbcr_pixel(uint8_t y, uint8_t cb, uint8_t cr)
{
    int32_t cbb = (int32_t)cb - 128, crr = (int32_t)cr - 128, yy = (int32_t)y << 14;
    uint32_t red = orc_norm_rgb(yy + 22970 * crr);
    uint32_t green = orc_norm_rgb(yy - 5638 * cbb - 11700 * crr);
    uint32_t blue = orc_norm_rgb(yy + 29032 * cbb);
    return blue | (green << 8) | (red << 16); /* rgb_pixel_t {b,g,r,a=0}, types.h:56-61 */
}

void orc_ycbcr_to_rgb_block(int h, int w, uint32_t w_size, const uint8_t Y[64],
                            const uint8_t Cb[64], const uint8_t Cr[64], uint32_t *rgb)
{
    for (int y = 0; y < 8; y++) {
        uint32_t *row = rgb + (size_t)(h + y) * w_size + (size_t)w;
        for (int x = 0; x < 8; x++) row[x] = orc_ycbcr_pixel(Y[8 * y + x], Cb[8 * y + x], Cr[8 * y + x]);
    }
}

/* --------------------------------------------------------------- dequant */
void orc_dequant_blocks(size_t n, const int16_t *Q, const int16_t q[64], int16_t *out)
{
    for (size_t i = 0; i < 64 * n; i++) out[i] = (int16_t)(int32_t)((int32_t)Q[i] * (int32_t)q[i & 63]);
}

/* --------------------------------------------------------------- geometry */
int orc_geometry(uint32_t width, uint32_t height, int chroma, orc_geom_t *g)
{
    uint32_t sx, sy;
    if (!g || width == 0 || height == 0) return -1;
    switch (chroma) {
    case ORC_CHROMA_444: sx = 1; sy = 1; break;
    case ORC_CHROMA_422: sx = 2; sy = 1; break;
    case ORC_CHROMA_420: sx = 2; sy = 2; break;
    default: return -1;
    }
    g->width = width;
    g->height = height;
    g->chroma = chroma;
    g->mcu_w = 8 * sx;
    g->mcu_h = 8 * sy;
    g->coded_w = (width + g->mcu_w - 1) / g->mcu_w * g->mcu_w;
    g->coded_h = (height + g->mcu_h - 1) / g->mcu_h * g->mcu_h;
    g->y_bw = g->coded_w / 8;
    g->y_bh = g->coded_h / 8;
    g->c_bw = g->y_bw / sx;
    g->c_bh = g->y_bh / sy;
    g->y_blocks = g->y_bw * g->y_bh;
    g->c_blocks = g->c_bw * g->c_bh;
    return 0;
}

/* ------------------------------------------------------------------ frame */
static void orc_plane_to_pixels(size_t nblocks, const int16_t *Q, const int16_t *q, int flags,
                                uint8_t *pix, int16_t *tmp)
{
    for (size_t b = 0; b < nblocks; b++) {
        const int16_t *src = Q + 64 * b;
        if (flags != ORC_INPUT_DEQUANTIZED) {
            orc_dequant_blocks(1, src, q, tmp);
            src = tmp;
        }
        orc_idct_block(src, pix + 64 * b);
    }
}

static int orc_decode_frame_scratch(const orc_geom_t *g, const int16_t *Yq, const int16_t *Cbq,
                                    const int16_t *Crq, const int16_t *yquant, const int16_t *cquant,
                                    int flags, uint32_t *out, uint32_t out_pitch, uint8_t *scratch)
{
    uint8_t *Yp = scratch, *Cbp = Yp + 64 * (size_t)g->y_blocks, *Crp = Cbp + 64 * (size_t)g->c_blocks;
    int16_t tmp[64];
    uint32_t sx = g->mcu_w / 8, sy = g->mcu_h / 8;
    if (!yquant) yquant = orc_yquant;
    if (!cquant) cquant = orc_cquant;
    /* HOT LOOP 1, decoder/mjpeg423_decoder.c:115-117 (dequant folded in, A5) */
    orc_plane_to_pixels(g->y_blocks, Yq, yquant, flags, Yp, tmp);
    orc_plane_to_pixels(g->c_blocks, Cbq, cquant, flags, Cbp, tmp);
    orc_plane_to_pixels(g->c_blocks, Crq, cquant, flags, Crp, tmp);
    /* HOT LOOP 2, decoder/mjpeg423_decoder.c:120-124, block by block like the reference
     * (ycbcr_to_rgb per 8x8 luma block); chroma fetch (x/sx, y/sy) per SURVEY §8 A7.
     * For 4:4:4 this visits exactly the pixels ycbcr_to_rgb() writes, with the same values. */
    const uint32_t lx = sx == 2, ly = sy == 2;
    for (uint32_t by = 0; by < g->y_bh && 8 * by < g->height; by++) {
        const uint32_t rows = g->height - 8 * by < 8 ? g->height - 8 * by : 8;
        for (uint32_t bx = 0; bx < g->y_bw && 8 * bx < g->width; bx++) {
            const uint32_t cols = g->width - 8 * bx < 8 ? g->width - 8 * bx : 8;
            const uint8_t *yb = Yp + ((size_t)by * g->y_bw + bx) * 64;
            for (uint32_t r = 0; r < rows; r++) {
                const uint32_t y = 8 * by + r, cy = y >> ly;
                const size_t crow = ((size_t)(cy >> 3) * g->c_bw) * 64 + (cy & 7) * 8;
                uint32_t *dst = out + (size_t)y * out_pitch + 8 * bx;
                for (uint32_t c = 0; c < cols; c++) {
                    const uint32_t cx = (8 * bx + c) >> lx;
                    const size_t ci = crow + (size_t)(cx >> 3) * 64 + (cx & 7);
                    dst[c] = orc_ycbcr_pixel(yb[8 * r + c], Cbp[ci], Crp[ci]);
                }
            }
        }
    }
    return 0;
}

int orc_decode_frame(uint32_t width, uint32_t height, int chroma, const int16_t *Yq,
                     const int16_t *Cbq, const int16_t *Crq, const int16_t *yquant,
                     const int16_t *cquant, int flags, uint32_t *out, uint32_t out_pitch)
{
    orc_geom_t g;
    if (orc_geometry(width, height, chroma, &g) || out_pitch < width) return -1;
    uint8_t *scratch = (uint8_t *)malloc(64 * ((size_t)g.y_blocks + 2 * (size_t)g.c_blocks));
    if (!scratch) return -1;
    int rc = orc_decode_frame_scratch(&g, Yq, Cbq, Crq, yquant, cquant, flags, out, out_pitch, scratch);
    free(scratch);
    return rc;
}

typedef struct {
    const orc_geom_t *g;
    const int16_t *coef;
    const int16_t *yq, *cq;
    uint32_t *out;
    uint32_t nframes;
    int flags, tid, nthreads;
} orc_mt_job;

static void *orc_mt_worker(void *arg)
{
    orc_mt_job *j = (orc_mt_job *)arg;
    const orc_geom_t *g = j->g;
    size_t fstride = 64 * ((size_t)g->y_blocks + 2 * (size_t)g->c_blocks);
    uint8_t *scratch = (uint8_t *)malloc(fstride);
    if (!scratch) return (void *)1;
    for (uint32_t f = (uint32_t)j->tid; f < j->nframes; f += (uint32_t)j->nthreads) {
        const int16_t *Y = j->coef + f * fstride;
        const int16_t *Cb = Y + 64 * (size_t)g->y_blocks;
        const int16_t *Cr = Cb + 64 * (size_t)g->c_blocks;
        orc_decode_frame_scratch(g, Y, Cb, Cr, j->yq, j->cq, j->flags,
                                 j->out + (size_t)f * g->width * g->height, g->width, scratch);
    }
    free(scratch);
    return NULL;
}

int orc_decode_frames_mt(uint32_t width, uint32_t height, int chroma, const int16_t *coef,
                         uint32_t nframes, const int16_t *yquant, const int16_t *cquant, int flags,
                         uint32_t *out, int nthreads)
{
    orc_geom_t g;
    if (orc_geometry(width, height, chroma, &g) || nthreads < 1) return -1;
    if (nthreads > 256) nthreads = 256;
    pthread_t th[256];
    orc_mt_job jobs[256];
    int rc = 0;
    for (int t = 0; t < nthreads; t++) {
        jobs[t] = (orc_mt_job){&g, coef, yquant, cquant, out, nframes, flags, t, nthreads};
        if (nthreads == 1) return orc_mt_worker(&jobs[0]) ? -1 : 0;
        if (pthread_create(&th[t], NULL, orc_mt_worker, &jobs[t])) return -1;
    }
    for (int t = 0; t < nthreads; t++) {
        void *ret = NULL;
        pthread_join(th[t], &ret);
        if (ret) rc = -1;
    }
    return rc;
}

/* ------------------------------------------------------------------ hashes */
uint64_t orc_fnv1a64(uint64_t h, const void *p, size_t n)
{
    const uint8_t *b = (const uint8_t *)p;
    for (size_t i = 0; i < n; i++) {
        h ^= b[i];
        h *= 0x100000001b3ULL;
    }
    return h;
}

uint64_t orc_csc_exhaustive_hash(void)
{
    uint64_t h = 0xcbf29ce484222325ULL;
    uint32_t px[64];
    for (uint32_t base = 0; base < (1u << 24); base += 64) {
        for (uint32_t i = 0; i < 64; i++) {
            uint32_t idx = base + i;
            px[i] = orc_ycbcr_pixel((uint8_t)(idx >> 16), (uint8_t)(idx >> 8), (uint8_t)idx);
        }
        h = orc_fnv1a64(h, px, sizeof(px));
    }
    return h;
}

/* ------------------------------------------------------- entropy front end */
/* MSB-first bit reader equivalent to update_buffer() (lossless_decode.c:139-162):
 * bytes are pulled in only when a peek needs them, so it never reads further
 * ahead than the reference's 32-bit window does. */
typedef struct {
    const uint8_t *p;
    uint64_t acc;  /* valid bits left-aligned at bit 63 */
    int nbits;
    size_t pos;    /* bits consumed */
} orc_bits;

static inline uint32_t orc_peek(orc_bits *b, int n)
{
    while (b->nbits < n) {
        b->acc |= (uint64_t)(*b->p++) << (56 - b->nbits);
        b->nbits += 8;
    }
    return (uint32_t)(b->acc >> (64 - n));
}

static inline void orc_skip(orc_bits *b, int n)
{
    b->acc <<= n;
    b->nbits -= n;
    b->pos += (size_t)n;
}

/* HUFF_EXTEND (lossless_decode.c:204): VLI amplitude of `size` bits -> signed value. */
static inline int32_t orc_vli(uint32_t v, int size)
{
    return v < (1u << (size - 1)) ? (int32_t)v - (int32_t)(1u << size) + 1 : (int32_t)v;
}

/* Decodes one symbol: DC = SIZE(4) + VLI (input_DC :210-224); AC = RUN(4) SIZE(4) + VLI
 * (input_AC :227-246). */
static inline int32_t orc_symbol(orc_bits *b, int ac, int *run)
{
    *run = 0;
    if (ac) {
        *run = (int)orc_peek(b, 4);
        orc_skip(b, 4);
    }
    int size = (int)orc_peek(b, 4);
    orc_skip(b, 4);
    if (size == 0) return 0;
    int32_t e = orc_vli(orc_peek(b, size), size);
    orc_skip(b, size);
    return e;
}

/* Shared walk of lossless_decode.c:82-134.  mode 0: reference (dequantizing)
 * semantics; mode 1: quantized-domain semantics. */
static size_t orc_lossless_walk(int num_blocks, const void *bitstream, int16_t *dst,
                                const int16_t *quant, int P, int mode)
{
    orc_bits b = {(const uint8_t *)bitstream, 0, 0, 0};
    int16_t cur = 0;
    int run;
    if (!P) memset(dst, 0, (size_t)num_blocks * 64 * sizeof(int16_t)); /* :77-78 */
    for (int blk = 0; blk < num_blocks; blk++) {
        int16_t *pe = dst + 64 * (size_t)blk;
        int32_t e = orc_symbol(&b, 0, &run);
        if (P) /* :90-92 */
            pe[0] = (int16_t)(pe[0] + (mode ? e : e * quant[0]));
        else { /* :93-96 running DC sum kept in int16 */
            cur = (int16_t)(cur + e);
            pe[0] = (int16_t)(mode ? cur : cur * quant[0]);
        }
        for (int index = 1;;) {
            e = orc_symbol(&b, 1, &run);
            if (e == 0) {
                if (run == 15) { /* ZRL: 16 zeros (:107-110) */
                    index += 16;
                    continue;
                }
                break; /* EOB (:111-114) */
            }
            index += run;
            /* A malformed stream can push index past 63; the reference then reads
             * zigzag_table out of bounds (UB).  Skip the write, keep the bit walk. */
            if (index <= 63) {
                int k = orc_zigzag[index];
                int32_t v = mode ? e : e * quant[k];
                pe[k] = (int16_t)(P ? pe[k] + v : v); /* :121-126 */
            }
            if (index >= 63) break;
            index++;
        }
    }
    return (b.pos + 7) / 8;
}

size_t orc_lossless_decode_ref(int num_blocks, const void *bitstream, int16_t *dcac,
                               const int16_t quant[64], int P)
{
    return orc_lossless_walk(num_blocks, bitstream, dcac, quant, P, 0);
}

size_t orc_lossless_decode_q(int num_blocks, const void *bitstream, int16_t *q_abs, int P)
{
    return orc_lossless_walk(num_blocks, bitstream, q_abs, NULL, P, 1);
}
