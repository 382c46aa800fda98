/*
 * ref_harness.c -- TEST INFRASTRUCTURE ONLY (never shipped, never measured as the product).
 *
 * Batch entry points around the *unmodified* reference C sources, which
 * oracle/Makefile.ref compiles straight from /root/reference into
 * oracle/_ref/libmjref.so.  Nothing here re-implements the reference: every
 * function below just loops over the reference's own symbols so that
 * oracle/gen_golden.py can drive them through ctypes without one FFI call per
 * 8x8 block.
 *
 * Reference symbols used (paths relative to core0/software/common/libs/mjpeg423/):
 *   idct()          decoder/idct.c:22
 *   ycbcr_to_rgb()  decoder/ycbcr_to_rgb.c:26
 *   lossless_decode decoder/lossless_decode.c:60   (exported directly, called from Python, and
 *                   inside ref_decode_mpg_frames)
 *   rgb_to_ycbcr()  encoder/rgb_to_ycbcr.c:58
 *   fdct()          encoder/fdct.c:17
 *   quantize_I/P()  encoder/quantize.c:18,33
 *   lossless_encode encoder/lossless_encode.c:30
 *   Yquant/Cquant/zigzag_table  common/tables.c:13,24,35
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "decoder/mjpeg423_decoder.h"
#include "encoder/mjpeg423_encoder.h"

/* HOT LOOP 1 of mjpeg423_decoder.c:115-117 for one plane. */
void ref_idct_batch(int n, const int16_t *in, uint8_t *out)
{
    for (int b = 0; b < n; b++)
        idct((pdct_block_t)(in + 64 * b), (pcolor_block_t)(out + 64 * b));
}

/* HOT LOOP 2 of mjpeg423_decoder.c:120-124 (4:4:4, block-raster planes). */
void ref_csc_frame(uint32_t w_size, uint32_t h_size, const uint8_t *Y, const uint8_t *Cb,
                   const uint8_t *Cr, rgb_pixel_t *rgb)
{
    int hb = (int)h_size / 8, wb = (int)w_size / 8;
    for (int h = 0; h < hb; h++)
        for (int w = 0; w < wb; w++) {
            int b = h * wb + w;
            ycbcr_to_rgb(h << 3, w << 3, w_size, (pcolor_block_t)(Y + 64 * b),
                         (pcolor_block_t)(Cb + 64 * b), (pcolor_block_t)(Cr + 64 * b), rgb);
        }
}

/* The per-frame body mjpeg423_decoder.c:114-124 on already-dequantized planes
 * (what lossless_decode leaves in YDCAC/CbDCAC/CrDCAC). scratch = 3*nb*64 bytes. */
void ref_decode_frame_444(uint32_t w_size, uint32_t h_size, const int16_t *Ydcac,
                          const int16_t *Cbdcac, const int16_t *Crdcac, uint8_t *scratch,
                          rgb_pixel_t *rgb)
{
    int nb = (int)(w_size / 8) * (int)(h_size / 8);
    uint8_t *Yb = scratch, *Cbb = scratch + 64 * nb, *Crb = scratch + 128 * nb;
    ref_idct_batch(nb, Ydcac, Yb);
    ref_idct_batch(nb, Cbdcac, Cbb);
    ref_idct_batch(nb, Crdcac, Crb);
    ref_csc_frame(w_size, h_size, Yb, Cbb, Crb, rgb);
}

/* The same frame body for 4:2:2 / 4:2:0 planes (coded size, whole MCUs): the reference's
 * idct() over every block of the three planes, then the reference's ycbcr_to_rgb() per
 * 8x8 luma block with the chroma blocks it needs gathered by nearest-neighbour
 * replication (pixel (x, y) <- chroma (x/2, y/sy)).  Only that gather is
 * harness code; every arithmetic operation is the reference's.  chroma 444 reduces to
 * ref_decode_frame_444.  scratch = 64 * (Yblocks + 2 * Cblocks) bytes; rgb is coded-size. */
void ref_decode_frame_sub(uint32_t w_size, uint32_t h_size, int chroma, const int16_t *Ydcac,
                          const int16_t *Cbdcac, const int16_t *Crdcac, uint8_t *scratch,
                          rgb_pixel_t *rgb)
{
    const int sx = chroma == 444 ? 1 : 2, sy = chroma == 420 ? 2 : 1;
    const int ybw = (int)w_size / 8, ybh = (int)h_size / 8, cbw = ybw / sx, cbh = ybh / sy;
    const int ny = ybw * ybh, nc = cbw * cbh;
    uint8_t *Yb = scratch, *Cbb = scratch + 64 * ny, *Crb = Cbb + 64 * nc;
    ref_idct_batch(ny, Ydcac, Yb);
    ref_idct_batch(nc, Cbdcac, Cbb);
    ref_idct_batch(nc, Crdcac, Crb);
    color_block_t cb8, cr8;
    for (int by = 0; by < ybh; by++)
        for (int bx = 0; bx < ybw; bx++) {
            const int cblk = (by / sy) * cbw + bx / sx;
            const uint8_t *cbs = Cbb + 64 * cblk, *crs = Crb + 64 * cblk;
            const int ox = sx == 2 ? (bx % 2) * 4 : 0, oy = sy == 2 ? (by % 2) * 4 : 0;
            for (int y = 0; y < 8; y++)
                for (int x = 0; x < 8; x++) {
                    const int k = (oy + y / sy) * 8 + ox + x / sx;
                    cb8[y][x] = cbs[k];
                    cr8[y][x] = crs[k];
                }
            ycbcr_to_rgb(by << 3, bx << 3, w_size, (pcolor_block_t)(Yb + 64 * (by * ybw + bx)), cb8, cr8, rgb);
        }
}

static uint64_t fnv1a(uint64_t h, const uint8_t *p, size_t n)
{
    for (size_t i = 0; i < n; i++) {
        h ^= p[i];
        h *= 0x100000001b3ULL;
    }
    return h;
}

/* FNV-1a over ycbcr_to_rgb() for all 2^24 (Y,Cb,Cr) triples, enumerated
 * as idx = (Y<<16)|(Cb<<8)|Cr, 64 triples per reference call, BGRA bytes hashed
 * in idx order. */
uint64_t ref_csc_exhaustive_hash(void)
{
    uint64_t h = 0xcbf29ce484222325ULL;
    color_block_t Y, Cb, Cr;
    rgb_pixel_t out[64];
    for (uint32_t base = 0; base < (1u << 24); base += 64) {
        for (int i = 0; i < 64; i++) {
            uint32_t idx = base + (uint32_t)i;
            Y[i >> 3][i & 7] = (uint8_t)(idx >> 16);
            Cb[i >> 3][i & 7] = (uint8_t)(idx >> 8);
            Cr[i >> 3][i & 7] = (uint8_t)idx;
        }
        ycbcr_to_rgb(0, 0, 8, Y, Cb, Cr, out);
        h = fnv1a(h, (const uint8_t *)out, sizeof(out));
    }
    return h;
}

/* Encoder front half for realistic coefficient statistics: one 4:4:4 I-frame.
 * rgb: w*h BGRA. Writes absolute quantized coefficients (quantize_I's
 * DCACq_next) and the differential ones lossless_encode consumes, per plane. */
void ref_encode_iframe(uint32_t w_size, uint32_t h_size, rgb_pixel_t *rgb, int16_t *Yq_abs,
                       int16_t *Cbq_abs, int16_t *Crq_abs, int16_t *Yq_diff, int16_t *Cbq_diff,
                       int16_t *Crq_diff)
{
    int hb = (int)h_size / 8, wb = (int)w_size / 8;
    color_block_t Y, Cb, Cr;
    dct_block_t dY, dCb, dCr;
    DCTELEM pY = 0, pCb = 0, pCr = 0;
    for (int h = 0; h < hb; h++)
        for (int w = 0; w < wb; w++) {
            int b = h * wb + w;
            rgb_to_ycbcr(h << 3, w << 3, w_size, rgb, Y, Cb, Cr);
            fdct(Y, dY);
            fdct(Cb, dCb);
            fdct(Cr, dCr);
            quantize_I(&pY, Yquant, dY, (pdct_block_t)(Yq_diff + 64 * b), (pdct_block_t)(Yq_abs + 64 * b));
            quantize_I(&pCb, Cquant, dCb, (pdct_block_t)(Cbq_diff + 64 * b), (pdct_block_t)(Cbq_abs + 64 * b));
            quantize_I(&pCr, Cquant, dCr, (pdct_block_t)(Crq_diff + 64 * b), (pdct_block_t)(Crq_abs + 64 * b));
        }
}

/* P-frame quantization (encoder/quantize.c:33): prev_abs is updated in place
 * to the new absolute coefficients, diff receives the deltas. */
void ref_encode_pframe(uint32_t w_size, uint32_t h_size, rgb_pixel_t *rgb, int16_t *Yprev,
                       int16_t *Cbprev, int16_t *Crprev, int16_t *Yq_diff, int16_t *Cbq_diff,
                       int16_t *Crq_diff)
{
    int hb = (int)h_size / 8, wb = (int)w_size / 8;
    color_block_t Y, Cb, Cr;
    dct_block_t dY, dCb, dCr;
    for (int h = 0; h < hb; h++)
        for (int w = 0; w < wb; w++) {
            int b = h * wb + w;
            rgb_to_ycbcr(h << 3, w << 3, w_size, rgb, Y, Cb, Cr);
            fdct(Y, dY);
            fdct(Cb, dCb);
            fdct(Cr, dCr);
            quantize_P(Yquant, (pdct_block_t)(Yprev + 64 * b), dY, (pdct_block_t)(Yq_diff + 64 * b));
            quantize_P(Cquant, (pdct_block_t)(Cbprev + 64 * b), dCb, (pdct_block_t)(Cbq_diff + 64 * b));
            quantize_P(Cquant, (pdct_block_t)(Crprev + 64 * b), dCr, (pdct_block_t)(Crq_diff + 64 * b));
        }
}

/* The reference decoder's frame loop, mjpeg423_decoder.c:90-124, over frames [f0, f1) of an .mpg
 * already in memory (`file`, the file's bytes; frame f's header at byte frame_pos[f]): per frame the
 * frame header and payload are read as the loop's two freads read them (:94-103; here a memcpy of the
 * same bytes into the same buffer), then the reference's own lossless_decode() of the three planes
 * (dequantizing; a P-frame accumulates into the previous frame's DCAC planes, :109-111), idct() over
 * every block (:114-117) and ycbcr_to_rgb() over the block grid (:120-124).  Only the BMP write
 * (:126-132) is left out.  Buffers are allocated as the reference allocates them (:54-72).  f0 must be
 * an I-frame (a GOP start: frames are not independent inside a GOP).  rgb_last (w_size * h_size
 * pixels, may be NULL) receives the last frame's pixels.  Returns the frames decoded, -1 on a frame
 * header the buffers cannot hold, -2 on an allocation failure. */
int ref_decode_mpg_frames(const uint8_t *file, const uint64_t *frame_pos, uint32_t f0, uint32_t f1,
                          uint32_t w_size, uint32_t h_size, rgb_pixel_t *rgb_last)
{
    const int hCb = (int)h_size / 8, wCb = (int)w_size / 8, hYb = (int)h_size / 8, wYb = (int)w_size / 8;
    const size_t stream_cap = (size_t)hYb * wYb * 64 * sizeof(DCTELEM) + 2 * (size_t)hCb * wCb * 64 * sizeof(DCTELEM);
    rgb_pixel_t *rgbblock = malloc((size_t)w_size * h_size * sizeof(rgb_pixel_t));
    color_block_t *Yblock = malloc((size_t)hYb * wYb * 64), *Cbblock = malloc((size_t)hCb * wCb * 64),
                  *Crblock = malloc((size_t)hCb * wCb * 64);
    dct_block_t *YDCAC = malloc((size_t)hYb * wYb * 64 * sizeof(DCTELEM)),
                *CbDCAC = malloc((size_t)hCb * wCb * 64 * sizeof(DCTELEM)),
                *CrDCAC = malloc((size_t)hCb * wCb * 64 * sizeof(DCTELEM));
    uint8_t *Ybitstream = malloc(stream_cap);
    int done = 0;
    if (!rgbblock || !Yblock || !Cbblock || !Crblock || !YDCAC || !CbDCAC || !CrDCAC || !Ybitstream) {
        done = -2;
        goto out;
    }
    for (uint32_t f = f0; f < f1; f++) {
        uint32_t frame_header[4];
        memcpy(frame_header, file + frame_pos[f], sizeof frame_header);
        const uint32_t frame_size = frame_header[0], frame_type = frame_header[1], Ysize = frame_header[2],
                       Cbsize = frame_header[3];
        if (frame_size < 16 || frame_size - 16 > stream_cap) {
            done = -1;
            goto out;
        }
        memcpy(Ybitstream, file + frame_pos[f] + 16, frame_size - 16);
        uint8_t *Cbbitstream = Ybitstream + Ysize, *Crbitstream = Cbbitstream + Cbsize;
        lossless_decode(hYb * wYb, Ybitstream, YDCAC, Yquant, frame_type);
        lossless_decode(hCb * wCb, Cbbitstream, CbDCAC, Cquant, frame_type);
        lossless_decode(hCb * wCb, Crbitstream, CrDCAC, Cquant, frame_type);
        for (int b = 0; b < hYb * wYb; b++) idct(YDCAC[b], Yblock[b]);
        for (int b = 0; b < hCb * wCb; b++) idct(CbDCAC[b], Cbblock[b]);
        for (int b = 0; b < hCb * wCb; b++) idct(CrDCAC[b], Crblock[b]);
        for (int h = 0; h < hCb; h++)
            for (int w = 0; w < wCb; w++) {
                int b = h * wCb + w;
                ycbcr_to_rgb(h << 3, w << 3, w_size, Yblock[b], Cbblock[b], Crblock[b], rgbblock);
            }
        done++;
    }
    if (rgb_last && done > 0) memcpy(rgb_last, rgbblock, (size_t)w_size * h_size * sizeof(rgb_pixel_t));
out:
    free(rgbblock);
    free(Yblock);
    free(Cbblock);
    free(Crblock);
    free(YDCAC);
    free(CbDCAC);
    free(CrDCAC);
    free(Ybitstream);
    return done;
}

/* Copy the reference tables out (common/tables.c). */
void ref_tables(int16_t yq[64], int16_t cq[64], int32_t zz[64])
{
    memcpy(yq, Yquant, 128);
    memcpy(cq, Cquant, 128);
    memcpy(zz, zigzag_table, 256);
}
