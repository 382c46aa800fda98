/* tools/dropin_bench.c -- cost of the reference's per-block symbols idct() / ycbcr_to_rgb()
 * (mj/decoder/mjpeg423_decoder.h:15-16) as served by libmj423gpu.so: per call, and per
 * 640x480 4:4:4 frame through the reference's own call pattern (mjpeg423_decoder.c:114-124:
 * every block's idct(), then one ycbcr_to_rgb() per 8x8 block).  Measurement tool only.
 *   usage: dropin_bench [frames]     (GPU box; prints one JSON line)
 * Built twice by `make -C oracle dropin`: oracle/_ref/dropin_bench against libmj423gpu.so, and
 * oracle/_ref/dropin_bench_ref (-DREF_BUILD) against the reference's own idct.c and
 * ycbcr_to_rgb.c compiled in place -- the same calls, timed on the same host.  Each frame ends
 * where the reference's decoder writes its BMP (mjpeg423_decoder.c:132): the library's
 * encode_bmp() flushes the deferred mode there, so the frame time here includes a
 * mj423_dropin_flush() (no file is written). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

typedef int16_t dct_block_t[8][8];
typedef uint8_t color_block_t[8][8];
typedef color_block_t *pcolor_block_t;
typedef struct { uint8_t blue, green, red, alpha; } rgb_pixel_t;
void idct(dct_block_t DCAC, color_block_t block);
void ycbcr_to_rgb(int h, int w, uint32_t w_size, pcolor_block_t Y, pcolor_block_t Cb, pcolor_block_t Cr,
                  rgb_pixel_t *rgbblock);
#ifdef REF_BUILD
static const char *mj423_last_error(void) { return ""; }
static int mj423_dropin_flush(void) { return 0; }
#else
const char *mj423_last_error(void);
int mj423_dropin_flush(void);
#endif

static double now(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

int main(int argc, char **argv) {
    const int frames = argc > 1 ? atoi(argv[1]) : 3;
    const int W = 640, H = 480, nb = (W / 8) * (H / 8);
    dct_block_t *Y = malloc(sizeof(dct_block_t) * nb), *Cb = malloc(sizeof(dct_block_t) * nb),
                *Cr = malloc(sizeof(dct_block_t) * nb);
    color_block_t *Yb = malloc(sizeof(color_block_t) * nb), *Cbb = malloc(sizeof(color_block_t) * nb),
                  *Crb = malloc(sizeof(color_block_t) * nb);
    rgb_pixel_t *rgb = malloc(sizeof(rgb_pixel_t) * W * H);
    srand(7);
    for (int b = 0; b < nb; b++)
        for (int i = 0; i < 64; i++) {  /* dequantized DC + a few small ACs */
            int16_t v = (i == 0) ? (int16_t)(rand() % 2040) : (rand() % 5 == 0 ? (int16_t)(rand() % 61 - 30) : 0);
            Y[b][i / 8][i % 8] = v;
            Cb[b][i / 8][i % 8] = (int16_t)(v / 2);
            Cr[b][i / 8][i % 8] = (int16_t)(-v / 2);
        }
    idct(Y[0], Yb[0]);  /* warm-up: context creation, first launches */
    ycbcr_to_rgb(0, 0, W, &Yb[0], &Yb[0], &Yb[0], rgb);
    const int ncall = 2000;
    double t0 = now();
    for (int i = 0; i < ncall; i++) idct(Y[i % nb], Yb[i % nb]);
    mj423_dropin_flush();  /* a deferred batch is decoded here */
    const double idct_us = (now() - t0) / ncall * 1e6;
    t0 = now();
    for (int i = 0; i < ncall; i++) ycbcr_to_rgb(0, 0, W, &Yb[i % nb], &Yb[i % nb], &Yb[i % nb], rgb);
    mj423_dropin_flush();
    const double csc_us = (now() - t0) / ncall * 1e6;
    double best = 1e30, tot = 0;
    for (int f = 0; f < frames; f++) {
        t0 = now();
        for (int b = 0; b < nb; b++) idct(Y[b], Yb[b]);
        for (int b = 0; b < nb; b++) idct(Cb[b], Cbb[b]);
        for (int b = 0; b < nb; b++) idct(Cr[b], Crb[b]);
        for (int h = 0; h < H / 8; h++)
            for (int w = 0; w < W / 8; w++) {
                const int b = h * (W / 8) + w;
                ycbcr_to_rgb(h << 3, w << 3, W, &Yb[b], &Cbb[b], &Crb[b], rgb);
            }
        mj423_dropin_flush();  /* = the flush inside the library's encode_bmp() */
        const double dt = now() - t0;
        tot += dt;
        if (dt < best) best = dt;
    }
    unsigned long long sum = 0;
    for (int i = 0; i < W * H; i++) sum = sum * 31 + rgb[i].red + 7 * rgb[i].green + 13 * rgb[i].blue;
    const char *defer = getenv("MJ423_DROPIN_DEFER");
#ifdef REF_BUILD
    const char *impl = "reference C (idct.c + ycbcr_to_rgb.c, -O3, one host thread)";
#else
    const char *impl = "libmj423gpu.so";
#endif
    printf("{\"tool\": \"dropin_bench\", \"impl\": \"%s\", \"defer\": %s, \"idct_us_per_call\": %.3f, \"ycbcr_to_rgb_us_per_call\": %.3f, "
           "\"frame\": \"640x480 4:4:4 (%d idct + %d ycbcr_to_rgb calls)\", \"frame_ms_best\": %.3f, "
           "\"frame_ms_mean\": %.3f, \"frames\": %d, \"rgb_hash\": \"%016llx\", \"last_error\": \"%s\"}\n",
           impl,
#ifdef REF_BUILD
           "null",
#else
           defer && *defer ? (atoi(defer) ? "true" : "false") : "\"default (deferred)\"",
#endif
           idct_us, csc_us, 3 * nb, nb, best * 1e3, tot / frames * 1e3,
           frames, sum, mj423_last_error());
    return 0;
}
