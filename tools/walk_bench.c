/* tools/walk_bench.c -- host entropy front end against the reference's (measurements only):
 * every frame of an .mpg through lossless_decode() (the dequantizing, reference-signature
 * symbol, decoder/lossless_decode.c:60) three planes at a time, and -- library build only --
 * through mj423_lossless_decode_q() (the bounded quantized-domain walk the pipeline uses).
 * The same source is built twice (oracle/Makefile): against the library alone, and with the
 * reference's lossless_decode.c compiled in place (REF_BUILD), whose symbol then wins.
 *
 *   walk_bench in.mpg REPS
 * Prints one JSON line: milliseconds per frame (best of REPS) and an FNV-1a hash of the
 * decoded planes of the last frame (equal between the two builds). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <time.h>

#include "../include/mj423io.h"

typedef int16_t blk8_t[8][8];
void lossless_decode(int num_blocks, void *bitstream, blk8_t *DCACq, blk8_t quant, int P);

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static uint64_t fnv(const void *p, size_t n, uint64_t h)
{
    const uint8_t *b = (const uint8_t *)p;
    for (size_t i = 0; i < n; i++) h = (h ^ b[i]) * 0x100000001b3ull;
    return h;
}

int main(int argc, char **argv)
{
    if (argc != 3) {
        fprintf(stderr, "usage: %s in.mpg REPS\n", argv[0]);
        return 2;
    }
    mj423_mpg *m;
    mj423_mpg_header_t hd;
    if (mj423_mpg_open(argv[1], &m) || mj423_mpg_header(m, &hd)) {
        fprintf(stderr, "%s\n", mj423_last_error());
        return 1;
    }
    const int reps = atoi(argv[2]);
    const int nb = (int)((hd.width / 8) * (hd.height / 8));
    blk8_t *pl[3];
    for (int i = 0; i < 3; i++) pl[i] = (blk8_t *)calloc((size_t)nb, sizeof(blk8_t));
    /* decoder/mjpeg423_decoder.c passes Yquant for Y and Cquant for Cb/Cr (common/tables.c) */
    static blk8_t yq = {{16, 11, 10, 16, 24, 40, 51, 61},     {12, 12, 14, 19, 26, 58, 60, 55},
                        {14, 13, 16, 24, 40, 57, 69, 56},     {14, 17, 22, 29, 51, 87, 80, 62},
                        {18, 22, 37, 56, 68, 109, 103, 77},   {24, 35, 55, 64, 81, 104, 113, 92},
                        {49, 64, 78, 87, 103, 121, 120, 101}, {72, 92, 95, 98, 112, 100, 103, 99}};
    static blk8_t cq = {{17, 18, 24, 47, 99, 99, 99, 99}, {18, 21, 26, 66, 99, 99, 99, 99},
                        {24, 26, 56, 99, 99, 99, 99, 99}, {47, 66, 99, 99, 99, 99, 99, 99},
                        {99, 99, 99, 99, 99, 99, 99, 99}, {99, 99, 99, 99, 99, 99, 99, 99},
                        {99, 99, 99, 99, 99, 99, 99, 99}, {99, 99, 99, 99, 99, 99, 99, 99}};
    double best = 1e30, best_q = 1e30;
    for (int r = 0; r < reps; r++) {
        double t = now();
        for (uint32_t f = 0; f < hd.num_frames; f++) {
            mj423_mpg_frame_t fr;
            mj423_mpg_frame(m, f, &fr);
            lossless_decode(nb, (void *)fr.y, pl[0], yq, fr.frame_type != 0);
            lossless_decode(nb, (void *)fr.cb, pl[1], cq, fr.frame_type != 0);
            lossless_decode(nb, (void *)fr.cr, pl[2], cq, fr.frame_type != 0);
        }
        t = (now() - t) * 1e3 / hd.num_frames;
        if (t < best) best = t;
    }
    uint64_t h = 0xcbf29ce484222325ull;
    for (int i = 0; i < 3; i++) h = fnv(pl[i], (size_t)nb * sizeof(blk8_t), h);
#ifndef REF_BUILD
    for (int r = 0; r < reps; r++) {
        double t = now();
        for (uint32_t f = 0; f < hd.num_frames; f++) {
            mj423_mpg_frame_t fr;
            mj423_mpg_frame(m, f, &fr);
            mj423_lossless_decode_q(nb, fr.y, fr.y_size, &pl[0][0][0][0], fr.frame_type != 0);
            mj423_lossless_decode_q(nb, fr.cb, fr.cb_size, &pl[1][0][0][0], fr.frame_type != 0);
            mj423_lossless_decode_q(nb, fr.cr, fr.cr_size, &pl[2][0][0][0], fr.frame_type != 0);
        }
        t = (now() - t) * 1e3 / hd.num_frames;
        if (t < best_q) best_q = t;
    }
    printf("{\"tool\": \"walk_bench\", \"build\": \"library\", \"frames\": %u, \"width\": %u, \"height\": %u, "
           "\"lossless_decode_ms_per_frame\": %.3f, \"lossless_decode_q_ms_per_frame\": %.3f, \"hash\": \"%016llx\"}\n",
           hd.num_frames, hd.width, hd.height, best, best_q, (unsigned long long)h);
#else
    (void)best_q;
    printf("{\"tool\": \"walk_bench\", \"build\": \"reference\", \"frames\": %u, \"width\": %u, \"height\": %u, "
           "\"lossless_decode_ms_per_frame\": %.3f, \"hash\": \"%016llx\"}\n",
           hd.num_frames, hd.width, hd.height, best, (unsigned long long)h);
#endif
    mj423_mpg_close(m);
    return 0;
}
