/* tools/e2e_phases.c -- where a native process running the library's mjpeg423_decode()
 * spends its wall time (measurements only, GPU box):
 *   - the first HIP call (hipFree(NULL): runtime + device init),
 *   - mj423_decode_file() twice (cold: code objects, default context, thread pools; warm),
 *   - the same work through the public pipeline API with its stages timed: pipeline create
 *     (pinned + device ring), decode with a no-op sink, decode with a one-thread BMP sink
 *     (front-end busy, sink busy, GPU span), destroy.
 *
 *   L=mjpeg423-video-decoder-software_amd; gcc -O2 -I include -o tools/e2e_phases tools/e2e_phases.c \
 *     -L$L -lmj423gpu -Wl,-rpath,'$ORIGIN/../'$L -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
 *   tools/e2e_phases in.mpg out0000.bmp CHUNK
 * Prints one JSON line. */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/mj423io.h"

/* the HIP runtime, a dependency of libmj423gpu.so */
int hipFree(void *p);
int hipMalloc(void **p, size_t n);
int hipHostMalloc(void **p, size_t n, unsigned flags);
int hipHostFree(void *p);

static double now(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + t.tv_nsec * 1e-9;
}

static int noop_sink(void *u, uint32_t fi, const rgb_pixel_t *px, uint32_t w, uint32_t h)
{
    (void)u, (void)fi, (void)px, (void)w, (void)h;
    return 0;
}

static int bmp_sink(void *u, uint32_t fi, const rgb_pixel_t *px, uint32_t w, uint32_t h)
{
    char name[4096];
    snprintf(name, sizeof name, "%s.p%04u.bmp", (const char *)u, fi);
    return mj423_write_bmp(name, px, w, h);
}

int main(int argc, char **argv)
{
    if (argc != 4) {
        fprintf(stderr, "usage: %s in.mpg out0000.bmp CHUNK\n", argv[0]);
        return 2;
    }
    const uint32_t chunk = (uint32_t)atoi(argv[3]);
    double t0 = now();
    if (hipFree(NULL) != 0) return 1;
    double t1 = now();
    int rc0 = mj423_decode_file(argv[1], argv[2]);
    double t2 = now();
    int rc1 = mj423_decode_file(argv[1], argv[2]);
    double t3 = now();
    printf("{\"tool\": \"e2e_phases\", \"hip_init_s\": %.4f, \"decode_file_cold_s\": %.4f, \"decode_file_warm_s\": %.4f",
           t1 - t0, t2 - t1, t3 - t2);
    mj423_ctx *ctx = NULL;
    mj423_mpg *m = NULL;
    mj423_mpg_header_t hd;
    if (rc0 || rc1 || mj423_ctx_create(&ctx, 0) || mj423_mpg_open(argv[1], &m) || mj423_mpg_header(m, &hd)) {
        printf(", \"error\": \"%s\"}\n", mj423_last_error());
        return 1;
    }
    mj423_pipeline *p = NULL;
    mj423_pipeline_stats_t sn, sb;
    double a = now();
    int rc = mj423_pipeline_create(&p, ctx, hd.width, hd.height, chunk, 0);
    double b = now();
    rc = rc ? rc : mj423_pipeline_decode(p, m, 0, hd.num_frames, noop_sink, NULL, &sn);
    double c = now();
    rc = rc ? rc : mj423_pipeline_decode(p, m, 0, hd.num_frames, bmp_sink, argv[2], &sb);
    double d = now();
    mj423_pipeline_destroy(p);
    double e = now();
    /* the allocation primitives behind create/destroy, 256 MiB each */
    void *hb = NULL, *db = NULL;
    const size_t nb = 256u << 20;
    double f0 = now();
    int arc = hipHostMalloc(&hb, nb, 0);
    double f1 = now();
    arc |= hipHostFree(hb);
    double f2 = now();
    arc |= hipMalloc(&db, nb);
    double f3 = now();
    arc |= hipFree(db);
    double f4 = now();
    printf(", \"pipeline\": {\"chunk\": %u, \"create_s\": %.4f, \"noop_s\": %.4f, \"bmp_s\": %.4f, \"destroy_s\": %.4f, "
           "\"bmp_frontend_busy_s\": %.4f, \"bmp_sink_busy_s\": %.4f, \"bmp_gpu_span_ms\": %.3f, \"noop_gpu_span_ms\": %.3f, "
           "\"rc\": %d}, \"alloc_256MiB\": {\"hipHostMalloc_s\": %.4f, \"hipHostFree_s\": %.4f, \"hipMalloc_s\": %.4f, "
           "\"hipFree_s\": %.4f, \"rc\": %d}}\n",
           chunk, b - a, c - b, d - c, e - d, sb.frontend_busy_s, sb.sink_busy_s, sb.gpu_span_ms, sn.gpu_span_ms, rc,
           f1 - f0, f2 - f1, f3 - f2, f4 - f3, arc);
    mj423_mpg_close(m);
    mj423_ctx_destroy(ctx);
    return rc;
}
