/*
 * mj423_multigpu -- a plain C host driving every GPU of a node through the C ABI
 * (include/mj423gpu.h section 5): the multi-GPU decode BASELINE.json configs[3]/[4] describe.
 *
 *   one process, one context + RCCL communicator per device (mj423_multi_create);
 *   rank 0's {Yquant, Cquant} to every device by ncclBroadcast (mj423_multi_set_quant);
 *   frames sharded as contiguous per-device ranges, generated on each device (no PCIe);
 *   K start-aligned timed decode steps (mj423_multi_time_decode); one JSON line on stdout.
 *
 * It replaces the reference's two-core split of each frame (c0/playback.c:80-134,
 * core1/software/main.c:227-335): here whole frames go to whole GPUs.
 *
 *   mj423_multigpu [--ndev N] [--devices 0,1,..] [--no-comm] [--width W] [--height H]
 *                  [--chroma 420|422|444] [--frames-per-gpu F | --total-frames T]
 *                  [--steps K] [--warmup W] [--seed S] [--hashes]
 *                  [--mpg FILE [--first F] [--count C]]
 *
 * --hashes prints the FNV-1a 64 of every decoded frame (BGRA bytes, global frame order) so
 * a test can compare them with the CPU oracle's.  --mpg decodes a real .mpg instead, cut at
 * I-frames over the devices, entropy decode included (mj423_multi_decode_mpg_gpu).
 */
#include <hip/hip_runtime_api.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../../../include/mj423gpu.h"
#include "../../../include/mj423io.h"

#define MAXDEV 64
#define HBM_PEAK_GBPS 8000.0 /* MI355X spec, /opt/skills/guides/MI355X_MICROARCH.md */

static void die(const char *what) {
    fprintf(stderr, "mj423_multigpu: %s: %s\n", what, mj423_last_error());
    exit(1);
}

static uint64_t fnv1a64(const void *p, size_t n) {
    const uint8_t *b = (const uint8_t *)p;
    uint64_t h = 0xCBF29CE484222325ull;
    for (size_t i = 0; i < n; i++) {
        h ^= b[i];
        h *= 0x100000001b3ull;
    }
    return h;
}

static double now_ms(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec * 1e3 + t.tv_nsec / 1e6;
}

/* Hashes `count` frames of w*h BGRA pixels at device pointer d (stride w*h) into hashes[]. */
static void hash_frames(const rgb_pixel_t *d, uint64_t count, uint32_t w, uint32_t h, uint64_t *hashes) {
    const size_t fb = (size_t)w * h * 4;
    void *host = malloc(fb);
    if (!host) {
        fprintf(stderr, "mj423_multigpu: out of host memory\n");
        exit(1);
    }
    for (uint64_t i = 0; i < count; i++) {
        if (hipMemcpy(host, (const char *)d + i * fb, fb, hipMemcpyDeviceToHost) != hipSuccess) {
            fprintf(stderr, "mj423_multigpu: download failed\n");
            exit(1);
        }
        hashes[i] = fnv1a64(host, fb);
    }
    free(host);
}

static int run_mpg(mj423_multi *g, int n, const int *devs, const char *path, uint32_t first, int64_t count_arg,
                   int steps, int warmup, int hashes) {
    mj423_mpg *m;
    if (mj423_mpg_open(path, &m)) die("mj423_mpg_open");
    mj423_mpg_header_t hdr;
    mj423_mpg_header(m, &hdr);
    const uint32_t count = count_arg < 0 ? hdr.num_frames - first : (uint32_t)count_arg;
    uint32_t rf[MAXDEV], rc[MAXDEV];
    if (mj423_mpg_gop_ranges(m, first, count, (uint32_t)n, rf, rc)) die("mj423_mpg_gop_ranges");
    rgb_pixel_t *out[MAXDEV];
    const size_t fb = (size_t)hdr.width * hdr.height * 4;
    for (int r = 0; r < n; r++) {
        out[r] = NULL;
        hipSetDevice(devs[r]);
        if (rc[r] && hipMalloc((void **)&out[r], rc[r] * fb) != hipSuccess) {
            fprintf(stderr, "mj423_multigpu: hipMalloc of rank %d's frames failed\n", r);
            return 1;
        }
    }
    for (int i = 0; i < warmup; i++)
        if (mj423_multi_decode_mpg_gpu(g, m, first, count, out, 0, NULL, NULL)) die("mj423_multi_decode_mpg_gpu");
    const double t0 = now_ms();
    for (int i = 0; i < steps; i++)
        if (mj423_multi_decode_mpg_gpu(g, m, first, count, out, 0, NULL, NULL)) die("mj423_multi_decode_mpg_gpu");
    const double wall = now_ms() - t0; /* synchronous: every device has finished */
    const double px = (double)count * hdr.width * hdr.height * steps;
    printf("{\"tool\": \"mj423_multigpu\", \"mode\": \"mpg\", \"ranks\": %d, \"comm_ranks\": %d, \"width\": %u, "
           "\"height\": %u, \"frames\": %u, \"steps\": %d, \"ms_per_step\": %.4f, \"mpix_s\": %.1f, \"ranges\": [",
           n, mj423_multi_comm_ranks(g), hdr.width, hdr.height, count, steps, wall / steps, px / (wall / 1e3) / 1e6);
    for (int r = 0; r < n; r++) printf("%s[%u, %u]", r ? ", " : "", rf[r], rc[r]);
    printf("]");
    if (hashes) {
        printf(", \"first\": %u, \"hashes\": [", first);
        int k = 0;
        for (int r = 0; r < n; r++) {
            if (!rc[r]) continue;
            uint64_t *hs = (uint64_t *)malloc(rc[r] * sizeof(uint64_t));
            hipSetDevice(devs[r]);
            hash_frames(out[r], rc[r], hdr.width, hdr.height, hs);
            for (uint32_t i = 0; i < rc[r]; i++) printf("%s\"%016llx\"", k++ ? ", " : "", (unsigned long long)hs[i]);
            free(hs);
        }
        printf("]");
    }
    printf("}\n");
    for (int r = 0; r < n; r++)
        if (out[r]) {
            hipSetDevice(devs[r]);
            hipFree(out[r]);
        }
    mj423_mpg_close(m);
    return 0;
}

int main(int argc, char **argv) {
    int ndev = 0, ndevs_listed = 0, flags = 0, steps = 20, warmup = 3, hashes = 0, chroma = 420;
    int devs[MAXDEV];
    uint32_t w = 3840, h = 2160;
    uint64_t per_gpu = 300, total = 0, seed = 0x4D4A3432ull;
    const char *mpg = NULL;
    uint32_t mpg_first = 0;
    int64_t mpg_count = -1;
    for (int i = 1; i < argc; i++) {
        const char *a = argv[i];
        const char *v = i + 1 < argc ? argv[i + 1] : NULL;
#define ARG(name) (!strcmp(a, name) && v && (++i, 1))
        if (ARG("--ndev")) ndev = atoi(v);
        else if (ARG("--devices")) {
            for (const char *p = v; *p && ndevs_listed < MAXDEV;) {
                devs[ndevs_listed++] = atoi(p);
                p = strchr(p, ',') ? strchr(p, ',') + 1 : p + strlen(p);
            }
        } else if (!strcmp(a, "--no-comm")) flags |= MJ423_MULTI_NO_COMM;
        else if (ARG("--width")) w = (uint32_t)atoi(v);
        else if (ARG("--height")) h = (uint32_t)atoi(v);
        else if (ARG("--chroma")) chroma = atoi(v);
        else if (ARG("--frames-per-gpu")) per_gpu = strtoull(v, NULL, 10);
        else if (ARG("--total-frames")) total = strtoull(v, NULL, 10);
        else if (ARG("--steps")) steps = atoi(v);
        else if (ARG("--warmup")) warmup = atoi(v);
        else if (ARG("--seed")) seed = strtoull(v, NULL, 0);
        else if (!strcmp(a, "--hashes")) hashes = 1;
        else if (ARG("--mpg")) mpg = v;
        else if (ARG("--first")) mpg_first = (uint32_t)atoi(v);
        else if (ARG("--count")) mpg_count = atoll(v);
        else {
            fprintf(stderr, "mj423_multigpu: unknown or incomplete argument %s (see the header of mj423_multigpu.c)\n", a);
            return 2;
        }
#undef ARG
    }
    if (steps < 1) steps = 1;
    int visible = 0;
    if (hipGetDeviceCount(&visible) != hipSuccess || visible == 0) {
        fprintf(stderr, "mj423_multigpu: no HIP device visible\n");
        return 1;
    }
    if (ndevs_listed == 0) {
        ndevs_listed = ndev > 0 ? ndev : visible;
        if (ndevs_listed > MAXDEV) ndevs_listed = MAXDEV;
        for (int r = 0; r < ndevs_listed; r++) devs[r] = r;
    }
    const int n = ndevs_listed;
    mj423_multi *g;
    if (mj423_multi_create(&g, n, devs, flags)) die("mj423_multi_create");
    if (mj423_multi_set_quant(g, NULL, NULL)) die("mj423_multi_set_quant (RCCL broadcast)");
    if (mpg) {
        int rc = run_mpg(g, n, devs, mpg, mpg_first, mpg_count, steps, warmup, hashes);
        mj423_multi_destroy(g);
        return rc;
    }

    mj423_geometry_t geo;
    if (mj423_geometry(w, h, chroma, &geo)) die("mj423_geometry");
    const uint64_t frames_all = total ? total : per_gpu * (uint64_t)n;
    int16_t *coef[MAXDEV];
    rgb_pixel_t *out[MAXDEV];
    uint64_t first[MAXDEV];
    uint32_t cnt[MAXDEV];
    mj423_frames_desc_t desc[MAXDEV];
    for (int r = 0; r < n; r++) {
        uint64_t f, c;
        mj423_frame_range((uint32_t)r, (uint32_t)n, frames_all, &f, &c);
        first[r] = f;
        cnt[r] = (uint32_t)c;
        coef[r] = NULL;
        out[r] = NULL;
        hipSetDevice(devs[r]);
        if (c && (hipMalloc((void **)&coef[r], c * geo.coef_per_frame * 2) != hipSuccess ||
                  hipMalloc((void **)&out[r], c * (size_t)w * h * 4) != hipSuccess)) {
            fprintf(stderr, "mj423_multigpu: hipMalloc of rank %d's %llu frames failed\n", r, (unsigned long long)c);
            return 1;
        }
        const int16_t *y = coef[r];
        mj423_frames_desc_t d = {y, y ? y + 64ull * geo.y_blocks : NULL,
                                 y ? y + 64ull * (geo.y_blocks + geo.c_blocks) : NULL, geo.coef_per_frame, out[r],
                                 (uint64_t)w * h, w, cnt[r], w, h, chroma, MJ423_INPUT_QUANTIZED};
        desc[r] = d;
    }
    /* every device generates its own range of the global synthetic stream: no bulk PCIe/xGMI traffic */
    if (mj423_multi_synth_frames_device(g, coef, first, cnt, w, h, chroma, seed)) die("mj423_multi_synth_frames_device");
    if (mj423_multi_synchronize(g)) die("synchronize");
    double mx, wall, per[MAXDEV];
    if (warmup > 0 && mj423_multi_time_decode(g, desc, (uint32_t)warmup, &mx, per, &wall)) die("warmup");
    if (mj423_multi_time_decode(g, desc, (uint32_t)steps, &mx, per, &wall)) die("mj423_multi_time_decode");

    const double px = (double)frames_all * w * h * steps;
    const double bytes_step = (double)mj423_frame_bytes(w, h, chroma) * frames_all;
    /* per-rank roofline: that rank's algorithmic bytes over its own event time */
    printf("{\"tool\": \"mj423_multigpu\", \"mode\": \"synthetic\", \"ranks\": %d, \"comm_ranks\": %d, "
           "\"width\": %u, \"height\": %u, \"chroma\": %d, \"total_frames\": %llu, \"scaling\": \"%s\", \"steps\": %d, "
           "\"max_ms\": %.4f, \"wall_ms\": %.4f, \"ms_per_step\": %.4f, \"mpix_s\": %.1f, \"mpix_s_wall\": %.1f, "
           "\"aggregate_GBps\": %.1f, \"per_rank\": [",
           n, mj423_multi_comm_ranks(g), w, h, chroma, (unsigned long long)frames_all, total ? "strong" : "weak", steps,
           mx, wall, mx / steps, px / (mx / 1e3) / 1e6, px / (wall / 1e3) / 1e6, bytes_step * steps / (mx / 1e3) / 1e9);
    for (int r = 0; r < n; r++) {
        const double gbps = cnt[r] ? (double)mj423_frame_bytes(w, h, chroma) * cnt[r] * steps / (per[r] / 1e3) / 1e9 : 0.0;
        printf("%s{\"rank\": %d, \"device\": %d, \"first\": %llu, \"frames\": %u, \"ms\": %.4f, \"GBps\": %.1f, "
               "\"hbm_frac\": %.4f}",
               r ? ", " : "", r, devs[r], (unsigned long long)first[r], cnt[r], per[r], gbps, gbps / HBM_PEAK_GBPS);
    }
    printf("]");
    if (hashes) {
        printf(", \"hashes\": [");
        int k = 0;
        for (int r = 0; r < n; r++) {
            if (!cnt[r]) continue;
            uint64_t *hs = (uint64_t *)malloc(cnt[r] * sizeof(uint64_t));
            hipSetDevice(devs[r]);
            hash_frames(out[r], cnt[r], w, h, hs);
            for (uint32_t i = 0; i < cnt[r]; i++) printf("%s\"%016llx\"", k++ ? ", " : "", (unsigned long long)hs[i]);
            free(hs);
        }
        printf("]");
    }
    printf("}\n");
    for (int r = 0; r < n; r++) {
        hipSetDevice(devs[r]);
        if (coef[r]) hipFree(coef[r]);
        if (out[r]) hipFree(out[r]);
    }
    mj423_multi_destroy(g);
    return 0;
}
