// tools/asan_host_paths.cpp -- the library's threaded host paths on the GPU under
// AddressSanitizer (host code instrumented with -Xarch_host -fsanitize=address; the device
// code is not).  Test infrastructure only, built by `make -C mjpeg423-video-decoder-software_amd
// asan`, run on the GPU box by tools/asan_host_paths.sh.
//
//   asan_host_paths sparse.mpg dense.mpg outdir
// (two streams of one size: seeded synthetic content, and fully populated planes)
//
// Every path decodes the same frames, so the outputs are also checked against each other:
//   1. mjpeg423_decode (one-shot ring, 8 BMP writer threads)      -> BMP files
//   2. reusable pipeline, chunk 4: dense stream first (every slot's transfer buffer grows),
//      then the sparse one from frame 0, from a P-frame (GOP seed from the host), and to
//      device memory (device sink)
//   3. mj423_decode_mpg_pipelined (ring sized to the call) of the dense stream
//   4. the GPU front end (mj423_mpg_decode_gpu)
//   5. deferred per-block symbols idct()/ycbcr_to_rgb() over frame 0, flushed by encode_bmp()
// Prints one JSON line; exits non-zero on any mismatch (ASan aborts on any invalid access).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <string>
#include <vector>

#include "../include/mj423gpu.h"
#include "../include/mj423io.h"

namespace {

int fail(const char* what) {
    fprintf(stderr, "asan_host_paths: %s: %s\n", what, mj423_last_error());
    return 1;
}

struct Frames {
    uint32_t w = 0, h = 0;
    std::vector<std::vector<uint32_t>> px;
    static int put(void* u, uint32_t fi, const rgb_pixel_t* p, uint32_t w, uint32_t h) {
        Frames* f = (Frames*)u;
        if (fi >= f->px.size()) return 1;
        f->px[fi].assign((const uint32_t*)p, (const uint32_t*)p + (size_t)w * h);
        return 0;
    }
};

// Device sink: the chunk's frames copied out on the decode's stream before the sink returns.
struct DevFrames {
    uint32_t w = 0, h = 0;
    std::vector<uint32_t> px;
    static int put(void* u, uint32_t first, uint32_t count, const rgb_pixel_t* d, size_t stride, void* stream) {
        DevFrames* f = (DevFrames*)u;
        const size_t fp = (size_t)f->w * f->h;
        if ((size_t)(first + count) * fp > f->px.size()) return 1;
        for (uint32_t i = 0; i < count; i++)
            if (hipMemcpyAsync(f->px.data() + (first + i) * fp, d + i * stride, fp * 4, hipMemcpyDeviceToHost,
                               (hipStream_t)stream) != hipSuccess)
                return 1;
        return hipStreamSynchronize((hipStream_t)stream) != hipSuccess;
    }
};

std::vector<uint32_t> read_bmp(const std::string& path, uint32_t w, uint32_t h) {
    std::vector<uint32_t> px((size_t)w * h);
    FILE* f = fopen(path.c_str(), "rb");
    if (!f) return {};
    fseek(f, 54, SEEK_SET);
    for (uint32_t row = h; row-- > 0;)
        if (fread(px.data() + (size_t)row * w, 4, w, f) != w) px.clear();
    fclose(f);
    return px;
}

}  // namespace

int main(int argc, char** argv) {
    if (argc != 4) {
        fprintf(stderr, "usage: %s sparse.mpg dense.mpg outdir\n", argv[0]);
        return 2;
    }
    const std::string out = argv[3];
    mj423_mpg *ms = nullptr, *md = nullptr;
    mj423_mpg_header_t hs, hd;
    if (mj423_mpg_open(argv[1], &ms) || mj423_mpg_open(argv[2], &md) || mj423_mpg_header(ms, &hs) ||
        mj423_mpg_header(md, &hd))
        return fail("open");
    if (hs.width != hd.width || hs.height != hd.height) return fail("the two streams differ in size");
    const uint32_t w = hs.width, h = hs.height, n = hs.num_frames, nd = hd.num_frames;
    mj423_ctx* ctx = nullptr;
    if (mj423_ctx_create(&ctx, 0)) return fail("ctx");

    // 1. whole-file decoder
    if (mj423_decode_file(argv[1], (out + "/f0000.bmp").c_str())) return fail("decode_file");
    std::vector<std::vector<uint32_t>> bmp(n);
    for (uint32_t i = 0; i < n; i++) {
        char name[64];
        snprintf(name, sizeof name, "/f%04u.bmp", i);
        bmp[i] = read_bmp(out + name, w, h);
        if (bmp[i].empty()) return fail("read bmp");
    }

    // 2. reusable pipeline: dense stream (grows every slot), then sparse from 0 and from a P-frame
    int mismatches = 0;
    mj423_pipeline* p = nullptr;
    if (mj423_pipeline_create(&p, ctx, w, h, 4, 3)) return fail("pipeline create");
    Frames dense;
    dense.px.resize(nd);
    if (mj423_pipeline_decode(p, md, 0, nd, &Frames::put, &dense, nullptr)) return fail("pipeline dense");
    Frames a;
    a.px.resize(n);
    if (mj423_pipeline_decode(p, ms, 0, n, &Frames::put, &a, nullptr)) return fail("pipeline sparse");
    for (uint32_t i = 0; i < n; i++) mismatches += a.px[i] != bmp[i];
    const uint32_t seek = n > 6 ? 5 : 1;
    Frames b;
    b.px.resize(n);
    if (mj423_pipeline_decode(p, ms, seek, n - seek, &Frames::put, &b, nullptr)) return fail("pipeline seek");
    for (uint32_t i = seek; i < n; i++) mismatches += b.px[i] != bmp[i];
    DevFrames dv;
    dv.w = w;
    dv.h = h;
    dv.px.resize((size_t)n * w * h);
    if (mj423_pipeline_decode_device(p, ms, 0, n, &DevFrames::put, &dv, nullptr)) return fail("pipeline device");
    for (uint32_t i = 0; i < n; i++) mismatches += memcmp(dv.px.data() + (size_t)i * w * h, bmp[i].data(), (size_t)w * h * 4) != 0;
    mj423_pipeline_destroy(p);

    // 3. one-shot pipelined call (host sink), the dense stream against step 2
    Frames c;
    c.px.resize(nd);
    if (mj423_decode_mpg_pipelined(ctx, md, 0, nd, 0, 0, &Frames::put, &c, nullptr)) return fail("pipelined dense");
    for (uint32_t i = 0; i < nd; i++) mismatches += c.px[i] != dense.px[i];

    // 4. GPU front end
    rgb_pixel_t* d_out = nullptr;
    if (hipMalloc((void**)&d_out, (size_t)n * w * h * 4) != hipSuccess) return fail("hipMalloc");
    if (mj423_mpg_decode_gpu(ctx, ms, 0, n, d_out, (uint64_t)w * h, 0)) return fail("decode_gpu");
    std::vector<uint32_t> g((size_t)n * w * h);
    if (mj423_ctx_synchronize(ctx) || hipMemcpy(g.data(), d_out, g.size() * 4, hipMemcpyDeviceToHost) != hipSuccess)
        return fail("download");
    (void)hipFree(d_out);
    for (uint32_t i = 0; i < n; i++) mismatches += memcmp(g.data() + (size_t)i * w * h, bmp[i].data(), (size_t)w * h * 4) != 0;

    // 5. deferred per-block symbols over frame 0 (4:4:4, dequantized planes), flushed by encode_bmp()
    mj423_geometry_t geo;
    if (mj423_geometry(w, h, MJ423_CHROMA_444, &geo)) return fail("geometry");
    std::vector<int16_t> q((size_t)geo.coef_per_frame);
    if (mj423_mpg_entropy_decode(ms, 0, 1, q.data(), 2)) return fail("entropy");
    int16_t yq[64], cq[64];
    if (mj423_ctx_get_quant(ctx, yq, cq)) return fail("quant");
    const uint32_t nb = (w / 8) * (h / 8);
    std::vector<uint8_t> blk((size_t)nb * 3 * 64);
    std::vector<rgb_pixel_t> rgb((size_t)w * h);
    for (uint32_t pl = 0; pl < 3; pl++)
        for (uint32_t bi = 0; bi < nb; bi++) {
            dct_block_t d;
            const int16_t* src = q.data() + ((size_t)pl * nb + bi) * 64;
            for (int k = 0; k < 64; k++) d[k / 8][k % 8] = (int16_t)(src[k] * (pl ? cq[k] : yq[k]));
            idct(d, (uint8_t(*)[8])(blk.data() + ((size_t)pl * nb + bi) * 64));
        }
    for (uint32_t by = 0; by < h / 8; by++)
        for (uint32_t bx = 0; bx < w / 8; bx++) {
            const size_t bi = (size_t)by * (w / 8) + bx;
            ycbcr_to_rgb((int)(by * 8), (int)(bx * 8), w, (pcolor_block_t)(blk.data() + bi * 64),
                         (pcolor_block_t)(blk.data() + ((size_t)nb + bi) * 64),
                         (pcolor_block_t)(blk.data() + ((size_t)2 * nb + bi) * 64), rgb.data());
        }
    encode_bmp(rgb.data(), w, h, (out + "/blocks.bmp").c_str());
    mismatches += read_bmp(out + "/blocks.bmp", w, h) != bmp[0];

    mj423_mpg_close(ms);
    mj423_mpg_close(md);
    mj423_ctx_destroy(ctx);
    printf("{\"tool\": \"asan_host_paths\", \"width\": %u, \"height\": %u, \"frames\": %u, \"dense_frames\": %u, "
           "\"mismatches\": %d}\n",
           w, h, n, nd, mismatches);
    // Leave without running the HIP runtime's exit-time teardown: under ASan it can trip the
    // sanitizer's own device-allocator check after the runtime has unloaded (ROCm 7.2), a
    // failure in neither this program nor the library.  Everything above has completed.
    fflush(stdout);
    fflush(stderr);
    _exit(mismatches != 0);
}
