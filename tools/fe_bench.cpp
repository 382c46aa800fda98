// tools/fe_bench.cpp -- host entropy front-end rate (CPU only): every plane of a .mpg
// through the product's block walk (csrc/mj423_walk.hpp), single thread, into buffers
// allocated once -- dense quantized-domain planes and the streaming decoder's sparse form.
// Build: /opt/rocm/llvm/bin/clang++ -O3 -std=c++17 tools/fe_bench.cpp -o tools/fe_bench
//        (the compiler hipcc builds the library with; g++ code differs by up to 30 %)
// Run:   tools/fe_bench file.mpg            (e.g. written by tools/mpg_synth.py)
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../mjpeg423-video-decoder-software_amd/csrc/mj423_walk.hpp"

static uint32_t rd32(const uint8_t* p) {
    uint32_t v;
    std::memcpy(&v, p, 4);
    return v;
}

int main(int argc, char** argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s file.mpg\n", argv[0]);
        return 2;
    }
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 1;
    std::fseek(f, 0, SEEK_END);
    const long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    std::vector<uint8_t> buf(sz);
    if (std::fread(buf.data(), 1, sz, f) != (size_t)sz) return 1;
    std::fclose(f);
    // header: num_frames, width, height, num_iframes, payload_size (include/mj423io.h)
    const uint32_t nf = rd32(&buf[0]), w = rd32(&buf[4]), h = rd32(&buf[8]);
    const int nb = (int)((w / 8) * (h / 8));
    struct Plane {
        const uint8_t* p;
        size_t n;
        bool P;
    };
    std::vector<Plane> planes;
    size_t off = 20;
    for (uint32_t i = 0; i < nf && off + 16 <= buf.size(); i++) {
        const uint32_t fs = rd32(&buf[off]), ft = rd32(&buf[off + 4]), ys = rd32(&buf[off + 8]),
                       cbs = rd32(&buf[off + 12]);
        const uint8_t* y = &buf[off + 16];
        planes.push_back({y, ys, ft != 0});
        planes.push_back({y + ys, cbs, ft != 0});
        planes.push_back({y + ys + cbs, fs - 16 - ys - cbs, ft != 0});
        off += fs;
    }
    std::vector<int16_t> dense((size_t)nb * 64);
    std::vector<uint8_t> counts(nb);
    std::vector<uint32_t> seg(nb / 256 + 2), ent((size_t)nb * 64);
    auto time_it = [&](const char* name, auto fn) {
        double best = 1e30;
        size_t total = 0;
        for (int r = 0; r < 5; r++) {
            const auto t0 = std::chrono::steady_clock::now();
            total = 0;
            for (const Plane& pl : planes) total += fn(pl);
            best = std::min(best, std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count());
        }
        const double blocks = (double)nb * planes.size();
        std::printf("%-8s %6.2f ns/block  %7.1f Mpix/s per thread  (%zu)\n", name, best / blocks * 1e9,
                    (double)w * h * (planes.size() / 3) / best / 1e6, total);
    };
    std::printf("%ux%u 4:4:4, %zu frames\n", w, h, planes.size() / 3);
    time_it("dense", [&](const Plane& pl) {
        bool over = false;
        return mj423fe::walk<true>(nb, pl.p, pl.p + pl.n, dense.data(), nullptr, pl.P, &over);
    });
    time_it("sparse", [&](const Plane& pl) {
        bool over = false;
        size_t used = 0;
        return mj423fe::walk_sparse(nb, pl.p, pl.p + pl.n, pl.P, counts.data(), seg.data(), ent.data(), &over, &used);
    });
    return 0;
}
