// tools/fuzz_frontend.cpp -- mutation fuzzing of the library's host front end (the .mpg container
// parser and the entropy walk, csrc/mj423_io.cpp + mj423_walk.hpp) under AddressSanitizer.  These
// parse untrusted bytes; the reference's own decoder indexes past its zig-zag table on damaged
// streams (lossless_decode.c:117-125, UB), the library must not.  Test infrastructure only.
//
//   usage: fuzz_frontend ITERATIONS SEED file.mpg [file.mpg ...]
//
// Each iteration takes one of the files and applies 1-8 random mutations (bit flips, byte
// stores, 32-bit field overwrites in the file header / frame tables / trailer, truncation,
// zero or random extension), then: mj423_mpg_open_memory; when accepted, the header, every
// frame record, the trailer, GOP starts, and an entropy decode (absolute planes, and per-frame
// deltas) of a random frame range on 1-2 host threads.  Every 4th iteration also feeds the raw
// quantized-domain walk (mj423_lossless_decode_q) a random or truncated bitstream.  ASan aborts
// the process on any invalid access; otherwise prints one JSON line of counts and exits 0.
// Built by `make -C mjpeg423-video-decoder-software_amd asan` (host code with -fsanitize=address;
// no GPU call is made).
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../include/mj423gpu.h"
#include "../include/mj423io.h"

namespace {

struct Rng {  // SplitMix64
    uint64_t s;
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ull);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
        return z ^ (z >> 31);
    }
    uint32_t below(uint32_t n) { return n ? (uint32_t)(next() % n) : 0; }
};

std::vector<uint8_t> read_file(const char* path) {
    std::vector<uint8_t> b;
    FILE* f = fopen(path, "rb");
    if (!f) return b;
    uint8_t buf[65536];
    size_t n;
    while ((n = fread(buf, 1, sizeof buf, f)) > 0) b.insert(b.end(), buf, buf + n);
    fclose(f);
    return b;
}

void put32(std::vector<uint8_t>& b, size_t off, uint32_t v) {
    if (off + 4 <= b.size()) memcpy(b.data() + off, &v, 4);
}

// A field value that is interesting to a size check: small, boundary, huge, or random.
uint32_t field_value(Rng& r, uint32_t old) {
    switch (r.below(8)) {
    case 0: return 0;
    case 1: return 1;
    case 2: return old + 1;
    case 3: return old - 1;
    case 4: return 0xffffffffu;
    case 5: return 0x80000000u;
    case 6: return old * 2 + 8;
    default: return (uint32_t)r.next();
    }
}

void mutate(std::vector<uint8_t>& b, Rng& r) {
    const uint32_t n = 1 + r.below(8);
    for (uint32_t i = 0; i < n && !b.empty(); i++) {
        switch (r.below(7)) {
        case 0: b[r.below((uint32_t)b.size())] ^= (uint8_t)(1u << r.below(8)); break;
        case 1: b[r.below((uint32_t)b.size())] = (uint8_t)r.next(); break;
        case 2: {  // a header field (5 x u32)
            const size_t off = 4 * r.below(5);
            uint32_t old = 0;
            if (off + 4 <= b.size()) memcpy(&old, b.data() + off, 4);
            put32(b, off, field_value(r, old));
            break;
        }
        case 3: {  // a field at an aligned offset anywhere (frame records, trailer)
            const size_t off = 4 * (size_t)r.below((uint32_t)(b.size() / 4 + 1));
            uint32_t old = 0;
            if (off + 4 <= b.size()) memcpy(&old, b.data() + off, 4);
            put32(b, off, field_value(r, old));
            break;
        }
        case 4: b.resize(r.below((uint32_t)b.size() + 1)); break;  // truncate
        case 5: {  // extend with zeros or noise
            const size_t add = r.below(4096);
            const bool noise = r.below(2);
            for (size_t k = 0; k < add; k++) b.push_back(noise ? (uint8_t)r.next() : 0);
            break;
        }
        default: {  // a run of random bytes
            const size_t at = r.below((uint32_t)b.size()), len = 1 + r.below(64);
            for (size_t k = 0; k < len && at + k < b.size(); k++) b[at + k] = (uint8_t)r.next();
            break;
        }
        }
    }
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) {
        fprintf(stderr, "usage: %s ITERATIONS SEED file.mpg [...]\n", argv[0]);
        return 2;
    }
    const long iters = atol(argv[1]);
    Rng r{strtoull(argv[2], nullptr, 0)};
    std::vector<std::vector<uint8_t>> files;
    for (int i = 3; i < argc; i++) {
        files.push_back(read_file(argv[i]));
        if (files.back().empty()) {
            fprintf(stderr, "cannot read %s\n", argv[i]);
            return 2;
        }
    }
    long opened = 0, rejected = 0, decoded = 0, decode_failed = 0, walks = 0;
    std::vector<int16_t> coef;
    std::vector<uint8_t> types;
    for (long it = 0; it < iters; it++) {
        std::vector<uint8_t> b = files[r.below((uint32_t)files.size())];
        if (it % 16 != 0) mutate(b, r);  // every 16th input unmutated: the accept path stays covered
        mj423_mpg* m = nullptr;
        if (mj423_mpg_open_memory(b.data(), b.size(), &m) != 0 || !m) {
            rejected++;
        } else {
            opened++;
            mj423_mpg_header_t h;
            if (mj423_mpg_header(m, &h) == 0) {
                mj423_mpg_frame_t f;
                for (uint32_t i = 0; i < h.num_frames && i < 4096; i++) (void)mj423_mpg_frame(m, i, &f);
                (void)mj423_mpg_frame(m, h.num_frames, &f);  // one past the end: must be refused
                std::vector<uint32_t> idx(64), pos(64);
                (void)mj423_mpg_trailer(m, idx.data(), pos.data(), 64);
                uint32_t g = 0;
                if (h.num_frames) (void)mj423_mpg_gop_start(m, r.below(h.num_frames), &g);
                mj423_geometry_t geo;
                if (h.num_frames && mj423_geometry(h.width, h.height, MJ423_CHROMA_444, &geo) == 0 &&
                    geo.coef_per_frame <= (1u << 22)) {
                    const uint32_t first = r.below(h.num_frames);
                    const uint32_t count = 1 + r.below(std::min<uint32_t>(h.num_frames - first, 6));
                    coef.assign((size_t)count * geo.coef_per_frame, 0);
                    types.assign(count, 0);
                    const int threads = 1 + (int)r.below(2);
                    const int a = mj423_mpg_entropy_decode(m, first, count, coef.data(), threads);
                    const int d = mj423_mpg_entropy_decode_deltas(m, first, count, coef.data(), types.data(), threads);
                    if (a == 0 && d == 0) decoded++;
                    else decode_failed++;
                }
            }
            mj423_mpg_close(m);
        }
        if (it % 4 == 0) {  // the raw walk on a random or truncated stream
            const int nblk = 1 + (int)r.below(2048);
            std::vector<uint8_t> s(r.below(4096));
            for (auto& x : s) x = (uint8_t)(r.below(4) ? r.next() : 0);
            std::vector<int16_t> q((size_t)nblk * 64, 0);
            (void)mj423_lossless_decode_q(nblk, s.data(), s.size(), q.data(), (int)r.below(2));
            walks++;
        }
    }
    printf("{\"tool\": \"fuzz_frontend\", \"iterations\": %ld, \"opened\": %ld, \"rejected\": %ld, \"decoded\": %ld, "
           "\"decode_rejected\": %ld, \"raw_walks\": %ld}\n",
           iters, opened, rejected, decoded, decode_failed, walks);
    return 0;
}
