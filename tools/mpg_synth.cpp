// mpg_synth.cpp -- synthetic MPEG423 (.mpg) stream writer for benchmarks and tests.
//
// Not part of the product and not the oracle: a from-scratch writer of the container
// and bitstream format that the product's front end reads (include/mj423io.h), fed with
// seeded synthetic quantized coefficients (SURVEY.md §8(d) statistics), so real-stream
// benchmarks can run at sizes no committed fixture has.  Format, as read by the
// reference decoder (core0/software/common/libs/mjpeg423/, "mj/"):
//   * per plane, per block in raster order: DC = SIZE(4 bits) + SIZE-bit VLI of the
//     difference to the previous block's DC (I-frames; P-frames code the delta itself),
//     then AC symbols RUN(4) SIZE(4) + VLI in zig-zag order, ZRL = 0xF0 (16 zeros),
//     EOB = 0x00 unless the block ends at position 63 (mj/decoder/lossless_decode.c:82-134,204-246);
//   * container: 5 x u32 header, per frame u32 {frame_size, type, Ysize, Cbsize} + the
//     three bitstreams padded to 4 bytes, then the I-frame trailer and 512 pad bytes
//     (mj/encoder/mjpeg423_encoder.c:82-88,188-225).
// The tests check these files against the reference's own decoder (oracle/_ref).
//
// Build: g++ -O2 -std=c++17 -shared -fPIC tools/mpg_synth.cpp -o tools/libmpgsynth.so -lpthread
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <thread>
#include <vector>

namespace {

const uint8_t kZigzag[64] = {0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
                             12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
                             35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
                             58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};
const int16_t kYq[64] = {16, 11, 10, 16, 24,  40,  51,  61,  12, 12, 14, 19, 26,  58,  60,  55,
                         14, 13, 16, 24, 40,  57,  69,  56,  14, 17, 22, 29, 51,  87,  80,  62,
                         18, 22, 37, 56, 68,  109, 103, 77,  24, 35, 55, 64, 81,  104, 113, 92,
                         49, 64, 78, 87, 103, 121, 120, 101, 72, 92, 95, 98, 112, 100, 103, 99};
const int16_t kCq[64] = {17, 18, 24, 47, 99, 99, 99, 99, 18, 21, 26, 66, 99, 99, 99, 99,
                         24, 26, 56, 99, 99, 99, 99, 99, 47, 66, 99, 99, 99, 99, 99, 99,
                         99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99,
                         99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99, 99};

struct BitWriter {
    std::vector<uint8_t>& out;
    uint64_t acc = 0;
    int n = 0;
    explicit BitWriter(std::vector<uint8_t>& o) : out(o) {}
    void put(uint32_t v, int k) {  // k <= 24
        acc = (acc << k) | (v & ((1u << k) - 1));
        n += k;
        while (n >= 8) {
            out.push_back((uint8_t)(acc >> (n - 8)));
            n -= 8;
        }
    }
    void flush() {
        if (n > 0) out.push_back((uint8_t)(acc << (8 - n)));
        n = 0;
    }
};

int bitlen(int32_t v) {
    uint32_t a = (uint32_t)(v < 0 ? -v : v);
    int s = 0;
    while (a) {
        s++;
        a >>= 1;
    }
    return s;
}
void put_vli(BitWriter& bw, int32_t e, int size) {
    if (size) bw.put((uint32_t)(e >= 0 ? e : e + (1 << size) - 1), size);
}

// One plane's bitstream.  I (P == 0): blocks are absolute, DC coded as int16 differences;
// P: blocks are the deltas lossless_decode adds.
void encode_plane(int nblocks, const int16_t* blocks, bool P, std::vector<uint8_t>& out) {
    BitWriter bw(out);
    int16_t prev = 0;
    for (int b = 0; b < nblocks; b++) {
        const int16_t* q = blocks + (size_t)b * 64;
        const int32_t e = P ? q[0] : (int16_t)(q[0] - prev);
        prev = q[0];
        const int s = bitlen(e);
        bw.put((uint32_t)s, 4);
        put_vli(bw, e, s);
        int run = 0;
        int last = 0;
        for (int k = 63; k >= 1; k--)
            if (q[kZigzag[k]]) {
                last = k;
                break;
            }
        for (int k = 1; k <= last; k++) {
            const int32_t v = q[kZigzag[k]];
            if (!v) {
                run++;
                continue;
            }
            while (run > 15) {
                bw.put(0xF0, 8);
                run -= 16;
            }
            const int sz = bitlen(v);
            bw.put((uint32_t)((run << 4) | sz), 8);
            put_vli(bw, v, sz);
            run = 0;
        }
        if (last < 63) bw.put(0x00, 8);
    }
    bw.flush();
}

inline uint64_t splitmix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
struct Rng {
    uint64_t s;
    uint32_t next() { return (uint32_t)((s = splitmix(s)) >> 32); }
    double uni() { return next() * (1.0 / 4294967296.0); }
};

// Frame f of plane `plane` (0 Y, 1 Cb, 2 Cr): I-frame content per SURVEY §8(d); a P-frame
// adds sparse small deltas to `state`, kept within |Q*q| <= 1023.  `state` = absolute
// coefficients (updated), `stream` = what the bitstream codes (I: absolute, P: deltas).
void gen_plane(uint64_t seed, uint32_t f, int plane, int nblocks, bool P, int16_t* state, int16_t* stream) {
    const int16_t* qt = plane == 0 ? kYq : kCq;
    for (int b = 0; b < nblocks; b++) {
        Rng r{seed ^ ((uint64_t)f << 40) ^ ((uint64_t)plane << 36) ^ (uint64_t)b * 0x2545F4914F6CDD1Dull};
        int16_t* a = state + (size_t)b * 64;
        int16_t* o = stream + (size_t)b * 64;
        if (!P) {
            std::memset(a, 0, 128);
            a[0] = (int16_t)(r.next() % (uint32_t)(2040 / qt[0] + 1));
            for (int k = 1; k < 64; k++) {
                if (r.uni() >= 0.6 * std::exp(-k / 8.0)) continue;
                int mag = 1;
                while (r.uni() < 0.65 && mag < 64) mag++;
                const int n = kZigzag[k];
                mag = std::min(mag, 1023 / qt[n]);
                if (mag == 0) continue;
                a[n] = (int16_t)((r.next() & 1) ? mag : -mag);
            }
            std::memcpy(o, a, 128);
        } else {
            std::memset(o, 0, 128);
            for (int k = 0; k < 64; k++) {
                if (r.uni() >= (k == 0 ? 0.5 : 0.15 * std::exp(-k / 8.0))) continue;
                const int n = kZigzag[k];
                const int d = (r.next() & 1) ? 1 + (int)(r.next() % 3) : -1 - (int)(r.next() % 3);
                const int v = a[n] + d;
                if (n == 0 ? (v < 0 || v > 2040 / qt[0]) : std::abs(v * qt[n]) > 1023) continue;
                a[n] = (int16_t)v;
                o[n] = (int16_t)d;
            }
        }
    }
}

void put32(std::vector<uint8_t>& v, uint32_t x) {
    for (int i = 0; i < 4; i++) v.push_back((uint8_t)(x >> (8 * i)));
}

struct Frame {
    uint32_t type;
    std::vector<uint8_t> plane[3];
};

void append_frame(std::vector<uint8_t>& file, const Frame& fr) {
    const uint32_t ys = (uint32_t)fr.plane[0].size(), cbs = (uint32_t)fr.plane[1].size(),
                   crs = (uint32_t)fr.plane[2].size();
    uint32_t size = ys + cbs + crs + 16;
    const uint32_t pad = (4 - size % 4) % 4;
    size += pad;
    put32(file, size);
    put32(file, fr.type);
    put32(file, ys);
    put32(file, cbs);
    for (int p = 0; p < 3; p++) file.insert(file.end(), fr.plane[p].begin(), fr.plane[p].end());
    file.insert(file.end(), pad, 0);
}

int finish_file(const char* path, std::vector<uint8_t>& file, uint32_t nframes, uint32_t w, uint32_t h,
                const std::vector<uint32_t>& iidx, const std::vector<uint32_t>& ipos) {
    const uint32_t payload = (uint32_t)(file.size() - 20);
    for (size_t i = 0; i < iidx.size(); i++) {
        put32(file, iidx[i]);
        put32(file, ipos[i]);
    }
    file.insert(file.end(), 512, 0);
    uint32_t hdr[5] = {nframes, w, h, (uint32_t)iidx.size(), payload};
    std::memcpy(file.data(), hdr, 20);
    FILE* fp = std::fopen(path, "wb");
    if (!fp) return -1;
    const bool ok = std::fwrite(file.data(), 1, file.size(), fp) == file.size();
    return (std::fclose(fp) == 0 && ok) ? 0 : -1;
}

}  // namespace

extern "C" {

// Bitstream of one plane (see encode_plane); returns its length, or -1 if cap is too small.
long mpg_synth_encode_plane(int nblocks, const int16_t* blocks, int P, uint8_t* out, size_t cap) {
    std::vector<uint8_t> v;
    encode_plane(nblocks, blocks, P != 0, v);
    if (v.size() > cap) return -1;
    std::memcpy(out, v.data(), v.size());
    return (long)v.size();
}

// Seeded content for nframes frames of w x h 4:4:4 (I-frame every `gop` frames):
// abs_out = absolute quantized coefficients, stream_out = the coded form (I absolute,
// P deltas), both [frame][Y | Cb | Cr] int16[64] blocks; types[f] = 0 (I) / 1 (P).
int mpg_synth_generate(uint32_t w, uint32_t h, uint32_t nframes, uint32_t gop, uint64_t seed, int16_t* abs_out,
                       int16_t* stream_out, uint8_t* types) {
    if (!w || !h || !gop) return -1;  // any size: the w/8 x h/8 whole blocks are coded
    const int nb = (int)((w / 8) * (h / 8));
    const size_t fs = (size_t)nb * 64 * 3;
    for (uint32_t f = 0; f < nframes; f++) {
        const bool P = (f % gop) != 0;
        types[f] = P ? 1 : 0;
        int16_t* a = abs_out + f * fs;
        if (P) std::memcpy(a, a - fs, fs * 2);
        for (int p = 0; p < 3; p++)
            gen_plane(seed, f, p, nb, P, a + (size_t)p * nb * 64, stream_out + f * fs + (size_t)p * nb * 64);
    }
    return 0;
}

// .mpg from explicit coded planes (I absolute / P deltas), [frame][Y | Cb | Cr].
int mpg_synth_write_coef(const char* path, uint32_t w, uint32_t h, uint32_t nframes, const uint8_t* types,
                         const int16_t* coef) {
    if (!w || !h || !nframes || types[0] != 0) return -1;
    const int nb = (int)((w / 8) * (h / 8));
    const size_t fs = (size_t)nb * 64 * 3;
    std::vector<uint8_t> file(20, 0);
    std::vector<uint32_t> iidx, ipos;
    for (uint32_t f = 0; f < nframes; f++) {
        Frame fr;
        fr.type = types[f];
        for (int p = 0; p < 3; p++) encode_plane(nb, coef + f * fs + (size_t)p * nb * 64, types[f] != 0, fr.plane[p]);
        if (!fr.type) {
            iidx.push_back(f);
            ipos.push_back((uint32_t)file.size());
        }
        append_frame(file, fr);
    }
    return finish_file(path, file, nframes, w, h, iidx, ipos);
}

// A whole seeded stream written straight to `path`, GOPs generated and encoded on up to
// `nthreads` host threads (<= 0: all); memory stays ~ one GOP of planes per thread.
// Returns the file size in bytes, or -1.
long long mpg_synth_write(const char* path, uint32_t w, uint32_t h, uint32_t nframes, uint32_t gop, uint64_t seed,
                          int nthreads) {
    if (!w || !h || !nframes || !gop) return -1;
    const int nb = (int)((w / 8) * (h / 8));
    const uint32_t ngops = (nframes + gop - 1) / gop;
    std::vector<std::vector<Frame>> gops(ngops);
    std::atomic<uint32_t> next{0};
    auto worker = [&]() {
        std::vector<int16_t> st((size_t)nb * 64), co((size_t)nb * 64);
        for (uint32_t gi; (gi = next.fetch_add(1)) < ngops;) {
            const uint32_t f0 = gi * gop, f1 = std::min(nframes, f0 + gop);
            std::vector<Frame>& out = gops[gi];
            out.resize(f1 - f0);
            for (int p = 0; p < 3; p++)
                for (uint32_t f = f0; f < f1; f++) {
                    const bool P = f != f0;
                    gen_plane(seed, f, p, nb, P, st.data(), co.data());
                    out[f - f0].type = P ? 1 : 0;
                    encode_plane(nb, co.data(), P, out[f - f0].plane[p]);
                }
        }
    };
    int nt = nthreads > 0 ? nthreads : (int)std::thread::hardware_concurrency();
    nt = std::max(1, std::min<int>(nt, (int)ngops));
    std::vector<std::thread> pool;
    for (int i = 1; i < nt; i++) pool.emplace_back(worker);
    worker();
    for (auto& t : pool) t.join();
    std::vector<uint8_t> file(20, 0);
    std::vector<uint32_t> iidx, ipos;
    for (uint32_t gi = 0; gi < ngops; gi++)
        for (size_t i = 0; i < gops[gi].size(); i++) {
            if (!gops[gi][i].type) {
                iidx.push_back(gi * gop + (uint32_t)i);
                ipos.push_back((uint32_t)file.size());
            }
            append_frame(file, gops[gi][i]);
            gops[gi][i] = Frame{};
        }
    if (finish_file(path, file, nframes, w, h, iidx, ipos) != 0) return -1;
    return (long long)file.size();
}

}  // extern "C"
