// mj423_gpu_frontend.cpp -- whole-GPU .mpg decode (include/mj423io.h, mj423_mpg_decode_gpu):
// the frames' bitstreams go to HBM once; entropy_kernel decodes every (frame, plane)
// stream on its own lane into per-frame delta planes; decode_gop_kernel accumulates the
// P-frames on chip and runs dequant + IDCT + CSC.  No coefficient crosses PCIe and no
// host thread decodes bits, so the batch is as parallel as it has streams (3 per frame).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/mj423io.h"
#include "mj423_internal.h"
#include "mj423_kernels.h"

namespace {

struct DevMem {  // hipFree on scope exit
    void* p = nullptr;
    ~DevMem() {
        if (p) (void)hipFree(p);
    }
};

}  // namespace

extern "C" int mj423_mpg_decode_gpu(mj423_ctx* ctx, const mj423_mpg* m, uint32_t first, uint32_t count,
                                    rgb_pixel_t* d_out, uint64_t out_frame_stride, uint32_t window_frames) {
    return mj423_guarded([&]() -> int {
        if (!ctx || !m || (!d_out && count)) return mj423_set_error(MJ423_EINVAL, "decode_gpu: null argument");
        mj423_mpg_header_t hdr;
        if (int rc = mj423_mpg_header(m, &hdr)) return rc;
        if ((uint64_t)first + count > hdr.num_frames) return mj423_set_error(MJ423_EINVAL, "decode_gpu: frame range out of range");
        if (count == 0) return 0;
        const uint32_t w = hdr.width, h = hdr.height;
        if (out_frame_stride < (uint64_t)w * h) return mj423_set_error(MJ423_EINVAL, "decode_gpu: out_frame_stride < w*h");
        mj423_geometry_t g;
        if (int rc = mj423_geometry(w, h, MJ423_CHROMA_444, &g)) return rc;
        const uint64_t coef_pf = g.coef_per_frame;
        const uint32_t nblk = g.y_blocks;
        if (nblk >= (1u << 26))  // the kernel forms plane positions 64 * block + index in 32 bits
            return mj423_set_error(MJ423_EINVAL, "decode_gpu: more than 2^26 blocks per plane");
        // Default window: as many frames as half the free HBM holds in dense delta planes (at
        // most 64 GiB).  A launch lasts as long as its longest stream (an I-frame plane), so
        // the more frames share it, the faster the batch: 1080p 4:4:4 is ~12 MB per frame,
        // so a whole file of a few thousand frames decodes in one window.
        uint64_t budget = 4ull << 30;
        if (!window_frames) {
            size_t free_b = 0, total_b = 0;
            int cur = -1;
            (void)hipGetDevice(&cur);
            if (hipSetDevice(mj423_ctx_device_id(ctx)) == hipSuccess && hipMemGetInfo(&free_b, &total_b) == hipSuccess)
                budget = std::max<uint64_t>(budget, std::min<uint64_t>(free_b / 2, 64ull << 30));
            if (cur >= 0) (void)hipSetDevice(cur);
        }
        const uint32_t win = window_frames ? window_frames : (uint32_t)std::max<uint64_t>(1, budget / (coef_pf * 2));
        const uint32_t wf = std::min(win, count);

        // frame table and the byte range [b0, b1) holding frames first .. first+count-1
        std::vector<mj423_mpg_frame_t> fr(count);
        for (uint32_t i = 0; i < count; i++)
            if (int rc = mj423_mpg_frame(m, first + i, &fr[i])) return rc;
        const uint64_t b0 = fr[0].position, b1 = fr[count - 1].position + fr[count - 1].frame_size;
        const uint8_t* host0 = fr[0].y - 16;  // the mapped file at b0

        const int dev = mj423_ctx_device_id(ctx);
        int prev = -1;
        (void)hipGetDevice(&prev);
        struct Restore {
            int d;
            ~Restore() {
                if (d >= 0) (void)hipSetDevice(d);
            }
        } restore{prev};
        if (hipSetDevice(dev) != hipSuccess) return mj423_set_error(MJ423_EHIP, "decode_gpu: hipSetDevice failed");
        hipStream_t s = (hipStream_t)mj423_ctx_stream(ctx);
        auto hipok = [&](hipError_t e, const char* what) {
            return e == hipSuccess ? 0 : mj423_set_error(MJ423_EHIP, std::string("decode_gpu: ") + what + ": " + hipGetErrorString(e));
        };
        DevMem d_bytes, d_coef, d_tasks, d_status, d_state[2];
        const uint64_t nbytes = b1 - b0;
        if (int rc = hipok(hipMalloc(&d_bytes.p, nbytes + 64), "hipMalloc")) return rc;
        if (int rc = hipok(hipMalloc(&d_coef.p, (size_t)wf * coef_pf * 2), "hipMalloc")) return rc;
        if (int rc = hipok(hipMalloc(&d_tasks.p, (size_t)count * 3 * sizeof(mj423::EntropyTask)), "hipMalloc")) return rc;
        if (int rc = hipok(hipMalloc(&d_status.p, (size_t)count * 3 * 4), "hipMalloc")) return rc;
        for (auto& st : d_state)
            if (int rc = hipok(hipMalloc(&st.p, coef_pf * 2), "hipMalloc")) return rc;
        if (int rc = hipok(hipMemcpyAsync(d_bytes.p, host0, nbytes, hipMemcpyHostToDevice, s), "upload")) return rc;
        // tasks: every (frame, plane) of the range, frame index relative to its window
        std::vector<mj423::EntropyTask> tasks((size_t)count * 3);
        std::vector<uint8_t> types(count);
        for (uint32_t i = 0; i < count; i++) {
            types[i] = (uint8_t)fr[i].frame_type;
            const uint64_t y0 = fr[i].position + 16 - b0;
            const uint64_t off[3] = {y0, y0 + fr[i].y_size, y0 + fr[i].y_size + fr[i].cb_size};
            const uint32_t len[3] = {fr[i].y_size, fr[i].cb_size, fr[i].cr_size};
            if (std::max({len[0], len[1], len[2]}) >= (1u << 28))  // the kernel counts bits in 32 bits
                return mj423_set_error(MJ423_EINVAL, "decode_gpu: a plane bitstream of 256 MiB or more");
            for (int pl = 0; pl < 3; pl++) tasks[(size_t)i * 3 + pl] = {off[pl], len[pl], i % wf, (uint32_t)pl, types[i]};
        }
        if (int rc = hipok(hipMemcpyAsync(d_tasks.p, tasks.data(), tasks.size() * sizeof(tasks[0]),
                                          hipMemcpyHostToDevice, s), "upload"))
            return rc;
        // seeking into a GOP: absolute coefficients of frame first-1 seed the accumulation
        std::vector<int16_t> seed;
        if (types[0] != 0) {
            seed.resize(coef_pf);
            if (int rc = mj423_mpg_entropy_decode(m, first - 1, 1, seed.data(), 0)) return rc;
            if (int rc = hipok(hipMemcpyAsync(d_state[1].p, seed.data(), coef_pf * 2, hipMemcpyHostToDevice, s), "upload"))
                return rc;
        }
        for (uint32_t w0 = 0, k = 0; w0 < count; w0 += wf, k++) {
            const uint32_t n = std::min(wf, count - w0);
            if (int rc = hipok(hipMemsetAsync(d_coef.p, 0, (size_t)n * coef_pf * 2, s), "memset")) return rc;
            mj423::EntropyParams ep{};
            ep.bytes = (const uint8_t*)d_bytes.p;
            ep.bytes_len = nbytes;
            ep.tasks = (const mj423::EntropyTask*)d_tasks.p + (size_t)w0 * 3;
            ep.ntasks = n * 3;
            ep.nblk = nblk;
            ep.out = (int16_t*)d_coef.p;
            ep.coef_pf = coef_pf;
            ep.status = (uint32_t*)d_status.p + (size_t)w0 * 3;
            if (int rc = hipok(mj423_launch_entropy(&ep, s), "entropy kernel")) return rc;
            const int16_t* y = (const int16_t*)d_coef.p;
            mj423_frames_desc_t d = {y, y + 64ull * g.y_blocks, y + 64ull * (g.y_blocks + g.c_blocks), coef_pf,
                                     d_out + (size_t)w0 * out_frame_stride, out_frame_stride, w, n, w, h,
                                     MJ423_CHROMA_444, MJ423_INPUT_QUANTIZED};
            // window k reads d_state[(k+1)%2] (window k-1's end state, or the seek seed), writes d_state[k%2]
            const int16_t* st_in = types[w0] != 0 ? (const int16_t*)d_state[(k + 1) % 2].p : nullptr;
            if (int rc = mj423_decode_stream_device(ctx, &d, types.data() + w0, st_in, (int16_t*)d_state[k % 2].p))
                return rc;
        }
        std::vector<uint32_t> status((size_t)count * 3);
        if (int rc = hipok(hipMemcpyAsync(status.data(), d_status.p, status.size() * 4, hipMemcpyDeviceToHost, s), "status"))
            return rc;
        if (int rc = hipok(hipStreamSynchronize(s), "synchronize")) return rc;
        for (size_t i = 0; i < status.size(); i++)
            if (status[i])
                return mj423_set_error(MJ423_EINVAL, "mpg: frame " + std::to_string(first + i / 3) + " plane " +
                                                         std::to_string(i % 3) +
                                                         (status[i] == 1 ? ": bitstream ended before all of its blocks were decoded"
                                                                         : ": runaway bitstream"));
        return 0;
    });
}
