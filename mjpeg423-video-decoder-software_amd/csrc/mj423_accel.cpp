// mj423_accel.cpp -- the reference's asynchronous accelerator API
// (core0/software/idct_ycbcr_to_rgb_accel.h:13-22, .c:52-122) re-implemented over
// one HIP stream.
//
// Reference mechanics -> MI355X mechanics:
//   3 mSGDMA MM->ST input channels (Y, Cb, Cr dct_block_t arrays)
//        -> hipMemcpyAsync H2D into a device frame buffer [Y | Cb | Cr]
//   FPGA IDCT + CSC core (RTL not in the repo)
//        -> the fused decode kernel (input already dequantized: unit table)
//   1 ST->MM output channel into the display buffer
//        -> hipMemcpyAsync D2H of the BGRA frame
//   CSR busy polling (wait_for_*_finsh)
//        -> hipEventSynchronize on the event recorded after the matching copy
// The firmware calls cb, cr, y, get_results, wait_y, wait_rgb in that order
// (c0/playback.c:71-121).  A frame is the set of four submissions {Y, Cb, Cr, output}:
//   * ycbcr_to_rgb_accel_get_results() ends the frame once any plane of it has been
//     submitted (the reference's order); issued before any plane it is an early request
//     and the frame ends with its third plane (output-first order);
//   * a submission that fails (NULL, oversized, a failed copy) still takes its slot and
//     marks the frame failed: the frame is dropped at its end, nothing of it is decoded;
//   * a plane submitted twice in one frame abandons the incomplete frame (an error) and
//     starts the next one with it; get_results with a plane missing drops the frame.
// So a rejected plane can never pair the remaining planes of frame N with frame N+1's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <mutex>
#include <vector>
#include <string>

#include "../../include/mj423gpu.h"
#include "mj423_internal.h"

namespace {

struct Accel {
    std::mutex mu;
    mj423_ctx* ctx = nullptr;
    uint32_t w = 640, h = 480;  // c0/common/config.h:23-24
    int chroma = MJ423_CHROMA_444;
    mj423_geometry_t g{};
    int16_t* d_coef = nullptr;  // [Y | Cb | Cr]
    rgb_pixel_t* d_out = nullptr;
    uint8_t* d_blocks = nullptr;  // ycbcr_to_rgb_accel_calculate_buffer staging
    size_t d_blocks_cap = 0;
    bool have[3] = {false, false, false};  // slots of the current frame (a failed submission takes its slot too)
    void* out_host = nullptr;
    uint32_t out_bytes = 0;
    bool out_requested = false;
    bool failed = false;  // a submission of the current frame failed: the frame is dropped at its end
    hipEvent_t ev_y = nullptr, ev_out = nullptr;
    bool y_pending = false, out_pending = false;
    // Sticky failure (mj423_accel_status): the first error since the status was last read.
    // The reference's calls return void, so a failed submission cannot report itself; the
    // frame it belonged to is dropped (nothing stays pending) and the error waits here.
    int status = MJ423_OK;
    std::string status_msg;
};
Accel g_acc;

hipStream_t stream() { return (hipStream_t)mj423_ctx_stream(g_acc.ctx); }

// Starts an empty frame (caller holds g_acc.mu).
void reset_frame() {
    g_acc.have[0] = g_acc.have[1] = g_acc.have[2] = false;
    g_acc.out_requested = false;
    g_acc.failed = false;
}

// Records a failure (caller holds g_acc.mu): this thread's mj423_last_error() and, if no
// earlier failure is pending, the sticky status.  The current frame is marked failed; the
// caller decides whether its slot is taken (a rejected submission) or the frame ends now.
void note(int code, const std::string& msg) {
    mj423_set_error(code, "accelerator: " + msg);
    if (g_acc.status == MJ423_OK) {
        g_acc.status = code;
        g_acc.status_msg = "accelerator: " + msg;
    }
    g_acc.failed = true;
}
// Records a failure of a call outside the frame's four submissions (the CSC-only entry):
// the frame being assembled is left as it is.
void record(int code, const std::string& msg) {
    const bool f = g_acc.failed;
    note(code, msg);
    g_acc.failed = f;
}
// A failure that ends the frame at once (launch / copy / event errors, calls before init).
void fail(int code, const std::string& msg) {
    note(code, msg);
    reset_frame();
}
void fail_hip(const char* what, hipError_t e) { fail(MJ423_EHIP, std::string(what) + ": " + hipGetErrorString(e)); }

void free_buffers() {
    if (g_acc.d_coef) (void)hipFree(g_acc.d_coef);
    if (g_acc.d_out) (void)hipFree(g_acc.d_out);
    if (g_acc.d_blocks) (void)hipFree(g_acc.d_blocks);
    g_acc.d_coef = nullptr;
    g_acc.d_out = nullptr;
    g_acc.d_blocks = nullptr;
    g_acc.d_blocks_cap = 0;
}

bool alloc_buffers() {
    free_buffers();
    if (mj423_geometry(g_acc.w, g_acc.h, g_acc.chroma, &g_acc.g) != 0) return false;
    if (hipMalloc(&g_acc.d_coef, g_acc.g.coef_per_frame * 2) != hipSuccess) return false;
    if (hipMalloc(&g_acc.d_out, (size_t)g_acc.w * g_acc.h * 4) != hipSuccess) return false;
    return true;
}

size_t plane_offset(int plane) {  // int16 elements
    return plane == 0 ? 0 : plane == 1 ? 64ull * g_acc.g.y_blocks : 64ull * (g_acc.g.y_blocks + g_acc.g.c_blocks);
}
size_t plane_bytes(int plane) { return 128ull * (plane == 0 ? g_acc.g.y_blocks : g_acc.g.c_blocks); }

// Ends the frame if all four slots are taken: a failed frame is dropped, a clean one decoded.
void maybe_launch() {
    if (!(g_acc.have[0] && g_acc.have[1] && g_acc.have[2] && g_acc.out_requested)) return;
    if (g_acc.failed) return reset_frame();  // its error is already recorded
    mj423_frames_desc_t d = {g_acc.d_coef,
                             g_acc.d_coef + plane_offset(1),
                             g_acc.d_coef + plane_offset(2),
                             g_acc.g.coef_per_frame,
                             g_acc.d_out,
                             (uint64_t)g_acc.w * g_acc.h,
                             g_acc.w,
                             1,
                             g_acc.w,
                             g_acc.h,
                             g_acc.chroma,
                             MJ423_INPUT_DEQUANTIZED};
    const int rc = mj423_decode_frames_device(g_acc.ctx, &d);
    if (rc != 0) return fail(rc, std::string("decode launch failed: ") + mj423_last_error());
    // The output channel moves sizeOfOutputBuffer bytes at most (a smaller display buffer
    // receives the frame's first bytes, like the reference's length-limited DMA).
    const size_t n = std::min((size_t)g_acc.out_bytes, (size_t)g_acc.w * g_acc.h * 4);
    hipError_t e = hipMemcpyAsync(g_acc.out_host, g_acc.d_out, n, hipMemcpyDeviceToHost, stream());
    if (e != hipSuccess) return fail_hip("result copy", e);
    if ((e = hipEventRecord(g_acc.ev_out, stream())) != hipSuccess) return fail_hip("result event", e);
    g_acc.out_pending = true;
    reset_frame();
}

void submit_plane(int plane, void* in, uint32_t bytes) {
    static const char* kName[3] = {"Y", "Cb", "Cr"};
    std::lock_guard<std::mutex> lk(g_acc.mu);
    if (!g_acc.ctx) return fail(MJ423_ESTATE, "init_idct_ycbcr_to_rgb_accel() has not succeeded");
    if (g_acc.have[plane]) {  // the frame before never completed: drop it, this plane opens the next one
        if (!g_acc.failed)
            note(MJ423_ESTATE, std::string(kName[plane]) + " submitted twice before ycbcr_to_rgb_accel_get_results(); "
                               "the incomplete frame was dropped");
        reset_frame();
    }
    g_acc.have[plane] = true;  // taken even when rejected below: the frame then ends as a failed one
    const size_t cap = plane_bytes(plane);
    if (!in) note(MJ423_EINVAL, std::string(kName[plane]) + " input buffer is NULL");
    else if (bytes > cap)  // rejected, never truncated
        note(MJ423_EINVAL, std::string(kName[plane]) + " input of " + std::to_string(bytes) +
                               " bytes is larger than the plane (" + std::to_string(cap) + " bytes)");
    else if (!g_acc.failed) {  // a failed frame's planes are not uploaded
        hipError_t e = hipMemcpyAsync(g_acc.d_coef + plane_offset(plane), in, bytes, hipMemcpyHostToDevice, stream());
        if (e != hipSuccess) return fail_hip("input copy", e);
        if (plane == 0) {
            if ((e = hipEventRecord(g_acc.ev_y, stream())) != hipSuccess) return fail_hip("input event", e);
            g_acc.y_pending = true;
        }
    }
    maybe_launch();
}

}  // namespace

extern "C" {

int mj423_accel_configure(uint32_t w, uint32_t h, int chroma) {
    std::lock_guard<std::mutex> lk(g_acc.mu);
    mj423_geometry_t g;
    if (mj423_geometry(w, h, chroma, &g) != 0) return MJ423_EINVAL;
    g_acc.w = w;
    g_acc.h = h;
    g_acc.chroma = chroma;
    reset_frame();
    if (g_acc.ctx) {
        (void)mj423_ctx_synchronize(g_acc.ctx);
        if (!alloc_buffers()) {
            fail(MJ423_ENOMEM, "device buffers for the new geometry");
            return MJ423_ENOMEM;
        }
    }
    return MJ423_OK;
}

// Reference returns 1 on success (accel.c:63-83; convention c0/key_controls.c:49-52).
int init_idct_ycbcr_to_rgb_accel(void) {
    std::lock_guard<std::mutex> lk(g_acc.mu);
    if (g_acc.ctx) return 1;
    if (mj423_ctx_create(&g_acc.ctx, -1) != 0) return 0;
    if (hipEventCreateWithFlags(&g_acc.ev_y, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&g_acc.ev_out, hipEventDisableTiming) != hipSuccess || !alloc_buffers()) {
        free_buffers();
        mj423_ctx_destroy(g_acc.ctx);
        g_acc.ctx = nullptr;
        return 0;
    }
    return 1;
}

void mj423_accel_shutdown(void) {
    std::lock_guard<std::mutex> lk(g_acc.mu);
    if (!g_acc.ctx) return;
    (void)mj423_ctx_synchronize(g_acc.ctx);
    free_buffers();
    if (g_acc.ev_y) (void)hipEventDestroy(g_acc.ev_y);
    if (g_acc.ev_out) (void)hipEventDestroy(g_acc.ev_out);
    g_acc.ev_y = g_acc.ev_out = nullptr;
    mj423_ctx_destroy(g_acc.ctx);
    g_acc.ctx = nullptr;
    reset_frame();
    g_acc.y_pending = g_acc.out_pending = false;
}

void idct_accel_calculate_buffer_y(void* inputBuffer, uint32_t sizeOfInputBuffer) {
    submit_plane(0, inputBuffer, sizeOfInputBuffer);
}
void idct_accel_calculate_buffer_cb(void* inputBuffer, uint32_t sizeOfInputBuffer) {
    submit_plane(1, inputBuffer, sizeOfInputBuffer);
}
void idct_accel_calculate_buffer_cr(void* inputBuffer, uint32_t sizeOfInputBuffer) {
    submit_plane(2, inputBuffer, sizeOfInputBuffer);
}

void ycbcr_to_rgb_accel_get_results(void* outputBuffer, uint32_t sizeOfOutputBuffer) {
    std::lock_guard<std::mutex> lk(g_acc.mu);
    if (!g_acc.ctx) return fail(MJ423_ESTATE, "init_idct_ycbcr_to_rgb_accel() has not succeeded");
    const bool any_plane = g_acc.have[0] || g_acc.have[1] || g_acc.have[2];
    if (!outputBuffer) return fail(MJ423_EINVAL, "output buffer is NULL");
    if (g_acc.out_requested) {  // a second request before the planes completed the first frame
        if (!g_acc.failed) note(MJ423_ESTATE, "ycbcr_to_rgb_accel_get_results() called twice; the incomplete frame was dropped");
        reset_frame();
    }
    g_acc.out_host = outputBuffer;
    g_acc.out_bytes = sizeOfOutputBuffer;
    g_acc.out_requested = true;
    if (any_plane && !(g_acc.have[0] && g_acc.have[1] && g_acc.have[2])) {  // the reference's frame end, planes missing
        if (!g_acc.failed) note(MJ423_ESTATE, "ycbcr_to_rgb_accel_get_results() with a plane missing; the frame was dropped");
        return reset_frame();
    }
    maybe_launch();  // no plane yet: an early request, the frame ends with its third plane
}

void ycbcr_to_rgb_accel_calculate_buffer(color_block_t* yBlock, color_block_t* crBlock, color_block_t* cbBlock,
                                         rgb_pixel_t* outputBuffer, int hCb_size, int wCb_size, int w_size) {
    std::lock_guard<std::mutex> lk(g_acc.mu);
    if (!g_acc.ctx) return record(MJ423_ESTATE, "init_idct_ycbcr_to_rgb_accel() has not succeeded");
    if (!yBlock || !crBlock || !cbBlock || !outputBuffer || hCb_size <= 0 || wCb_size <= 0 || w_size < 8 * wCb_size)
        return record(MJ423_EINVAL, "ycbcr_to_rgb_accel_calculate_buffer: bad arguments");
    // CSC over hCb x wCb blocks into a frame of row pitch w_size (HOT LOOP 2,
    // mj/decoder/mjpeg423_decoder.c:120-124).  Runs on the accelerator stream and
    // completes under wait_for_ycbcr_to_rgb_finsh().
    const uint32_t fw = 8u * (uint32_t)wCb_size, fh = 8u * (uint32_t)hCb_size;
    std::vector<rgb_pixel_t> tmp((size_t)fw * fh);
    const int rc = mj423_ycbcr_to_rgb_444(g_acc.ctx, fw, fh, &yBlock[0][0][0], &cbBlock[0][0][0], &crBlock[0][0][0],
                                          tmp.data());
    if (rc != 0) return record(rc, std::string("colour conversion failed: ") + mj423_last_error());
    for (uint32_t y = 0; y < fh; y++)
        std::memcpy(outputBuffer + (size_t)y * (uint32_t)w_size, tmp.data() + (size_t)y * fw, fw * sizeof(rgb_pixel_t));
}

void wait_for_ycbcr_to_rgb_finsh(void) {
    std::lock_guard<std::mutex> lk(g_acc.mu);
    if (g_acc.ctx && g_acc.out_pending) {
        const hipError_t e = hipEventSynchronize(g_acc.ev_out);
        g_acc.out_pending = false;
        if (e != hipSuccess) fail_hip("result", e);
    }
    // a frame that failed never became pending: repeat its error for this thread
    if (g_acc.status != MJ423_OK) mj423_set_error(g_acc.status, g_acc.status_msg);
}

void wait_for_idct_y_finsh(void) {
    std::lock_guard<std::mutex> lk(g_acc.mu);
    if (g_acc.ctx && g_acc.y_pending) {
        const hipError_t e = hipEventSynchronize(g_acc.ev_y);
        g_acc.y_pending = false;
        if (e != hipSuccess) fail_hip("Y input", e);
    }
    if (g_acc.status != MJ423_OK) mj423_set_error(g_acc.status, g_acc.status_msg);
}

int mj423_accel_status(void) {
    std::lock_guard<std::mutex> lk(g_acc.mu);
    const int st = g_acc.status;
    if (st != MJ423_OK) mj423_set_error(st, g_acc.status_msg);
    g_acc.status = MJ423_OK;
    g_acc.status_msg.clear();
    return st;
}

}  // extern "C"
