// mj423_margin.hip -- the defined fill outside an .mpg frame's coded region.
//
// The reference codes and decodes only the w/8 x h/8 whole blocks of a w x h frame
// (mjpeg423_encoder.c:21-24, mjpeg423_decoder.c:45-48,120-124) and writes a w x h BMP whose
// remaining right columns and bottom rows it never sets (uninitialised malloc memory,
// mjpeg423_decoder.c:55).  The library sets them to zero: BGRA {0, 0, 0, 0}.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mj423_internal.h"

namespace {
// One lane per margin pixel of a frame: the right strip [cw, w) of rows [0, ch), then the
// bottom rows [ch, h) whole; frames along grid y (strided past 65535).
__global__ void __launch_bounds__(256) fill_margin_kernel(uint32_t* out, uint64_t frame_stride, uint32_t pitch,
                                                          uint32_t cw, uint32_t ch, uint32_t w, uint32_t h,
                                                          uint32_t nframes) {
    const uint64_t strip = (uint64_t)ch * (w - cw), total = strip + (uint64_t)(h - ch) * w;
    const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= total) return;
    uint64_t x, y;
    if (i < strip) {
        y = i / (w - cw);
        x = cw + i % (w - cw);
    } else {
        y = ch + (i - strip) / w;
        x = (i - strip) % w;
    }
    for (uint32_t f = blockIdx.y; f < nframes; f += gridDim.y) out[f * frame_stride + y * pitch + x] = 0u;
}
}  // namespace

int mj423_launch_fill_margin(rgb_pixel_t* out, uint64_t frame_stride, uint32_t pitch, uint32_t cw, uint32_t ch,
                             uint32_t w, uint32_t h, uint32_t nframes, void* stream) {
    if (nframes == 0 || (cw >= w && ch >= h)) return (int)hipSuccess;
    if (!out || cw > w || ch > h || pitch < w) return (int)hipErrorInvalidValue;
    // every frame's rows inside its stride (the kernel writes [f * frame_stride, f * frame_stride + (h-1) * pitch + w))
    if (nframes > 1 && (uint64_t)(h - 1) * pitch + w > frame_stride) return (int)hipErrorInvalidValue;
    const uint64_t total = (uint64_t)ch * (w - cw) + (uint64_t)(h - ch) * w;
    const dim3 grid((uint32_t)((total + 255) / 256), nframes < 65535u ? nframes : 65535u);
    hipLaunchKernelGGL(fill_margin_kernel, grid, dim3(256), 0, (hipStream_t)stream, reinterpret_cast<uint32_t*>(out),
                       frame_stride, pitch, cw, ch, w, h, nframes);
    return (int)hipGetLastError();
}
