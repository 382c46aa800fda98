// mj423_kernels.h -- parameter blocks shared by the HIP kernels and the C-ABI runtime.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mj423 {

constexpr uint32_t kFgroupXcd = 0xffffffffu;  // DecodeParams::fgroup: XCD-contiguous workgroup order
constexpr uint32_t kGopOrderEighths = 2;      // DecodeParams::gop_order: each XCD one eighth of every segment

// Fused decode of `nframes` frames, one tile per workgroup.  4:2:0: a tile is a run of
// <= TW MCUs inside one MCU row.  4:2:2 / 4:4:4: a tile is a run of TW consecutive MCUs
// in raster order, wrapping across MCU rows (an MCU's blocks sit in one block row, so
// the run is contiguous in every plane).  Passed by value as the kernel argument.
struct DecodeParams {
    const int16_t* coef;       // luma plane of frame 0 (block-raster, int16[64] per block)
    int64_t cb_off, cr_off;    // chroma planes, in int16 elements relative to coef
    uint64_t plane_fstride;    // int16 elements between consecutive frames of a plane
    uint32_t* out;             // BGRA frame 0
    uint64_t out_fstride;      // pixels between consecutive output frames
    uint32_t out_pitch;        // pixels between output rows
    uint32_t aligned16;        // out and out_pitch allow 16-B stores
    uint32_t width, height;    // displayed size (crop of the coded MCU grid)
    uint32_t y_bw, c_bw;       // blocks per row: luma / chroma plane
    uint32_t mcu_cols, mcu_rows;
    uint32_t tiles_per_row, tw;  // tw = MCUs per tile (<= TWMAX); tiles_per_row: 4:2:0 only
    uint32_t tiles_per_frame;  // 4:2:0: mcu_rows * tiles_per_row; else ceil(mcu_cols * mcu_rows / tw)
    uint32_t mcus_per_frame;   // mcu_cols * mcu_rows
    uint32_t cols_magic;       // floor(2^32 / mcu_cols): MCU index -> (row, col) with one correction step
    uint32_t ntiles;           // nframes * tiles_per_frame
    uint32_t fgroup;           // batch kernel workgroup order: fgroup (> 1) consecutive workgroups take
                               // one tile position in fgroup consecutive frames; 0/1: frame-major;
                               // kFgroupXcd: one contiguous eighth of the batch per XCD
    uint32_t qt[2][32];        // [0] luma, [1] chroma: natural-order table as packed int16 pairs
    // stream mode (decode_gop_kernel) only
    const uint32_t* qt_dev;    // qt on the device (same packing), for the stream kernel
    const uint8_t* ftype;      // per frame: 0 = I (absolute), 1 = P (deltas)
    const uint32_t* seg_start; // nseg + 1 frame indices; every segment but the first starts at an I-frame
    const int16_t* state;      // absolute coefficients before frame 0 (read if frame 0 is P)
    int16_t* state_out;        // absolute coefficients after the last frame (optional)
    int64_t st_cb_off, st_cr_off;  // chroma planes inside the state buffers (int16 elements)
    uint32_t* jobflag;         // stream kernel, per (segment, tile) job: the optimistic form sets 1 when it cannot
                               // guarantee exact output (int8 state overflow, a block too wide for the int16 IDCT);
                               // the exact form with kGopFixup re-runs exactly the flagged jobs and clears them
    unsigned long long* reruns;  // kGopFixup: jobs re-run, 64-bit (one vector atomic per re-run job; optional)
    uint32_t nseg;             // segments (GOP runs) in seg_start
    uint32_t gop_order;        // stream kernel workgroup order: 0 = grid (tiles, nseg); kGopOrderEighths =
                               // XCD x the x-th eighth of every segment's tiles; kFgroupXcd = one
                               // contiguous range of the (segment, tile) jobs per XCD (1-D grids)
};

// Sparse-to-dense expansion of a streaming-decoder transfer buffer (mj423_pipeline.cpp).
// Tasks = (frame, plane) pairs, task t = 3 * frame + plane.  Layout of `xfer` (device):
//   task_base[ntask]  uint32  first entry word of the task (16-B aligned)
//   task_mode[ntask]  uint32  0 sparse, 1 dense (the plane's int16 coefficients verbatim)
//   seg_off[ntask][nseg+1] uint32  entries before each 256-block segment (sparse tasks)
//   counts[ntask][nblk]    uint8   coefficients per block (sparse tasks)
//   entries (at entries_off bytes)  uint32: natural index << 16 | uint16 value
struct ExpandParams {
    const uint8_t* xfer;
    uint64_t off_mode, off_seg, off_counts, entries_off;  // bytes from xfer
    uint32_t ntask, nblk, nseg;
    int16_t* out;           // dense [frame][Y | Cb | Cr] planes
    uint64_t coef_pf;       // int16 per frame
};

// GPU entropy front end (mj423_kernels.hip entropy_kernel): one lane per (frame, plane)
// bitstream of an .mpg already in device memory.  Output: the frame's plane in the
// stream-decode input form (I-frames absolute quantized coefficients, DC prefix-summed;
// P-frames their deltas) written into a ZEROED dense plane.
struct EntropyTask {
    uint64_t byte_off;  // first byte of the plane's bitstream in `bytes`
    uint32_t nbytes;    // its length (bits past it read as zero, like the bounded host reader)
    uint32_t frame;     // output frame index (within the launch's coefficient buffer)
    uint32_t plane;     // 0 Y, 1 Cb, 2 Cr
    uint32_t ptype;     // 0 I, 1 P
};
struct EntropyParams {
    const uint8_t* bytes;  // device copy of the stream bytes; readable up to 16 B past bytes_len
    uint64_t bytes_len;
    const EntropyTask* tasks;
    uint32_t ntasks;
    uint32_t nblk;         // blocks per plane (4:4:4)
    int16_t* out;          // [frame][Y | Cb | Cr] dense planes, zero-filled beforehand
    uint64_t coef_pf;      // int16 per frame
    uint32_t* status;      // per task: 0 ok, 1 the blocks needed bits past the stream's end, 2 runaway stream
    // Fallback use behind the many-lanes front end (mj423_entropy.hip): decode only tasks with
    // tchg[t] == unsettled, clearing their plane first; tchg == nullptr: every task, planes
    // already zero-filled.
    const uint32_t* tchg;
    uint32_t unsettled;
};

struct SynthParams {
    int16_t* coef;             // [frame][Y | Cb | Cr] blocks
    uint64_t frame_stride;     // int16 elements per frame
    uint32_t y_blocks, c_blocks;
    uint32_t nframes;
    uint64_t frame0;           // global index of the first frame (rank sharding)
    uint64_t seed;
    int16_t yq[64], cq[64];    // natural-order quant tables (AC clip |Q*q| <= 1023)
    int32_t zigzag[64];
    uint32_t ac_thresh[64];    // P(AC at zig-zag k != 0) * 2^32
};

// One deferred ycbcr_to_rgb() call (mj423_dropin.cpp): the colour-block slots of its Y, Cb
// and Cr inputs (64 B each in the flush's block buffer) and where its 8x8 BGRA pixels go
// (pixel offset of the top-left corner, row pitch in pixels; 16-B aligned rows).
struct DropinCsc {
    uint32_t sy, scb, scr, pitch;
    uint64_t off, pad;
};

}  // namespace mj423

extern "C" {
hipError_t mj423_launch_decode(const mj423::DecodeParams* p, uint32_t nframes, int chroma, hipStream_t stream);
int mj423_tile_max_mcus(int chroma);
int mj423_gop_tile_max_mcus(int chroma);  // same, for the stream (GOP) kernel
uint32_t mj423_batch_fgroup(int chroma, uint32_t tiles_per_frame);  // DecodeParams::fgroup for the batch kernel
hipError_t mj423_launch_decode_gop(const mj423::DecodeParams* p, uint32_t nseg, int chroma, hipStream_t stream);
hipError_t mj423_launch_idct_blocks(const int16_t* in, uint8_t* out, uint32_t n, const uint32_t* qt,
                                    hipStream_t stream);
hipError_t mj423_launch_csc444(const uint8_t* Y, const uint8_t* Cb, const uint8_t* Cr, uint32_t* rgb,
                               uint32_t w_size, uint32_t h_size, uint32_t out_pitch, hipStream_t stream);
hipError_t mj423_launch_synth(const mj423::SynthParams* p, hipStream_t stream);
// bytes rounded up to 16; src/dst 16-B aligned (device or host-mapped pointers)
hipError_t mj423_launch_copy16(const void* src, void* dst, uint64_t bytes, hipStream_t stream);
// One block for idct() (op 0) / ycbcr_to_rgb() (op 1) on host-mapped buffers; stores seq into
// *done (host-mapped) once the result is visible to the host.
hipError_t mj423_launch_dropin_block(int op, const uint8_t* in, uint8_t* out, uint32_t* done, uint32_t seq,
                                     hipStream_t stream);
// The deferred ycbcr_to_rgb() calls of one flush: n records, colour blocks in `col`.
hipError_t mj423_launch_dropin_csc(const uint8_t* col, const mj423::DropinCsc* calls, uint32_t n, uint32_t* rgb,
                                   hipStream_t stream);
hipError_t mj423_launch_expand(const mj423::ExpandParams* p, hipStream_t stream);
hipError_t mj423_launch_entropy(const mj423::EntropyParams* p, hipStream_t stream);
}
