/*
 * mj423gpu.h -- C ABI of the MI355X (gfx950) MPEG423 decode hot path.
 *
 * Drop-in for the reference's per-block hot path
 *     dequantize -> 8x8 integer IDCT -> YCbCr->BGRA
 * of ghananigans/mjpeg423-video-decoder-software.  Reference paths below are
 * relative to core0/software/ (the "c0" firmware tree) and to
 * core0/software/common/libs/mjpeg423/ ("mj/", the portable codec library).
 *
 * Output is bit-exact to the reference's integer C code (mj/decoder/idct.c,
 * mj/decoder/ycbcr_to_rgb.c) for 4:4:4; 4:2:2 / 4:2:0 add the nearest-neighbour
 * chroma fetch of SURVEY.md §8 A7 (pixel (x,y) takes chroma (x/2, y/sy)).
 *
 * Four entry families, all plain C (no HIP / torch types):
 *   1. the reference's own per-block symbols  idct(), ycbcr_to_rgb()
 *   2. the frame call decode_frame() / decode_frames()  (host buffers)
 *   3. the reference's async accelerator API  (c0/idct_ycbcr_to_rgb_accel.h)
 *   4. device-resident batches  mj423_decode_frames_device()  (the fast path)
 *
 * Every int-returning mj423_* / decode_* call returns 0 on success or a negative
 * MJ423_E* code; mj423_last_error() describes the last failure of the calling
 * thread.  The reference's own void symbols cannot return errors (the reference
 * has none either); they record them in mj423_last_error().
 */
#ifndef MJ423GPU_H
#define MJ423GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------------------ types */
/* The reference's types (mj/common/mjpeg423_types.h:33-61).  Skipped when the
 * reference header (include guard mjpeg423app_mjpeg423_types_h) came first, so
 * the reference's decoder sources can include both. */
#ifndef mjpeg423app_mjpeg423_types_h
typedef uint8_t color_block_t[8][8];  /* types.h:33 */
typedef uint8_t (*pcolor_block_t)[8]; /* types.h:34 */
typedef int16_t dct_block_t[8][8];    /* types.h:42, DCTELEM = int16_t (:39) */
typedef int16_t (*pdct_block_t)[8];   /* types.h:43 */
typedef struct {
    uint8_t blue;
    uint8_t green;
    uint8_t red;
    uint8_t alpha;
} rgb_pixel_t;                        /* types.h:56-61 (BMP byte order) */
#endif

/* Chroma layouts; 444 is the reference's (mj/decoder/mjpeg423_decoder.c:45-48). */
#define MJ423_CHROMA_444 444
#define MJ423_CHROMA_422 422
#define MJ423_CHROMA_420 420

/* Input forms.  QUANTIZED: absolute quantized coefficients per block in natural
 * order (the quantized-domain output of the entropy front end);
 * the kernel computes (int16)(Q[k] * q[k]).  DEQUANTIZED: dct_block_t exactly as
 * the reference's lossless_decode leaves it (mj/decoder/lossless_decode.c:89-129)
 * and as the accelerator receives it (c0/playback.c:71-75,102). */
#define MJ423_INPUT_QUANTIZED   0
#define MJ423_INPUT_DEQUANTIZED 1

/* Error codes */
#define MJ423_OK          0
#define MJ423_EINVAL     -1 /* bad argument / geometry */
#define MJ423_EHIP       -2 /* HIP runtime error (message in mj423_last_error) */
#define MJ423_ENOMEM     -3 /* device or host allocation failed */
#define MJ423_ESTATE     -4 /* call out of order (accelerator API) */

/* Frame geometry: coded size rounds the displayed size up to whole MCUs
 * (8x8 / 16x8 / 16x16); planes are block-raster arrays of int16[64]. */
typedef struct {
    uint32_t width, height;    /* displayed pixels */
    int32_t chroma;            /* 444 / 422 / 420 */
    uint32_t mcu_w, mcu_h;
    uint32_t coded_w, coded_h;
    uint32_t y_bw, y_bh;       /* luma plane in blocks */
    uint32_t c_bw, c_bh;       /* each chroma plane in blocks */
    uint32_t y_blocks, c_blocks;
    uint64_t coef_per_frame;   /* int16 coefficients per frame, [Y | Cb | Cr] */
} mj423_geometry_t;

typedef struct mj423_ctx mj423_ctx;

/* -------------------------------------------------------- library / context */
int mj423_version(void);                      /* 0xMMmmpp */
const char *mj423_last_error(void);           /* thread-local, never NULL */
/* Pure host arithmetic: no GPU needed. */
int mj423_geometry(uint32_t width, uint32_t height, int chroma, mj423_geometry_t *g);
/* Algorithmic HBM bytes of one decoded frame: 2 B per coded coefficient read +
 * 4 B per displayed pixel written. */
uint64_t mj423_frame_bytes(uint32_t width, uint32_t height, int chroma);

/* device < 0: the current HIP device.  One context per host thread (or per GPU);
 * calls on one context are not thread-safe (the reference is single-threaded). */
int mj423_ctx_create(mj423_ctx **ctx, int device);
void mj423_ctx_destroy(mj423_ctx *ctx);
/* Work of this context is issued on `hip_stream` (a hipStream_t; NULL = the
 * context's own stream).  Lets a caller (e.g. torch) share its stream. */
int mj423_ctx_set_stream(mj423_ctx *ctx, void *hip_stream);
void *mj423_ctx_stream(mj423_ctx *ctx);
/* Quantization tables in natural order (mj/common/tables.c:13-32 layout);
 * NULL restores the reference's Yquant / Cquant.  In the reference they are
 * compile-time constants; here they are per-context state. */
int mj423_ctx_set_quant(mj423_ctx *ctx, const int16_t yquant[64], const int16_t cquant[64]);
int mj423_ctx_get_quant(mj423_ctx *ctx, int16_t yquant[64], int16_t cquant[64]);
/* Blocks until the context's stream is idle. */
int mj423_ctx_synchronize(mj423_ctx *ctx);
/* Kernel timing: when enabled, every fused decode launch of this context is
 * bracketed by HIP events on the stream it runs on; mj423_ctx_kernel_ms()
 * waits for the last bracketed launch and returns its device time (ms), or a
 * negative value if none was recorded. */
int mj423_ctx_enable_timing(mj423_ctx *ctx, int on);
double mj423_ctx_kernel_ms(mj423_ctx *ctx);
/* Frames decoded by that last bracketed launch (0 if none). */
uint32_t mj423_ctx_kernel_frames(mj423_ctx *ctx);
/* Every bracketed launch since timing was last enabled: the sum of their device
 * times (ms), of their frames, and their count (waits for them).  Up to 65536
 * launches are logged; past that it fails until timing is enabled again. */
int mj423_ctx_kernel_totals(mj423_ctx *ctx, double *ms, uint64_t *frames, uint32_t *launches);
/* Stream decode at 4:2:2 runs an optimistic kernel (int8 coefficient state, int16 IDCT
 * workspace) and then re-runs with the exact kernel every (GOP segment, tile) job in which
 * those widths did not hold.  Total jobs re-run by this context so far (waits for its
 * stream); results are exact either way, this only tells how often the slow path ran. */
int mj423_ctx_stream_reruns(mj423_ctx *ctx, uint64_t *jobs);

/* ------------------------------------------- 1. reference per-block symbols */
/* void idct(dct_block_t DCAC, color_block_t block)  -- mj/decoder/mjpeg423_decoder.h:16,
 * defined at mj/decoder/idct.c:22.  Caller-owned host buffers; immediate (one GPU launch per
 * call, the output written on return like the reference's C) or deferred (queued, decoded at
 * the thread's next flush point), see the modes below. */
void idct(dct_block_t DCAC, color_block_t block);
/* void ycbcr_to_rgb(...) -- mj/decoder/mjpeg423_decoder.h:15, mj/decoder/ycbcr_to_rgb.c:26.
 * Writes the 64 pixels of one 8x8 4:4:4 block at rgbblock[(h+y)*w_size + w + x]. */
void ycbcr_to_rgb(int h, int w, uint32_t w_size, pcolor_block_t Y, pcolor_block_t Cb,
                  pcolor_block_t Cr, rgb_pixel_t *rgbblock);
/* Extensions for the two symbols above (they return void, like the reference's):
 *   Modes (MJ423_DROPIN_DEFER=0|1|2 in the environment, or mj423_dropin_defer()):
 *     0 immediate: every call's output is in the caller's buffer when it returns.
 *     1 deferred: calls only queue (per thread); the queue is decoded in two launches and
 *       written to the callers' buffers, in call order, at the library's encode_bmp() or
 *       lossless_decode(), mj423_dropin_flush(), mj423_dropin_defer(0), when full, or at
 *       the thread's exit.
 *     2 adaptive (the default): immediate until the calling thread reaches the library's own
 *       lossless_decode() or encode_bmp() -- proof that its frame loop ends in a flush point,
 *       as the reference's does (mjpeg423_decoder.c:110-132, which calls one of them before it
 *       reads any output) -- and deferred on that thread from then on.  A caller that keeps
 *       the reference's lossless_decode() and libbmp stays synchronous; when deferral
 *       engages with the variable unset the library says so once on stderr.
 *   mj423_dropin_defer(mode): set the mode; returns the previous one (0/1/2) or an MJ423_E*
 *     code if the flush it implies failed.
 *   mj423_dropin_flush(): decode and write this thread's queued calls now.
 *   mj423_dropin_status(): first MJ423_E* failure of these symbols since the last call
 *     (read-and-clear; MJ423_OK if none), its message in mj423_last_error(). */
int mj423_dropin_defer(int on);
int mj423_dropin_flush(void);
int mj423_dropin_status(void);

/* The two HOT LOOPs of mj/decoder/mjpeg423_decoder.c as batched calls (host buffers):
 *   mj423_idct_blocks      : :115-117, n blocks; quant == NULL means DCAC is already
 *                            dequantized (the reference's form)
 *   mj423_ycbcr_to_rgb_444 : :120-124, block-raster Y/Cb/Cr planes of a w x h frame */
int mj423_idct_blocks(mj423_ctx *ctx, size_t n, const int16_t *DCAC, const int16_t *quant,
                      uint8_t *blocks);
int mj423_ycbcr_to_rgb_444(mj423_ctx *ctx, uint32_t w_size, uint32_t h_size, const uint8_t *Y,
                           const uint8_t *Cb, const uint8_t *Cr, rgb_pixel_t *rgb);

/* ----------------------------------------------------------- 2. frame call */
/* The per-frame body of mj/decoder/mjpeg423_decoder.c:109-124 (after the three
 * lossless_decode calls): dequant + IDCT of every Y/Cb/Cr block + CSC of every
 * pixel, fused on the GPU.  Host buffers, synchronous.  Yq/Cbq/Crq are
 * block-raster planes sized by mj423_geometry(); out is width*height pixels. */
int decode_frame(mj423_ctx *ctx, const int16_t *Yq, const int16_t *Cbq, const int16_t *Crq,
                 rgb_pixel_t *out, uint32_t w, uint32_t h, int chroma);
int mj423_decode_frame_ex(mj423_ctx *ctx, const int16_t *Yq, const int16_t *Cbq, const int16_t *Crq,
                          rgb_pixel_t *out, uint32_t w, uint32_t h, int chroma, int input_form);
/* n frames, coefficients [frame][Y | Cb | Cr] (geometry.coef_per_frame each),
 * output [frame][h][w]; one upload, one launch, one download. */
int decode_frames(mj423_ctx *ctx, uint32_t n, const int16_t *coef, rgb_pixel_t *out, uint32_t w,
                  uint32_t h, int chroma, int input_form);

/* ------------------------------ 3. reference accelerator API (async, per process) */
/* c0/idct_ycbcr_to_rgb_accel.h:13-22, same names and spelling.  The process-wide
 * accelerator decodes one frame per ycbcr_to_rgb_accel_get_results(): the three
 * idct_accel_calculate_buffer_* calls stage DEQUANTIZED dct_block_t planes (the
 * reference's input contract, c0/playback.c:71-75,102), get_results launches the
 * fused kernel once all three planes and the output request are present, and
 * copies the BGRA frame back.  Frame geometry defaults to the reference's
 * 640x480 4:4:4 (c0/common/config.h:23-24,56-62); see mj423_accel_configure.
 * init returns 1 on success, 0 on failure, like the reference (accel.c:63-83). */
int init_idct_ycbcr_to_rgb_accel(void);
void idct_accel_calculate_buffer_y(void *inputBuffer, uint32_t sizeOfInputBuffer);
void idct_accel_calculate_buffer_cb(void *inputBuffer, uint32_t sizeOfInputBuffer);
void idct_accel_calculate_buffer_cr(void *inputBuffer, uint32_t sizeOfInputBuffer);
void ycbcr_to_rgb_accel_get_results(void *outputBuffer, uint32_t sizeOfOutputBuffer);
/* Declared by the reference (accel.h:19-20) but never defined there: the CSC
 * stage alone over already-IDCT'd 4:4:4 blocks (hCb_size x wCb_size blocks,
 * frame width w_size).  Note the reference's argument order Y, Cr, Cb. */
void ycbcr_to_rgb_accel_calculate_buffer(color_block_t *yBlock, color_block_t *crBlock,
                                         color_block_t *cbBlock, rgb_pixel_t *outputBuffer,
                                         int hCb_size, int wCb_size, int w_size);
/* Block until the BGRA frame has landed in outputBuffer (accel.c:108-114). */
void wait_for_ycbcr_to_rgb_finsh(void);
/* Block until the Y input has been consumed, so the caller may refill it (accel.c:116-122). */
void wait_for_idct_y_finsh(void);
/* Extension: geometry of the accelerator's frames (default 640, 480, 444). */
int mj423_accel_configure(uint32_t w, uint32_t h, int chroma);
/* Extension: release the accelerator's device resources. */
void mj423_accel_shutdown(void);
/* Extension: the reference's accelerator calls return void, so a failed submission (call
 * before a successful init, NULL buffer, an input larger than its plane -- rejected, never
 * truncated --, or a failed HIP copy/launch/event) drops the frame it belonged to and is
 * recorded here: returns the first MJ423_E* code since the last call (MJ423_OK if none),
 * sets mj423_last_error() to its message, and clears it (read-and-clear, like a CSR error
 * bit).  wait_for_*_finsh() also repeat a pending error into mj423_last_error(). */
int mj423_accel_status(void);

/* ------------------------------------------------ 4. device-resident batches */
/* Decode nframes frames that are already in device memory.  Plane bases are
 * device pointers to frame 0; plane_frame_stride is the int16 distance between
 * frames (same for all three planes); out_frame_stride / out_pitch are in pixels.
 * Asynchronous on the context's stream. */
typedef struct {
    const int16_t *y, *cb, *cr;
    uint64_t plane_frame_stride;
    rgb_pixel_t *out;
    uint64_t out_frame_stride;
    uint32_t out_pitch;
    uint32_t nframes;
    uint32_t width, height;
    int32_t chroma;
    int32_t input_form;
} mj423_frames_desc_t;
int mj423_decode_frames_device(mj423_ctx *ctx, const mj423_frames_desc_t *desc);

/* Stream decode with on-GPU P-frame accumulation.
 * frame_types (host array, nframes): 0 = I-frame, planes hold absolute quantized
 * coefficients; 1 = P-frame, planes hold that frame's DELTAS (what lossless_decode
 * adds at mj/decoder/lossless_decode.c:90-92,121-122, before dequantization).  The
 * kernel keeps each tile's accumulated coefficients on chip across the frames of a
 * GOP, so a P-frame costs the same HBM bytes as an I-frame.  state_in (device,
 * geometry.coef_per_frame int16 laid out [Y | Cb | Cr]) holds the absolute
 * coefficients before frame 0 and is required iff frame 0 is a P-frame; state_out
 * (optional, same layout) receives them after the last frame, for the next batch;
 * it may be state_in itself or overlap it anyhow (an overlapping state_in is read from a copy
 * unless the launch is one GOP segment with state_out == state_in exactly).
 * input_form must be MJ423_INPUT_QUANTIZED.  Asynchronous on the context's stream. */
int mj423_decode_stream_device(mj423_ctx *ctx, const mj423_frames_desc_t *desc, const uint8_t *frame_types,
                               const int16_t *state_in, int16_t *state_out);

/* Synthetic quantized-coefficient stream written on the device:
 * frames [frame0, frame0+nframes) of a seeded counter-based generator, laid out
 * [frame][Y | Cb | Cr] with geometry.coef_per_frame int16 per frame.  Uses the
 * context's quant tables for the DC range and the |Q*q| <= 1023 AC clip. */
int mj423_synth_frames_device(mj423_ctx *ctx, int16_t *coef, uint32_t w, uint32_t h, int chroma,
                              uint32_t nframes, uint64_t frame0, uint64_t seed);

/* ------------------------------------------ 5. multi-GPU (one process, N devices) */
/* The reference splits a frame's work across two Nios II cores that hand buffers over a
 * mailbox (c0/playback.c:80-134, core1/software/main.c:227-335).  Here frames are
 * independent given absolute coefficients, so a group of N devices splits a
 * job into contiguous frame ranges (mj423_frame_range) with no data-path exchange; the one
 * collective is an RCCL broadcast (ncclBroadcast over xGMI, ncclUint8) of the 256-byte
 * {Yquant, Cquant} (mj/common/tables.c:13-32) from rank 0.  A group owns one context (own
 * stream) per device and one RCCL communicator per device from ncclCommInitAll.  RCCL is
 * loaded on first use (librccl.so.1).  Calls on one group are not thread-safe.
 *
 * flags: MJ423_MULTI_NO_COMM builds the group without RCCL -- devices may then repeat
 * (e.g. {0, 0, 0} on a one-GPU box to exercise the sharding) and the broadcast becomes
 * host copies.  A rehearsal aid; mj423_multi_comm_ranks() then returns 0. */
#define MJ423_MULTI_NO_COMM 1
typedef struct mj423_multi mj423_multi;
/* devices == NULL: devices 0..ndev-1; ndev <= 0: every visible device. */
int mj423_multi_create(mj423_multi **m, int ndev, const int *devices, int flags);
void mj423_multi_destroy(mj423_multi *m);
int mj423_multi_size(const mj423_multi *m);          /* ranks (= devices) in the group */
mj423_ctx *mj423_multi_ctx(mj423_multi *m, int rank); /* the rank's context (owned by the group) */
/* Ranks RCCL reports for rank 0's communicator (ncclCommCount); 0 without RCCL. */
int mj423_multi_comm_ranks(const mj423_multi *m);
/* Rank 0 takes these tables (NULL: the reference's), then ncclBroadcast hands the 256 B to
 * every rank and each rank's context adopts what it received. */
int mj423_multi_set_quant(mj423_multi *m, const int16_t yquant[64], const int16_t cquant[64]);
/* Contiguous [first, first+count) of `total` frames for `rank` of `world`; sizes differ by
 * <= 1 and earlier ranks take the extra frames.  Pure host arithmetic. */
int mj423_frame_range(uint32_t rank, uint32_t world, uint64_t total, uint64_t *first, uint64_t *count);
/* Host buffers, like decode_frames(): n frames [frame][Y | Cb | Cr] -> out [frame][h][w],
 * split by mj423_frame_range over the ranks, every device uploading, decoding and
 * downloading its range concurrently.  Synchronous. */
int mj423_multi_decode_frames(mj423_multi *m, uint64_t n, const int16_t *coef, rgb_pixel_t *out, uint32_t w,
                              uint32_t h, int chroma, int input_form);
/* Device-resident: descs[r] (device pointers on rank r's device) is decoded by rank r; all
 * ranks launch, asynchronously on their own streams.  A desc with nframes == 0 is skipped. */
int mj423_multi_decode_frames_device(mj423_multi *m, const mj423_frames_desc_t *descs);
/* Rank r writes frames [frame0[r], frame0[r]+nframes[r]) of the seeded synthetic stream
 * (mj423_synth_frames_device) at coef[r] on its device.  Asynchronous. */
int mj423_multi_synth_frames_device(mj423_multi *m, int16_t *const *coef, const uint64_t *frame0,
                                    const uint32_t *nframes, uint32_t w, uint32_t h, int chroma, uint64_t seed);
int mj423_multi_synchronize(mj423_multi *m);
/* Timed run of `steps` device-resident decodes of descs on every rank, start-aligned: every
 * device is drained, then each records a start event, enqueues the steps and an end event.
 * per_rank_ms[r] (may be NULL, size = ranks) = rank r's event time for all steps; *max_ms =
 * the largest of them; *wall_ms (may be NULL) = host time from before the first start event
 * to the moment every device has finished. */
int mj423_multi_time_decode(mj423_multi *m, const mj423_frames_desc_t *descs, uint32_t steps, double *max_ms,
                            double *per_rank_ms, double *wall_ms);

#ifdef __cplusplus
}
#endif
#endif /* MJ423GPU_H */
