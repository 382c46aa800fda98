/*
 * mj423io.h -- host side of the MPEG423 decoder around the GPU hot path
 * (SURVEY.md §8(f) rows 1, 2 and 4): the entropy front end, the .mpg container,
 * the BMP sink and the whole-file decoder.  Exported by libmj423gpu.so next to
 * the C ABI of mj423gpu.h.  Reference paths are relative to
 * core0/software/common/libs/mjpeg423/ ("mj/").
 *
 * The entropy front end is bit-serial and stays on host cores, exactly where the
 * reference runs it (north_star: the GPU path "drops in behind the existing
 * bitstream front end"); it is not a fallback for the GPU path, which has none.
 */
#ifndef MJ423IO_H
#define MJ423IO_H

#include <stddef.h>
#include <stdint.h>

#include "mj423gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* ------------------------------------------------------ 1. entropy front end */
/* void lossless_decode(int num_blocks, void* bitstream, dct_block_t* DCACq,
 *                      dct_block_t quant, bool P)
 * -- mj/decoder/mjpeg423_decoder.h:17, defined mj/decoder/lossless_decode.c:60.
 * Same semantics: DC/AC VLI decode with EOB/ZRL, zig-zag scatter, dequantization;
 * I-frames (P == 0) clear the planes and prefix-sum DC, P-frames accumulate into
 * DCACq.  Like the reference it is unbounded (reads as far as the stream says).
 * (The reference's `bool` is `typedef int bool`, mj/common/mjpeg423_types.h:16-19.) */
void lossless_decode(int num_blocks, void *bitstream, dct_block_t *DCACq, dct_block_t quant, int P);

/* Quantized-domain form of the same walk: writes ABSOLUTE quantized
 * coefficients (DC prefix-summed, P deltas accumulated mod 2^16, no multiply) for
 * decode_frame().  Bounded by nbytes: returns the bytes consumed, or (size_t)-1 if
 * the stream ran past nbytes (missing bits read as zero). */
size_t mj423_lossless_decode_q(int num_blocks, const void *bitstream, size_t nbytes, int16_t *q_abs, int P);

/* ------------------------------------------------------- 2. .mpg container */
/* File layout (writer mj/encoder/mjpeg423_encoder.c:82-88,188-225; reader
 * mj/decoder/mjpeg423_decoder.c:33-38,78-107):
 *   u32 num_frames, width, height, num_iframes, payload_size
 *   per frame: u32 frame_size, frame_type (0 = I, 1 = P), Ysize, Cbsize, then the
 *              Y | Cb | Cr bitstreams, padded to 4 bytes (frame_size includes the 16 B)
 *   trailer:   num_iframes x {u32 frame_index, u32 frame_position}, then 512 B pad */
typedef struct {
    uint32_t num_frames, width, height, num_iframes, payload_size;
} mj423_mpg_header_t;

typedef struct {
    uint32_t index;
    uint32_t frame_type;           /* 0 = I, 1 = P */
    uint32_t frame_size;           /* bytes incl. the 16-byte frame header and padding */
    uint64_t position;             /* file offset of the frame header */
    const uint8_t *y, *cb, *cr;    /* bitstreams inside the mapped file */
    uint32_t y_size, cb_size, cr_size; /* cr_size includes the 4-byte alignment pad */
} mj423_mpg_frame_t;

typedef struct mj423_mpg mj423_mpg;

int mj423_mpg_open(const char *path, mj423_mpg **out);
int mj423_mpg_open_memory(const void *data, size_t nbytes, mj423_mpg **out); /* copies the bytes */
void mj423_mpg_close(mj423_mpg *m);
int mj423_mpg_header(const mj423_mpg *m, mj423_mpg_header_t *h);
/* Frame size: any width/height in [1, 2^20].  Like the reference, only the w/8 x h/8 whole
 * 8x8 blocks are coded (mj/encoder/mjpeg423_encoder.c:21-24) and decoded
 * (mj/decoder/mjpeg423_decoder.c:45-48,120-124): the planes are those of
 * mj423_geometry(w & ~7, h & ~7, 444), returned here (zero blocks and coef_per_frame 0 when w
 * or h is below 8).  Decoded frames are still w x h: the coded region holds the decode, and
 * the right (w & 7) columns and bottom (h & 7) rows -- which the reference leaves as
 * uninitialised memory in the BMPs it writes (mjpeg423_decoder.c:55,132) -- are set to zero
 * (BGRA 0,0,0,0) by every decode entry below. */
int mj423_mpg_geometry(const mj423_mpg *m, mj423_geometry_t *g);
int mj423_mpg_frame(const mj423_mpg *m, uint32_t index, mj423_mpg_frame_t *f);
/* I-frame trailer (mj/common/mjpeg423_types.h:22-25): up to max entries; returns the count. */
int mj423_mpg_trailer(const mj423_mpg *m, uint32_t *frame_index, uint32_t *frame_position, uint32_t max);
/* The I-frame at or before `index` (GOP start), from the frame types. */
int mj423_mpg_gop_start(const mj423_mpg *m, uint32_t index, uint32_t *gop_start);

/* Entropy-decode frames [first, first+count) into absolute quantized planes laid out
 * [frame][Y | Cb | Cr] (mj423_mpg_geometry().coef_per_frame int16 each), ready
 * for decode_frames()/mj423_decode_frames_device().  P-frame state is rebuilt from
 * the GOP's I-frame when `first` is a P-frame.  Planes and GOPs are decoded on up
 * to `nthreads` host threads (<= 0: the CPUs the process may run on -- affinity mask, capped
 * by a cgroup v2 cpu.max quota; the same default everywhere `nthreads` appears). */
int mj423_mpg_entropy_decode(const mj423_mpg *m, uint32_t first, uint32_t count, int16_t *coef, int nthreads);

/* Same frames in the form mj423_decode_stream_device() takes: I-frames as absolute
 * quantized coefficients, P-frames as their own deltas (no accumulation on the host,
 * every frame independent, so all (frame, plane) pairs decode in parallel).
 * frame_types[i] receives 0 (I) or 1 (P). */
int mj423_mpg_entropy_decode_deltas(const mj423_mpg *m, uint32_t first, uint32_t count, int16_t *coef,
                                    uint8_t *frame_types, int nthreads);

/* Front end + GPU: frames [first, first+count) to BGRA (out: count * w * h pixels).
 * Host threads emit per-frame deltas; the GPU accumulates P-frames on chip
 * (mj423_decode_stream_device). */
int mj423_decode_mpg(mj423_ctx *ctx, const mj423_mpg *m, uint32_t first, uint32_t count, rgb_pixel_t *out,
                     int nthreads);

/* Streaming form of mj423_decode_mpg for whole files (the reference's frame loop,
 * mj/decoder/mjpeg423_decoder.c:88-141, as a pipeline): chunks of `chunk_frames`
 * frames (0: 48 = two GOPs at the reference's maximum I-interval, or ceil(count / 6) when
 * that is smaller so a short call allocates no more than it fills, capped so a chunk's
 * device buffers stay near 1 GiB and a quarter of the device memory free at creation; the
 * footprint is 3 slots x (chunk coefficients + pixels + transfer buffer) on the device plus
 * 3 x (pixels + transfer buffer) pinned on the host; the transfer buffers hold what the
 * call's bitstreams can expand to, at most the dense planes) flow through
 * entropy decode on `nthreads` host threads -> H2D -> stream-decode kernel -> D2H ->
 * `sink`, all stages overlapped (3-slot ring of pinned host and device buffers,
 * separate copy streams).  P-frame state crosses chunk boundaries on the GPU.  `sink`
 * runs on a library thread, once per frame in frame order; the pixels are valid only
 * during the call; a non-zero return stops the pipeline.  `stats` may be NULL. */
typedef int (*mj423_frame_sink_fn)(void *user, uint32_t frame_index, const rgb_pixel_t *bgra, uint32_t w, uint32_t h);
typedef struct {
    uint64_t frames, chunks;
    double wall_s;           /* whole call */
    double frontend_busy_s;  /* time the front-end stage spent decoding (its threads in parallel) */
    double sink_busy_s;      /* time spent inside `sink` */
    double gpu_span_ms;      /* first kernel start -> last kernel end, on the GPU clock */
} mj423_pipeline_stats_t;
int mj423_decode_mpg_pipelined(mj423_ctx *ctx, const mj423_mpg *m, uint32_t first, uint32_t count,
                               uint32_t chunk_frames, int nthreads, mj423_frame_sink_fn sink, void *user,
                               mj423_pipeline_stats_t *stats);
/* The same as a reusable object: buffers (pinned host ring, device ring, state), copy
 * streams and the front-end thread pool are set up once for w x h streams and kept
 * across decode calls (a player decoding many files or seeking repeatedly).  The transfer
 * buffers start at an eighth of the dense planes and grow, once, when a chunk's bitstreams
 * could expand to more.  One decode call at a time per pipeline; the context must outlive it. */
typedef struct mj423_pipeline mj423_pipeline;
int mj423_pipeline_create(mj423_pipeline **p, mj423_ctx *ctx, uint32_t w, uint32_t h, uint32_t chunk_frames,
                          int nthreads);
int mj423_pipeline_decode(mj423_pipeline *p, const mj423_mpg *m, uint32_t first, uint32_t count,
                          mj423_frame_sink_fn sink, void *user, mj423_pipeline_stats_t *stats);
void mj423_pipeline_destroy(mj423_pipeline *p);
/* Decode to device memory (no D2H): `sink` is called once per chunk, in order, with the
 * chunk's BGRA frames in HBM (frame i of the chunk at bgra + i * frame_stride pixels) and
 * the HIP stream (hipStream_t) the decode was enqueued on.  The frames are complete in
 * stream order: the sink enqueues its consumers on that stream (or waits on it) and
 * returns; the buffers are reused only after work it enqueued there.  A non-zero return
 * stops the pipeline. */
typedef int (*mj423_device_sink_fn)(void *user, uint32_t first_frame, uint32_t count, const rgb_pixel_t *bgra,
                                    size_t frame_stride, void *stream);
int mj423_pipeline_decode_device(mj423_pipeline *p, const mj423_mpg *m, uint32_t first, uint32_t count,
                                 mj423_device_sink_fn sink, void *user, mj423_pipeline_stats_t *stats);

/* Whole-GPU decode of frames [first, first+count) into device memory: the frames'
 * bytes are uploaded once, every (frame, plane) bitstream is entropy-decoded on its own
 * GPU lane (P-frames as deltas, so all frames' streams are independent), then
 * mj423_decode_stream_device accumulates + decodes them; frame i lands at
 * d_out + i * out_frame_stride pixels.  window_frames bounds the dense coefficient
 * staging in HBM (0: half the free HBM, at most 64 GiB, at least 4 GiB worth); state
 * crosses windows on the GPU.  Synchronizes the
 * context's stream before returning (the per-stream status check); a bitstream that
 * ends early is reported like mj423_mpg_entropy_decode does. */
int mj423_mpg_decode_gpu(mj423_ctx *ctx, const mj423_mpg *m, uint32_t first, uint32_t count, rgb_pixel_t *d_out,
                         uint64_t out_frame_stride, uint32_t window_frames);

/* Multi-GPU form (group from mj423gpu.h section 5): frames [first, first+count) are cut at
 * I-frames into one balanced range per rank (mj423_mpg_gop_ranges: a range that starts at an
 * I-frame needs no earlier frame, mj/decoder/lossless_decode.c:77-78), and every rank runs
 * mj423_mpg_decode_gpu on its own device concurrently; rank r's frames land at d_out[r] +
 * i * out_frame_stride (device pointers on rank r's device; stride 0 = w*h).  range_first / range_count
 * (may be NULL; one entry per rank) receive the ranges.  Synchronous. */
int mj423_mpg_gop_ranges(const mj423_mpg *m, uint32_t first, uint32_t count, uint32_t world, uint32_t *range_first,
                         uint32_t *range_count);
int mj423_multi_decode_mpg_gpu(mj423_multi *g, const mj423_mpg *m, uint32_t first, uint32_t count,
                               rgb_pixel_t *const *d_out, uint64_t out_frame_stride, uint32_t *range_first,
                               uint32_t *range_count);

/* ---------------------------------------------------------- 4. BMP sink */
/* 32-bpp bottom-up BMP, byte-identical to the reference's encode_bmp -> bmp_save
 * (mj/libbmp/encode_bmp.c:7-24, mj/libbmp/bmpfile.c:628-700). */
int mj423_write_bmp(const char *filename, const rgb_pixel_t *rgb, uint32_t w_size, uint32_t h_size);
/* The reference's own symbol (declared at mj/decoder/mjpeg423_decoder.c:16). */
void encode_bmp(rgb_pixel_t *rgbblock, uint32_t w_size, uint32_t h_size, const char *filename);

/* ------------------------------------------------------ whole-file decoder */
/* void mjpeg423_decode(const char* filename_in, const char* filenamebase_out)
 * -- mj/decoder/mjpeg423_decoder.h:14, mj/decoder/mjpeg423_decoder.c:20-149:
 * every frame of the .mpg to <base with the last 8 chars replaced by NNNN.bmp>,
 * e.g. "out0000.bmp" -> out0000.bmp, out0001.bmp, ...  Runs
 * the pipeline on the process-default context, sized to the file, with a BMP-writing sink:
 * entropy decode on host threads, dequant + IDCT + CSC on the GPU, BMPs byte-identical to
 * the reference's written by up to 8 threads (one file per frame, in no particular order)
 * while later chunks decode.  Errors are reported through mj423_last_error() (the
 * reference prints and exit(-1)s instead). */
void mjpeg423_decode(const char *filename_in, const char *filenamebase_out);
/* Same, returning a status code. */
int mj423_decode_file(const char *filename_in, const char *filenamebase_out);

#ifdef __cplusplus
}
#endif
#endif /* MJ423IO_H */
