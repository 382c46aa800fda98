// mj423_entropy.h -- parameter block of the many-lanes-per-stream GPU entropy front end
// (mj423_entropy.hip), shared with its host driver (mj423_gpu_frontend.cpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mj423_check.hpp"
#include "mj423_kernels.h"

namespace mj423 {

// Subsequence length: one lane decodes the symbols that start in each kSubBytes bytes of
// a stream (~40 symbols), after finding its true start by self-synchronisation.
#ifndef MJ423_ENTPAR_SUB_BYTES
#define MJ423_ENTPAR_SUB_BYTES 64
#endif
constexpr uint32_t kSubBytes = MJ423_ENTPAR_SUB_BYTES;
constexpr uint32_t kSubBits = 8 * kSubBytes;

// The fused .mpg decode (mj423_fused.hip) works on tiles of kFuseTw MCUs = kFuseTw consecutive
// blocks of every plane (4:4:4); the index pass records where each tile's blocks start.
constexpr uint32_t kFuseTw = 64;

struct EntParParams {
    const uint8_t* bytes;      // the frames' bytes in HBM, readable 64 B past bytes_len
    uint64_t bytes_len;
    const EntropyTask* tasks;  // one (frame, plane) bitstream per task
    uint32_t ntasks;
    const uint32_t* sub0;      // ntasks + 1: first subsequence of each task (prefix of ceil(nbytes / kSubBytes), >= 1 each)
    uint32_t g0, nsub;         // this launch's subsequences: [g0, nsub) = [sub0[0], sub0[ntasks])
    uint32_t nblk;             // blocks per plane
    uint64_t* start;           // per subsequence: the state its lane decoded from
    uint64_t* exit_;           // per subsequence: the state after its last symbol
    uint32_t* nb;              // per subsequence: DC symbols (blocks started); after the scan: blocks before it
    uint32_t* dcs;             // per subsequence: sum of DC differences; after the scan: DC before it (mod 2^16)
    uint32_t* flags;           // per sync iteration: 1 if any lane changed (+ the index pass's overflow word)
    uint32_t* zrun;            // per subsequence: first lane of its run of all-zero lanes, ~0 if not all-zero
    uint32_t* zlast;           // at a run's first lane: the run's last lane
    uint32_t* lane_task;       // per subsequence: its task (entpar_map_kernel)
    uint32_t* qbits;           // work lists of the synchronisation iterations >= 2: two lane bitmaps of
    uint32_t qwords;           // qwords words each (every lane of the call), zeroed beforehand
    uint32_t* tchg;            // per task: 1 + the last sync iteration in which one of its lanes changed
    uint32_t* wcnt;            // per task: [16] its lanes' walks in each list iteration (zeroed by the init kernel)
    uint32_t unsettled;        // = the iteration count: emit skips tasks with tchg == unsettled (the fallback decodes them)
    // multi-class resolution of the streams still changing in the last iteration (entmc_*; null: off).
    // Per lane of the launch (index g - g0):
    uint32_t* mc_list;         // the lanes of those streams, compacted (mc_count entries)
    uint32_t* mc_count;        // one word, zeroed beforehand
    uint64_t* mc_x;            // [16] the distinct exit states of the lane's seed walks (unused: ~0)
    uint64_t* mc_map;          // nibble i: the class (mc_x index) of the lane's exit when it starts at its
                               //  predecessor's class i (15: not among them)
    uint32_t* mc_rec;          // [16] per predecessor class: blocks started | DC sum << 16
    uint64_t* mc_st;           // [16] the classes kernel's distinct phase-1 states (~0: none) ...
    uint32_t* mc_sfx;          // [16] ... their exit's class | blocks << 4 | DC sum << 16 from there
    uint32_t* mc_ck;           // the phase-1 checkpoint (bits into the lane) those states sit at
    int16_t* out;              // [frame][Y | Cb | Cr] dense planes, zero-filled beforehand
    uint64_t coef_pf;          // int16 per frame
    uint32_t* status;          // per task: 0 ok, 1 the blocks needed bits past the stream's end, 2 not finished
    uint32_t lds_window;       // walks read a per-lane window staged in LDS (mj423_entropy.hip kWin)
    // index pass (fused path, instead of emit's dense planes), per (frame, plane) of the launch:
    uint32_t* bpos;            // [frame][plane][nblk + 1] each block's first bit in its plane's bitstream,
                               //  then the end of the plane's last block
    uint2* tiles;              // [frame][plane][tiles_pp] {bit position of the tile's first block,
                               //  DC before it (I-frames; 0 for P)} for tiles of kFuseTw blocks
    uint32_t tiles_pp;         // ceil(nblk / kFuseTw)
    BufLimits lim;             // what each pointer may index (bounds-check builds, mj423_check.hpp)
};

// The fused .mpg decode (mj423_fused.hip): one workgroup per (tile of kFuseTw MCUs, GOP segment)
// walks the segment's frames; per frame every block of the tile is entropy-decoded by its own
// lane (from `tiles` and `bpos`), accumulated (P) in LDS, then dequantized, transformed and
// converted like decode_gop_kernel<444>.
struct FusedParams {
    DecodeParams d;            // output, geometry (4:4:4, tw = kFuseTw), qt_dev, ftype, seg_start, nseg,
                               // state / state_out (+ st_cb_off, st_cr_off; natural order); coef unused
    const uint8_t* bytes;      // the frames' bytes in HBM, readable 64 B past bytes_len
    uint64_t bytes_len;
    const EntropyTask* tasks;  // per (frame, plane) of the launch, 3 * frame + plane
    const uint32_t* bpos;      // the index pass's outputs for the launch's frames (EntParParams)
    const uint2* tiles;
    uint32_t nblk, tiles_pp;
    uint32_t state_quantized;  // d.state holds quantized coefficients (the host's seek seed), else dequantized
                               // (a previous launch's state_out: the kernel keeps its state dequantized)
    BufLimits lim;             // what each pointer may index (bounds-check builds, mj423_check.hpp)
};

}  // namespace mj423

extern "C" {
// The fused decode of d.nseg GOP segments x d.tiles_per_frame tiles.
hipError_t mj423_launch_mpg_fused(const mj423::FusedParams* p, hipStream_t stream);
// init + zero-run scan + max_iters synchronisation iterations (flags[0 .. max_iters) zeroed beforehand)
hipError_t mj423_launch_entpar(const mj423::EntParParams* p, uint32_t max_iters, hipStream_t stream);
// scan + emit (streams with tchg == unsettled are skipped: still changing after the last iteration)
hipError_t mj423_launch_entpar_finish(const mj423::EntParParams* p, hipStream_t stream);
// scan + index pass (bpos / tiles instead of dense planes), then the serial index walk of the streams
// still changing after the last iteration.
hipError_t mj423_launch_entpar_index(const mj423::EntParParams* p, hipStream_t stream);
}
