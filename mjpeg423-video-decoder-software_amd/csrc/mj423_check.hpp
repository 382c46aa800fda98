// mj423_check.hpp -- bounds checks for the whole-file decoder's kernels (mj423_entropy.hip,
// mj423_fused.hip, mj423_margin.hip), compiled in only with -DMJ423_BOUNDS_CHECK (the diagnostic build
// tools/build_variant.sh bounds '-DMJ423_BOUNDS_CHECK'; the product build has none).  Every global
// index a kernel derives from a table is checked against the elements the launcher says the
// allocation holds from that pointer; a failing check prints the access and traps, so the kernel that
// makes it and the buffer it misses are named instead of surfacing later as an illegal address.
#pragma once
#include <stdint.h>

#ifdef MJ423_BOUNDS_CHECK
#include <stdio.h>
#define MJ423_BOUND(i, n, what)                                                                                    \
    do {                                                                                                           \
        const unsigned long long i_ = (unsigned long long)(i), n_ = (unsigned long long)(n);                       \
        if (!(i_ < n_)) {                                                                                          \
            printf("mj423 bound: %s: index %llu, limit %llu (workgroup %u,%u thread %u, %s:%d)\n", what, i_, n_,   \
                   blockIdx.x, blockIdx.y, threadIdx.x, __FILE__, __LINE__);                                       \
            __builtin_trap();                                                                                      \
        }                                                                                                          \
    } while (0)
#else
#define MJ423_BOUND(i, n, what) ((void)0)
#endif

namespace mj423 {
// Elements each pointer of a launch may index (from the pointer as passed, not from the allocation's
// start): the launchers fill it from the allocations' capacities in every build; only bounds-check
// builds read it.
struct BufLimits {
    uint64_t bytes_dw;   // dwords of the uploaded bytes (bytes_len + 64 B)
    uint64_t tasks;      // EntropyTask entries
    uint64_t sub0;       // uint32 entries
    uint64_t lanes;      // start / exit_ / nb / dcs / zrun / zlast / lane_task entries (absolute lane index)
    uint64_t qbits;      // uint32 words, both bitmaps
    uint64_t flags;      // uint32 words
    uint64_t tchg;       // uint32 entries
    uint64_t status;     // uint32 entries
    uint64_t bpos;       // uint32 entries
    uint64_t tiles;      // uint2 entries
    uint64_t ftype;      // bytes
    uint64_t seg_start;  // uint32 entries
    uint64_t state;      // int16 elements (state and state_out)
    uint64_t out;        // pixels
    uint64_t mc;         // lanes of the multi-class arrays (mc_list / mc_map entries; mc_x / mc_rec: 16 each)
};
}  // namespace mj423
