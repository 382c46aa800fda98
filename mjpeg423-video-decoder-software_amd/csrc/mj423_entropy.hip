// mj423_entropy.hip -- GPU entropy front end, many lanes per bitstream.
//
// The walk of lossless_decode.c:82-134 is bit-serial, and the format has no restart
// points, so entropy_kernel (mj423_kernels.hip) gives each (frame, plane) stream one wave
// and a launch lasts as long as its longest stream (~17 ms for a 1080p I-frame plane).
// Here every stream is cut into subsequences of kSubBytes bytes, one lane each, and the
// lanes find their true starting points by self-synchronisation (the idea of
// Weissenberger & Schmidt's parallel Huffman decoding, applied to this format's fixed
// 4-bit fields):
//
//   state   = (bit position, next symbol DC or AC, zig-zag index) at a symbol boundary;
//   sync    : lane k decodes from its start state until the first symbol boundary at or
//             past the end of subsequence k and publishes that exit state; lane k+1 takes
//             it as its start.  Lanes start from a guess, so early exits are wrong, but a
//             parse from a wrong position falls onto the true symbol boundaries within a
//             few symbols and onto the true state at the next block end; each iteration
//             re-decodes only the lanes whose start changed.  When an iteration changes
//             nothing, every lane starts where its predecessor's (exact, by induction from
//             lane 0) parse ends: the partition of the true parse is exact.
//   zeros   : a run of zero bits (DC size 0 + EOB, 12 bits a block: flat I-frame regions,
//             static P-frame regions) is periodic, and a parse that enters it out of phase
//             never falls into phase there -- plain iteration would need one round per
//             subsequence of the run.  A lane whose bits (plus the longest symbol past its
//             end) are all zero is an all-zero lane; the parse crosses it with DC symbols at
//             d0 + 12j and EOBs at d0 + 12j + 4, so its exit follows in closed form from the
//             state at which the parse entered the run (the exit of the lane before the
//             run's first lane): the whole run settles in the iteration after that lane.
//   scan    : per stream, exclusive prefix sums over its lanes of (blocks started, DC
//             differences mod 2^16) -> each lane's first block index and running DC.
//   emit    : every lane decodes its range once more, assembles each block whose DC
//             symbol starts there in LDS and stores it whole (128 B, zeros included, so no
//             plane clearing): the same output as entropy_kernel (I-frames absolute, DC
//             prefix-summed; P-frames their deltas), with the same per-stream status.
//
// Symbol rules (lossless_decode.c:86-129, HUFF_EXTEND :204): DC = SIZE(4) + VLI;
// AC = RUN(4) SIZE(4) + VLI; SIZE 0: RUN 15 = ZRL (index += 16), else EOB; a coefficient
// at index + RUN is written when <= 63 and ends the block when >= 63.  Indices past 63
// behave alike (no write, the next coefficient or EOB ends the block), so the state
// saturates the index at 64.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <stdlib.h>

#include <algorithm>

#include "mj423_bits.hpp"
#include "mj423_entropy.h"

namespace mj423 {

namespace {

struct Lane {
    uint32_t task, k, nsub;  // stream, subsequence within it, subsequences of the stream
    EntropyTask t;
};

// The stream (task) of subsequence g: lane_task (entpar_map_kernel) -- one load, where a binary
// search over the tasks was a chain of ~10 dependent loads at the head of every lane's work.
__device__ __forceinline__ bool lane_of(const EntParParams& p, uint32_t g, Lane& l) {
    if (g < p.g0 || g >= p.nsub) return false;  // (a work-list bitmap word may hold another window's lanes)
    MJ423_BOUND(g, p.lim.lanes, "lane_task");
    l.task = p.lane_task[g];
    if (l.task >= p.ntasks) return false;  // (never, with consistent tables: no access outside them)
    MJ423_BOUND(l.task + 1, p.lim.sub0, "sub0");
    MJ423_BOUND(l.task, p.lim.tasks, "tasks");
    const uint32_t s0 = p.sub0[l.task];
    l.k = g - s0;
    l.nsub = p.sub0[l.task + 1] - s0;
    l.t = p.tasks[l.task];
    return true;
}

struct Walk {
    Reader r;
    uint64_t base;  // absolute bit of the stream's first bit
    uint32_t guard;
    // Without a slot: the reader loads from global memory.
    __device__ __forceinline__ Walk(const EntParParams& p, const Lane& l, uint32_t pos) { setup(p, l, pos); }
    // lw: this lane's LDS slot (kWin dwords), staged with the window starting one dword before `pos`,
    // each dword masked at the stream's end and byte-swapped here (Reader::fixed), once, instead of
    // at every refill of every parse
    __device__ __forceinline__ Walk(const EntParParams& p, const Lane& l, uint32_t pos, lds_u32* lw) {
        r.dw = reinterpret_cast<const uint32_t*>(p.bytes);
        r.dw_max = (p.bytes_len + 60) / 4;  // the dword holding byte bytes_len + 63 at most
        MJ423_BOUND(r.dw_max, p.lim.bytes_dw, "bytes (walk window)");
        r.end = l.t.byte_off + l.t.nbytes;
        const uint64_t b = l.t.byte_off * 8 + pos;
        const uint64_t w0 = (b >> 5) - ((b >> 5) ? 1 : 0);
        uint32_t v[kWin];
#pragma unroll
        for (uint32_t j = 0; j < kWin; j++) v[j] = r.dw[w0 + j < r.dw_max ? w0 + j : r.dw_max];  // independent loads
        // bytes of the window before the stream's end (Reader::fix in 32 bits: the window is 4 * kWin bytes)
        const uint32_t e = 4 * w0 >= r.end ? 0u : (uint32_t)min<uint64_t>(r.end - 4 * w0, 4 * kWin);
#pragma unroll
        for (uint32_t j = 0; j < kWin; j++) {
            const uint32_t k = e > 4 * j ? min(e - 4 * j, 4u) : 0u;  // bytes of dword j to keep
            const uint32_t m = k >= 4 ? 0xffffffffu : (1u << (8 * k)) - 1u;
            lw[j] = __builtin_bswap32(v[j] & m);
        }
        r.lw = lw;
        r.w0 = w0;
        r.lds = true;
        setup(p, l, pos);
    }
    __device__ __forceinline__ void setup(const EntParParams& p, const Lane& l, uint32_t pos) {
        r.dw = reinterpret_cast<const uint32_t*>(p.bytes);
        r.end = l.t.byte_off + l.t.nbytes;
        r.dw_max = (p.bytes_len + 60) / 4;  // the dword holding byte bytes_len + 63 at most
        MJ423_BOUND(r.dw_max, p.lim.bytes_dw, "bytes (walk)");
        base = l.t.byte_off * 8;
        r.init(base + pos);
        // Symbols: every one takes >= 4 bits, and past the stream's end (zeros) a block is
        // DC size 0 + EOB, so 2 * nbytes + 2 * nblk bounds any walk.
        guard = 2 * l.t.nbytes + 2 * p.nblk + 64;
    }
    __device__ __forceinline__ uint32_t at() const { return (uint32_t)(r.abspos() - base); }
    __device__ __forceinline__ int32_t dc() {  // DC: SIZE(4) + VLI
        const uint32_t size = r.take(4);
        return huff_extend(r.take(size), size);
    }
    // AC: RUN(4) SIZE(4) + VLI.  Returns true when the block ends; `e` != 0 is a coefficient
    // at zig-zag index `idx` (before the post-increment) when idx <= 63.
    __device__ __forceinline__ bool ac(uint32_t& idx, int32_t& e, uint32_t& at_idx) {
        const uint32_t run = r.take(4), size = r.take(4);
        e = 0;
        if (size == 0) {
            if (run != 15) return true;  // EOB
            idx = min(idx + 16, 64u);   // ZRL: 16 zeros
            return false;
        }
        idx = min(idx + run, 64u);
        e = huff_extend(r.take(size), size);
        at_idx = idx;
        const bool end = idx >= 63;
        idx++;
        return end;
    }
};

// Sync walk: symbols from state (pos, ac, idx) while the next one starts before `stop`
// (bits); counts DC symbols (nb) and sums their differences (dcs, mod 2^16).
// The same walk with one branch-free symbol step: the DC and AC interpretations of the next 8 bits
// are selected, not branched on, so lanes of a wave in different modes do not serialise.
__device__ __forceinline__ void walk_sync_bf(const EntParParams& p, const Lane& l, uint32_t& pos, uint32_t& ac,
                                             uint32_t& idx, uint32_t stop, uint32_t& nb, uint32_t& dcs, lds_u32* lw) {
    Walk w(p, l, pos, lw);
    Reader& r = w.r;
#ifdef MJ423_DEBUG_WINDOW
    if (pos + 600 < stop) printf("walk_sync_bf: start %u far before stop %u (k=%u)\n", pos, stop, l.k);
#endif
    // `at` runs alongside the reader (32-bit, one add per symbol) instead of being recomputed
    // from its 64-bit state; the symbol comes from the window's top 32 bits
    // (no symbol guard: every symbol takes >= 4 bits, so the walk reaches `stop`)
    uint32_t at = w.at();
    // one state word: idx = 0 at a DC symbol, else the AC position (ac is idx != 0; a start in
    // DC mode may carry idx 1 -- the zero runs' closed form -- so it is cleared here)
    idx = ac ? idx : 0u;
    for (;;) {
        if (at >= stop) {
            pos = at;
            ac = idx != 0 ? 1u : 0u;
            return;
        }
        r.refill_lds();  // >= 33 bits in the window; a symbol takes <= 8 + 15
        const bool A = idx != 0;
        const uint32_t hi = (uint32_t)(r.win >> 32), hi4 = hi >> 28, lo4 = (hi >> 24) & 15u;
        const uint32_t hdr = A ? 8u : 4u, size = A ? lo4 : hi4;
        const uint32_t v = __builtin_amdgcn_ubfe(hi, 32u - hdr - size, size);  // VLI (0 when size is 0)
        const uint32_t tot = hdr + size;
        r.win <<= tot;
        r.n -= tot;
        at += tot;
        // DC: SIZE + VLI (lossless_decode.c:86-96)
        const int32_t e = huff_extend(v, size);
        dcs += A ? 0u : (uint32_t)e;
        nb += A ? 0u : 1u;
        // AC: RUN + SIZE + VLI; size 0: RUN 15 = ZRL, else EOB; a coefficient at min(idx + run, 64)
        // ends the block at index >= 63 (lossless_decode.c:100-129)
        const uint32_t t = min(idx + hi4, 64u);
        const bool zrl = size == 0 && hi4 == 15, eob = size == 0 && hi4 != 15;
        const bool end = eob || (size != 0 && t >= 63);
        const uint32_t nidx = zrl ? min(idx + 16, 64u) : t + 1;
        idx = A ? (end ? 0u : nidx) : 1u;
    }
}

__device__ __forceinline__ void walk_sync(const EntParParams& p, const Lane& l, uint32_t& pos, uint32_t& ac, uint32_t& idx,
                                          uint32_t stop, uint32_t& nb, uint32_t& dcs) {
    Walk w(p, l, pos);
    for (;;) {
        const uint32_t at = w.at();
        if (at >= stop || w.guard-- == 0) {
            pos = at;
            return;
        }
        w.r.refill();
        if (!ac) {
            dcs += (uint32_t)w.dc();
            nb++;
            ac = 1;
            idx = 1;
            continue;
        }
        int32_t e;
        uint32_t ai;
        if (w.ac(idx, e, ai)) {
            ac = 0;
            idx = 0;
        }
    }
}

// Through an all-zero run entered at state (q, ac): DC symbols at d0 + 12j, EOBs at
// d0 + 12j + 4 (j >= 0), plus the EOB at q when entered in AC mode (d0 = q + 8).  The
// first symbol boundary at or past `at` and the DC symbols in [from, it).
__device__ __forceinline__ uint32_t zero_next(uint32_t d0, uint32_t at, uint32_t& ac) {
    if (at <= d0) {
        ac = 0;
        return d0;
    }
    const uint32_t jd = (at - d0 + 11) / 12, xd = d0 + 12 * jd;  // next DC
    const uint32_t je = (at - d0 - 4 + 11 + 12) / 12 - 1;        // next EOB (at > d0 so at - d0 - 4 >= -3)
    const uint32_t xe = d0 + 4 + 12 * je;
    if (xe < xd && xe >= at) {
        ac = 1;
        return xe;
    }
    ac = 0;
    return xd;
}
__device__ __forceinline__ uint32_t zero_dcs_between(uint32_t d0, uint32_t from, uint32_t to) {  // DC positions in [from, to)
    auto upto = [&](uint32_t x) -> uint32_t { return x <= d0 ? 0u : (x - d0 + 11) / 12; };  // positions < x
    return upto(to) - upto(from);
}

}  // namespace

// Is every bit of subsequence k's bytes [b0, b0 + kSubBytes + 3) zero (bytes past the stream's end
// counting as zero)?  Whole dwords covering them, masked at both ends and at the stream end.
__device__ __forceinline__ bool lane_all_zero(const EntParParams& p, const EntropyTask& t, uint32_t k) {
    const uint32_t* dw = reinterpret_cast<const uint32_t*>(p.bytes);
    const uint64_t dw_max = (p.bytes_len + 60) / 4, end = t.byte_off + t.nbytes;
    MJ423_BOUND(dw_max, p.lim.bytes_dw, "bytes (zero test)");
    const uint64_t b0 = t.byte_off + (uint64_t)k * kSubBytes, b1 = b0 + kSubBytes + 3;
    const uint64_t hi = min(b1, end);  // bytes [b0, hi) count
    constexpr uint32_t kDw = (kSubBytes + 3 + 3) / 4 + 1;  // dwords that can hold them, whatever b0's alignment
    uint32_t v[kDw];
#pragma unroll
    for (uint32_t j = 0; j < kDw; j++) {  // independent loads: one latency, not kDw
        const uint64_t i = (b0 >> 2) + j;
        v[j] = dw[i < dw_max ? i : dw_max];
    }
    uint32_t any = 0;
#pragma unroll
    for (uint32_t j = 0; j < kDw; j++) {
        const uint64_t a = ((b0 >> 2) + j) * 4;  // bytes [a, a + 4) of the dword; keep those in [b0, hi)
        const uint32_t lo_cut = a < b0 ? (uint32_t)min<uint64_t>(b0 - a, 4) : 0u;
        const uint32_t hi_keep = hi <= a ? 0u : (uint32_t)min<uint64_t>(hi - a, 4);
        const uint32_t keep = hi_keep > lo_cut ? (((hi_keep == 4 ? 0xffffffffu : (1u << (8 * hi_keep)) - 1u)) &
                                                  ~((1u << (8 * lo_cut)) - 1u))
                                               : 0u;
        any |= v[j] & keep;
    }
    return any == 0;
}

constexpr uint32_t kScanThreads = 1024;  // per-stream scans: a 1080p plane's ~1 700 lanes in two steps, not seven

// Per stream: the first lane of each run of all-zero lanes.  entpar_init_kernel left
// zrun[g] = 1 for an all-zero lane, 0 otherwise; this turns it into the run's first lane (an
// all-zero lane) or ~0 (not all-zero) with a max-scan of "1 + last non-zero lane" per stream, and
// records each run's last lane at its first: zlast[first] = last.
__global__ void __launch_bounds__(kScanThreads) entpar_zrun_kernel(const EntParParams p) {
    constexpr uint32_t W = kScanThreads / 64;
    const uint32_t task = blockIdx.x;
    MJ423_BOUND(task + 1, p.lim.sub0, "sub0 (zero runs)");
    const uint32_t s0 = p.sub0[task], s1 = p.sub0[task + 1];
    if (s1 > s0) MJ423_BOUND(s1 - 1, p.lim.lanes, "zrun (zero runs)");
    __shared__ uint32_t wmax[W];
    uint32_t carry = 0;  // 1 + the last lane (relative) that is not all-zero, 0 if none yet
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t c = s0; c < s1; c += kScanThreads) {
        const uint32_t g = c + threadIdx.x;
        const bool zero = g < s1 && p.zrun[g] != 0u;
        const bool next_zero = g + 1 < s1 && p.zrun[g + 1] != 0u;  // (not rewritten yet: this chunk's after the barrier)
        uint32_t m = (g < s1 && !zero) ? g - s0 + 1 : 0u;  // inclusive max-scan of "1 + non-zero lane"
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t tm = __shfl_up(m, o);
            if (lane >= (uint32_t)o) m = max(m, tm);
        }
        if (lane == 63) wmax[wave] = m;
        __syncthreads();
        uint32_t pm = carry, all = carry;
#pragma unroll
        for (uint32_t w = 0; w < W; w++) {
            if (w < wave) pm = max(pm, wmax[w]);
            all = max(all, wmax[w]);
        }
        m = max(m, pm);
        if (g < s1) p.zrun[g] = zero ? s0 + m : ~0u;  // run start: the lane after the last non-zero one
        if (zero && !next_zero) p.zlast[s0 + m] = g;    // the run's last lane
        carry = all;
        __syncthreads();
    }
}

// lane_task[g] = the stream of every subsequence g of the launch; one workgroup per stream.
__global__ void __launch_bounds__(256) entpar_map_kernel(const EntParParams p) {
    const uint32_t task = blockIdx.x;
    MJ423_BOUND(task + 1, p.lim.sub0, "sub0 (map)");
    const uint32_t s0 = p.sub0[task], s1 = p.sub0[task + 1];
    if (s1 > s0) MJ423_BOUND(s1 - 1, p.lim.lanes, "lane_task (map)");
    for (uint32_t g = s0 + threadIdx.x; g < s1; g += 256) p.lane_task[g] = task;
}

// (MJ423_INIT_IN_IT0=0 builds only: iteration 0 does this itself, sync_lane0.)
// Initial guesses: every lane's "exit" = a guessed start for its successor (AC, index 1,
// at the successor's first bit); starts invalid; status = runaway until a lane finishes.
// Also the all-zero test (every bit of [start, end + 24) zero, bytes past the stream's end
// counting as zero) of each lane, zrun[g] = 1 / 0, for entpar_zrun_kernel.
__global__ void __launch_bounds__(256) entpar_init_kernel(const EntParParams p) {
    Lane l;
    if (!lane_of(p, p.g0 + blockIdx.x * 256 + threadIdx.x, l)) return;
    const uint32_t g = p.sub0[l.task] + l.k;
    p.start[g] = ~0ull;
    p.exit_[g] = pack((l.k + 1) * kSubBits, 1, 1);
    if (l.k == 0) {
        MJ423_BOUND(l.task, p.lim.status, "status (init)");
        MJ423_BOUND(l.task, p.lim.tchg, "tchg (init)");
        p.status[l.task] = 2u;
        p.tchg[l.task] = 0u;
        MJ423_BOUND((uint64_t)l.task * 16 + 15, p.lim.tchg * 16, "wcnt (init)");
        for (uint32_t j = 0; j < 16; j++) p.wcnt[l.task * 16 + j] = 0u;
    }
    p.zrun[g] = lane_all_zero(p, l.t, l.k) ? 1u : 0u;
}

// All-zero lane g of the run starting at lane zr: its start state, exit (pos, ac) and DC symbols,
// in closed form from the exit of the lane before the run (the stream's first bit if none).
__device__ __forceinline__ uint64_t zero_lane(const EntParParams& p, uint32_t g, const Lane& l, uint32_t zr, uint32_t& pos,
                                              uint32_t& ac, uint32_t& nb) {
    const uint32_t first = p.sub0[l.task];
    MJ423_BOUND(zr - first, g - first + 1, "zero-run start outside [stream start, lane]");
    const uint64_t en = zr == first ? pack(0, 0, 0) : __hip_atomic_load(p.exit_ + zr - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t q = (uint32_t)en, d0 = q + (((uint32_t)(en >> 32) & 1u) ? 8u : 0u);
    uint32_t a_in = (uint32_t)(en >> 32) & 1u, from = q;
    if (g != zr) from = zero_next(d0, l.k * kSubBits, a_in);
    pos = zero_next(d0, (l.k + 1) * kSubBits, ac);
    if (from >= (l.k + 1) * kSubBits) {  // entered past its own end: nothing inside
        pos = from;
        ac = a_in;
    }
    nb = zero_dcs_between(d0, from, pos);
    return g == zr ? en : pack(from, a_in, 1);
}

// One synchronisation iteration of lane g: decode from its predecessor's current exit (or, for an
// all-zero lane, the closed form from the state its run was entered with) unless that is the
// start it already decoded from.  Returns true when the lane's exit changed (its successors'
// inputs did).  Iteration `it` sets flags[it] = 1 when any lane changed.
__device__ __forceinline__ bool sync_lane(const EntParParams& p, uint32_t g, const Lane& l, uint32_t it, lds_u32* wins) {
    // the predecessor's exit (64-bit: read whole; it may be rewritten during this launch --
    // a fresher value only speeds convergence, and the final iteration changes nothing)
    const uint32_t zr = p.zrun[g];
    uint64_t st;
    uint32_t pos, ac, idx, nb = 0, dcs = 0;
    if (zr != ~0u) {  // all-zero lane: closed form from the state the parse entered its run with
        st = zero_lane(p, g, l, zr, pos, ac, nb);
        if (st == p.start[g]) return false;
        idx = 1;
    } else {
        st = l.k == 0 ? pack(0, 0, 0) : __hip_atomic_load(p.exit_ + g - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (st == p.start[g]) return false;
        pos = (uint32_t)st;
        ac = (uint32_t)(st >> 32) & 1u;
        idx = (uint32_t)(st >> 33) & 127u;
        if (p.lds_window)
            walk_sync_bf(p, l, pos, ac, idx, (l.k + 1) * kSubBits, nb, dcs, wins);
        else
            walk_sync(p, l, pos, ac, idx, (l.k + 1) * kSubBits, nb, dcs);
    }
    if (it >= 2) atomicAdd(p.wcnt + l.task * 16 + it, 1u);  // walks of the stream in this list iteration
    const uint64_t ex = pack(pos, ac, idx);
    const bool moved = ex != __hip_atomic_load(p.exit_ + g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    p.start[g] = st;
    p.nb[g] = nb;
    p.dcs[g] = dcs;
    __hip_atomic_store(p.exit_ + g, ex, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    MJ423_BOUND(it, p.lim.flags, "flags");
    MJ423_BOUND(l.task, p.lim.tchg, "tchg");
#ifdef MJ423_SYNC_COUNT
    atomicAdd(p.flags + it, 1u);  // diagnostic build: walks per iteration (still nonzero iff any ran)
#else
    p.flags[it] = 1u;
#endif
    p.tchg[l.task] = it + 1;
    return moved;
}

// Work lists.  Once every lane has decoded from its predecessor's first exit (iterations 0 and 1,
// full grids), only the lanes whose predecessor's exit then moved have anything left to do -- a
// few per cent.  From iteration 1 on, a lane whose exit moved queues its successors for the next
// iteration as bits of a lane bitmap (qbits, two of them in turn): the next lane, or, when a run
// of all-zero lanes follows, the run's last lane (its closed form reads the exit before the run
// directly; the lanes inside the run are brought up to date once, by entpar_scan_kernel).  A bit
// set twice is one entry, so no lane runs twice in an iteration (two threads on one lane would mix
// their outputs), and the only atomics are bit sets.
__device__ __forceinline__ void queue_lane(const EntParParams& p, uint32_t m, uint32_t next) {
    MJ423_BOUND((uint64_t)(next & 1u) * p.qwords + (m >> 5), p.lim.qbits, "qbits (queue)");
    atomicOr(p.qbits + (size_t)(next & 1u) * p.qwords + (m >> 5), 1u << (m & 31u));
}

__device__ __forceinline__ void queue_successors(const EntParParams& p, uint32_t g, const Lane& l, uint32_t it) {
    const uint32_t next = it + 1, s1 = p.sub0[l.task + 1];
    if (g + 1 >= s1) return;  // the stream's last lane
    MJ423_BOUND(s1 - 1, p.lim.lanes, "zrun (successors)");
    const uint32_t n = g + 1, zn = p.zrun[n];
    if (zn == ~0u) {
        queue_lane(p, n, next);
    } else if (p.zrun[g] != zn) {  // g is the lane before a zero run: its last lane
        MJ423_BOUND(zn, p.lim.lanes, "zlast (successors)");
        const uint32_t last = p.zlast[zn];
        MJ423_BOUND(last - zn, s1 - zn, "zero-run end outside [run start, stream end)");
        queue_lane(p, last, next);
    }
    // (g inside a run, n too: n's closed form does not read g's exit -- nothing to queue)
}

#ifndef MJ423_INIT_IN_IT0
#define MJ423_INIT_IN_IT0 1
#endif
// Iteration 0 of lane g, with the window's set-up folded in (no separate guesses kernel: the chain of
// synchronisation launches is what the next fused kernel waits for): every lane walks from its guessed
// start -- the stream's first bit, or AC index 1 at the lane's first bit -- all-zero lanes included
// (their closed form needs the zero runs, found after this iteration), and records the all-zero test
// of its bytes (read by the walk just before: cached) for entpar_zrun_kernel; the stream's first lane
// resets its status and walk counts.
__device__ __forceinline__ void sync_lane0(const EntParParams& p, uint32_t g, const Lane& l, lds_u32* wins) {
    const uint64_t st = l.k == 0 ? pack(0, 0, 0) : pack(l.k * kSubBits, 1, 1);
    uint32_t pos = (uint32_t)st, ac = l.k == 0 ? 0u : 1u, idx = ac, nb = 0, dcs = 0;
    if (p.lds_window)
        walk_sync_bf(p, l, pos, ac, idx, (l.k + 1) * kSubBits, nb, dcs, wins);
    else
        walk_sync(p, l, pos, ac, idx, (l.k + 1) * kSubBits, nb, dcs);
    p.start[g] = st;
    p.nb[g] = nb;
    p.dcs[g] = dcs;
    __hip_atomic_store(p.exit_ + g, pack(pos, ac, idx), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    p.zrun[g] = lane_all_zero(p, l.t, l.k) ? 1u : 0u;
    MJ423_BOUND(l.task, p.lim.status, "status (iteration 0)");
    MJ423_BOUND(l.task, p.lim.tchg, "tchg (iteration 0)");
    if (l.k == 0) {
        p.status[l.task] = 2u;
        MJ423_BOUND((uint64_t)l.task * 16 + 15, p.lim.tchg * 16, "wcnt (iteration 0)");
        for (uint32_t j = 0; j < 16; j++) p.wcnt[l.task * 16 + j] = 0u;
    }
    p.tchg[l.task] = 1u;
#ifdef MJ423_SYNC_COUNT
    atomicAdd(p.flags, 1u);
#else
    p.flags[0] = 1u;
#endif
}

// Iterations 0 and 1 (full grid); from iteration 1 on the lanes whose exit moved queue their
// successors.  Once an iteration changed nothing, later ones return at once.
// (MJ423_SYNC_THREADS per workgroup, A/B: 128 or 64 threads' LDS windows would fit beside the fused
// kernel's four workgroups on a CU -- measured no faster, profiles/r06/synth_ab/sync_threads.log)
#ifndef MJ423_SYNC_THREADS
#define MJ423_SYNC_THREADS 256
#endif
constexpr uint32_t kSyncThreads = MJ423_SYNC_THREADS;
__global__ void __launch_bounds__(kSyncThreads) entpar_sync_kernel(const EntParParams p, uint32_t it) {
    __shared__ uint32_t wins[kSyncThreads * kWin];  // each lane's staged window (lane-private: no barrier)
    if (it > 0 && __builtin_nontemporal_load(p.flags + it - 1) == 0) return;
    Lane l;
    const uint32_t g = p.g0 + blockIdx.x * kSyncThreads + threadIdx.x;
    if (!lane_of(p, g, l)) return;
#if MJ423_INIT_IN_IT0
    if (it == 0) {
        sync_lane0(p, g, l, (lds_u32*)(wins + kWin * threadIdx.x));
        return;
    }
#endif
    if (sync_lane(p, g, l, it, (lds_u32*)(wins + kWin * threadIdx.x)) && it >= 1) queue_successors(p, g, l, it);
}

// A stream whose walks per iteration hardly fall off is a periodic one the iteration will not settle
// (a static scene's DC-only or empty P-blocks; its walks fall ~10 % per iteration where a converging
// stream's fall ~60 %): from iteration kPeriodicFrom on, one that walked >= kPeriodicMin lanes in the
// previous iteration and > 0.7 of the iteration before's is not iterated further but marked
// unsettled, for the multi-class resolution (mc_list != null) -- which resolves the whole stream
// anyway, so each iteration spent on it was wasted.  No launch added: the counts are atomic adds of
// the list iterations' walks (a few per cent of the lanes), the test two loads per listed lane.
// (Iteration 3, with one count, uses the share of the stream's lanes that walked in iteration 2.)
#ifndef MJ423_PERIODIC_FROM
#define MJ423_PERIODIC_FROM 4
#endif
#ifndef MJ423_PERIODIC_MIN
#define MJ423_PERIODIC_MIN 16
#endif
constexpr uint32_t kPeriodicFrom = MJ423_PERIODIC_FROM, kPeriodicMin = MJ423_PERIODIC_MIN;
// Iteration 3 has one count only (iteration 1 is not counted: every lane walks in it): there a stream
// is cut when more than kPeriodicShare % of its lanes walked in iteration 2 (the synthetic streams
// ~2 %, the noisy static scene ~5 %, a clean static scene's P-planes ~30 %).
#ifndef MJ423_PERIODIC_SHARE
#define MJ423_PERIODIC_SHARE 15
#endif
__device__ __forceinline__ bool periodic(const EntParParams& p, uint32_t task, uint32_t nsub, uint32_t it) {
    if (!p.mc_list || it < kPeriodicFrom - 1) return false;
    MJ423_BOUND((uint64_t)task * 16 + it, p.lim.tchg * 16, "wcnt (periodic)");
    const uint32_t c1 = p.wcnt[task * 16 + it - 1];
    if (it == kPeriodicFrom - 1) return kPeriodicFrom == 4 && c1 >= kPeriodicMin && 100 * c1 > MJ423_PERIODIC_SHARE * nsub;
    const uint32_t c2 = p.wcnt[task * 16 + it - 2];
    return c1 >= kPeriodicMin && 10 * c1 > 7 * c2;
}

// Iterations 2 ...: the lanes queued for this iteration.  Each workgroup takes chunks of kListWords
// bitmap words (32 lanes each), clears them, gathers the set bits into an LDS list and runs those
// lanes, one per thread.  64 words (2048 lanes) and 512 threads: on the synthetic streams a chunk
// holds ~75 queued lanes (smaller chunks only add workgroups to every launch, the empty ones
// included: 8 words +2.5 % per pass), while a stream whose lanes keep changing -- a static scene's
// periodic planes -- fills a chunk, and 512 threads take it in four rounds of walks instead of
// eight (latency-bound walks: more waves per CU hide each other's waits).  1024 threads: two
// rounds, but 106 KB of LDS per workgroup, which no CU running a fused-kernel workgroup can hold
// beside it: the synthetic pass +1 % (profiles/r06/synth_ab/list_threads.log).
#ifndef MJ423_LIST_WORDS
#define MJ423_LIST_WORDS 64
#endif
#ifndef MJ423_LIST_THREADS
#define MJ423_LIST_THREADS 512
#endif
constexpr uint32_t kListWords = MJ423_LIST_WORDS, kListThreads = MJ423_LIST_THREADS;
static_assert(kListWords >= 1 && kListWords <= 64, "list chunk: one wave reads and scans its words");
static_assert(kListThreads % 64 == 0 && kListThreads <= 1024, "list workgroup: whole waves");
__global__ void __launch_bounds__(kListThreads) entpar_sync_list_kernel(const EntParParams p, uint32_t it) {
    __shared__ uint32_t wins[kListThreads * kWin];
    __shared__ uint32_t list[kListWords * 32];
    __shared__ uint32_t ltot;
    if (__builtin_nontemporal_load(p.flags + it - 1) == 0) return;
    uint32_t* bits = p.qbits + (size_t)(it & 1u) * p.qwords;
    const uint32_t w0 = p.g0 >> 5, w1 = (p.nsub + 31) >> 5;
    const uint32_t tid = threadIdx.x;
    for (uint32_t c = w0 + blockIdx.x * kListWords; c < w1; c += gridDim.x * kListWords) {  // (uniform per workgroup)
        if (tid < 64) {  // wave 0: read and clear the chunk's words, exclusive prefix of their set-bit counts
            uint32_t word = 0;
            if (tid < kListWords && c + tid < w1) {
                MJ423_BOUND((uint64_t)(it & 1u) * p.qwords + c + tid, p.lim.qbits, "qbits (list)");
                word = bits[c + tid];
                if (word) bits[c + tid] = 0u;  // (each word has one reader: this iteration's)
            }
            const uint32_t cnt = __builtin_popcount(word);
            uint32_t incl = cnt;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t t = __shfl_up(incl, o);
                if (tid >= (uint32_t)o) incl += t;
            }
            uint32_t k = incl - cnt;
            for (uint32_t b = word; b; b &= b - 1) {
                MJ423_BOUND(k, kListWords * 32, "list (LDS)");
                list[k++] = ((c + tid) << 5) + (uint32_t)__builtin_ctz(b);
            }
            if (tid == 63) ltot = incl;
        }
        __syncthreads();
        const uint32_t total = ltot;
        for (uint32_t e = tid; e < total; e += kListThreads) {
            const uint32_t g = list[e];
            Lane l;
            if (!lane_of(p, g, l)) continue;
            if (periodic(p, l.task, l.nsub, it)) {  // left to the multi-class resolution
                p.tchg[l.task] = p.unsettled;
                continue;
            }
            if (sync_lane(p, g, l, it, (lds_u32*)(wins + kWin * tid))) queue_successors(p, g, l, it);
        }
        __syncthreads();  // list and ltot are rewritten by the next chunk
    }
}


// Per stream: exclusive prefix sums of (nb, dcs) over its lanes, in place
// (nb -> blocks started before the lane, dcs -> DC running value before it).
__global__ void __launch_bounds__(kScanThreads) entpar_scan_kernel(const EntParParams p) {
    constexpr uint32_t W = kScanThreads / 64;
    const uint32_t task = blockIdx.x;
    MJ423_BOUND(task + 1, p.lim.sub0, "sub0 (scan)");
    const uint32_t s0 = p.sub0[task], s1 = p.sub0[task + 1];
    if (s1 > s0) MJ423_BOUND(s1 - 1, p.lim.lanes, "nb/dcs (scan)");
    __shared__ uint32_t wsum[2][W];
    uint32_t carry_nb = 0, carry_dc = 0;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (uint32_t c = s0; c < s1; c += kScanThreads) {
        const uint32_t g = c + threadIdx.x;
        uint32_t own_a = 0, own_d = 0;
        if (g < s1) {
            const uint32_t zr = p.zrun[g];
            if (zr != ~0u) {  // all-zero lane: its state from the final exit before its run (the iterations
                              // only kept the run's last lane current)
                Lane l;
                l.task = task;
                l.k = g - s0;
                uint32_t pos, ac;
                p.start[g] = zero_lane(p, g, l, zr, pos, ac, own_a);
            } else {
                own_a = p.nb[g];
                own_d = p.dcs[g];
            }
        }
        uint32_t a = own_a, d = own_d;
        // inclusive wave scan
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t ta = __shfl_up(a, o), td = __shfl_up(d, o);
            if (lane >= (uint32_t)o) {
                a += ta;
                d += td;
            }
        }
        if (lane == 63) {
            wsum[0][wave] = a;
            wsum[1][wave] = d;
        }
        __syncthreads();
        uint32_t pa = carry_nb, pd = carry_dc, ta = 0, td = 0;
#pragma unroll
        for (uint32_t w = 0; w < W; w++) {
            if (w < wave) {
                pa += wsum[0][w];
                pd += wsum[1][w];
            }
            ta += wsum[0][w];
            td += wsum[1][w];
        }
        if (g < s1) {
            p.nb[g] = pa + a - own_a;
            p.dcs[g] = pd + d - own_d;
        }
        carry_nb += ta;
        carry_dc += td;
        __syncthreads();
    }
}

// Final pass.  A lane owns the blocks whose DC symbol starts in its range and decodes each
// to its end (past its range's end if need be); a block in progress at its start belongs to
// its predecessor and is skipped.  Blocks are assembled in a 128-B LDS slot per lane and
// stored whole -- zeros included, so the planes need no clearing -- in wave-wide rounds:
// every lane decodes its next block, then the wave stores eight whole blocks per store
// instruction (lanes 8j..8j+7 write the eight 16-B pieces of one block), so each
// instruction writes 8 full 128-B lines instead of 64 partial ones.  The lane that
// finishes block nblk - 1 records the stream's status.
__global__ void __launch_bounds__(256) entpar_emit_kernel(const EntParParams p) {
    __shared__ uint8_t zz[64];
    __shared__ uint4 slots[256 * 8];  // one 128-B block per lane
    if (threadIdx.x < 64) zz[threadIdx.x] = kZz[threadIdx.x];
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    uint4* slot = slots + 8 * threadIdx.x;
    int16_t* s16 = reinterpret_cast<int16_t*>(slot);
    // Every lane stays to the end: the stores are cooperative.
    Lane l = {};
    const uint32_t g = p.g0 + blockIdx.x * 256 + threadIdx.x;
    bool done = !lane_of(p, g, l);
    if (!done && p.unsettled && p.tchg[l.task] == p.unsettled) done = true;  // left to the one-wave fallback
    uint64_t st = 0;
    uint32_t blk0 = 0, dc = 0;
    if (!done) {
        st = p.start[g];
        blk0 = p.nb[g];
        dc = p.dcs[g];
        done = blk0 > p.nblk;  // wholly past the plane's last block
    }
    int16_t* plane = nullptr;
    uint32_t stop = 0, ac = 0, idx = 0;
    bool P = false;
    Walk w(p, l, done ? 0u : (uint32_t)st);  // (a valid in-bounds reader even for idle lanes)
    if (!done && (uint64_t)l.t.frame * 3 + l.t.plane >= p.ntasks) done = true;  // (never, with a consistent task table)
    if (!done) {
        plane = p.out + (uint64_t)l.t.frame * p.coef_pf + (uint64_t)l.t.plane * p.nblk * 64;
        stop = l.k + 1 == l.nsub ? 0xffffffffu : (l.k + 1) * kSubBits;  // the last lane runs to the plane's end
        ac = (uint32_t)(st >> 32) & 1u;
        idx = (uint32_t)(st >> 33) & 127u;
        P = l.t.ptype != 0;
        while (ac) {  // the predecessor's block in progress: skip to its end
            if (w.guard-- == 0) {
                done = true;
                break;
            }
            w.r.refill();
            int32_t e;
            uint32_t ai;
            if (w.ac(idx, e, ai)) ac = 0;
        }
    }
    int64_t blk = (int64_t)blk0 - 1;
    for (;;) {
        // this lane's next block into its slot
        uint64_t dst = 0;  // byte address of the block just completed, 0 if none
        if (!done) {
            w.r.refill();
            if (w.at() >= stop || ++blk >= (int64_t)p.nblk) {
                done = true;
            } else {
                const int32_t e = w.dc();
                dc += (uint32_t)e;
#pragma unroll
                for (int i = 0; i < 8; i++) slot[i] = make_uint4(0, 0, 0, 0);
                s16[0] = (int16_t)(P ? (uint32_t)e : dc);
                idx = 1;
                for (;;) {
                    if (w.guard-- == 0) {  // status stays "not finished"
                        done = true;
                        break;
                    }
                    w.r.refill();
                    int32_t v;
                    uint32_t ai = 64;
                    const bool end = w.ac(idx, v, ai);
                    if (v != 0 && ai <= 63) s16[zz[ai]] = (int16_t)v;
                    if (end) {
                        dst = reinterpret_cast<uint64_t>(plane + (uint64_t)blk * 64);
                        if (blk == (int64_t)p.nblk - 1) {  // the plane's last block just ended
                            p.status[l.task] = w.at() > 8u * l.t.nbytes ? 1u : 0u;
                            done = true;
                        }
                        break;
                    }
                }
            }
        }
        if (__ballot(dst != 0) == 0) {  // no lane completed a block this round
            if (__ballot(!done) == 0) break;
            continue;
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        // lanes 8j + (lane >> 3)'s blocks: this lane stores piece lane & 7 of each
        const uint4* wslots = slots + 8 * (threadIdx.x & ~63u);
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint32_t src = 8 * j + (lane >> 3);
            const uint64_t d = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(dst >> 32), (int)src) << 32) |
                               (uint32_t)__shfl((int)(uint32_t)dst, (int)src);
            if (d)  // streaming stores: the planes are read back only by the stream kernel, after this launch
                __builtin_nontemporal_store(reinterpret_cast<const v4u32*>(wslots)[8 * src + (lane & 7)],
                                            reinterpret_cast<v4u32*>(d) + (lane & 7));
        }
        __builtin_amdgcn_wave_barrier();  // slots are rewritten next round only after every lane read them
    }
}

// Index pass of the fused path.  The same lanes, starts and prefix sums as the emit pass, but a
// lane records only where its blocks are: each block's first bit (bpos; bpos[nblk] = the end of
// the plane's last block, so a block's coded length is the difference of neighbours) and, for a
// block that starts a tile of kFuseTw blocks, the DC before it (tiles).  The fused kernel decodes
// every block of a tile in parallel from those (mj423_fused.hip), so no dense plane is written
// or read.
// index_plane: one lane over a whole plane (entidx_serial_kernel).
__device__ __forceinline__ void index_plane(const EntParParams& p, const EntropyTask& t, uint32_t task, Walk& w,
                                            uint32_t blk0, uint32_t dc, uint32_t stop) {
    if ((uint64_t)t.frame * 3 + t.plane >= p.ntasks) return;  // (never, with a consistent task table; status stays set)
    MJ423_BOUND(((uint64_t)t.frame * 3 + t.plane) * (p.nblk + 1) + p.nblk, p.lim.bpos, "bpos (serial index)");
    MJ423_BOUND(((uint64_t)t.frame * 3 + t.plane + 1) * p.tiles_pp - 1, p.lim.tiles, "tiles (serial index)");
    MJ423_BOUND(task, p.lim.status, "status (serial index)");
    uint32_t* bpos = p.bpos + ((uint64_t)t.frame * 3 + t.plane) * (p.nblk + 1);
    uint2* tiles = p.tiles + ((uint64_t)t.frame * 3 + t.plane) * p.tiles_pp;
    const bool P = t.ptype != 0;
    for (uint32_t blk = blk0; blk < p.nblk; blk++) {
        w.r.refill();
        const uint32_t at = w.at();
        if (at >= stop) return;
        const int32_t e = w.dc();
        bpos[blk] = at;
        if (blk % kFuseTw == 0) tiles[blk / kFuseTw] = make_uint2(at, P ? 0u : (dc & 0xffffu));
        dc += (uint32_t)e;
        uint32_t idx = 1;
        for (;;) {
            if (w.guard-- == 0) return;  // status stays "not finished"
            w.r.refill();
            int32_t v;
            uint32_t ai;
            if (w.ac(idx, v, ai)) break;
        }
        if (blk + 1 == p.nblk) {  // the plane's last block just ended
            bpos[p.nblk] = w.at();
            p.status[task] = w.at() > 8u * t.nbytes ? 1u : 0u;
            return;
        }
    }
}

// The lanes' index walk: walk_sync_bf's branch-free symbol step over the symbols that start in
// the lane (the synchronisation's final parse of it, from the same start), recording each DC
// symbol's position; a block in progress at the lane's start is its predecessor's, and the one in
// progress at its end its successor's to finish, except that the plane's last block is ended by
// whichever lane reaches its last symbol.  The plane's last lane goes on past its own bits (zeros)
// until that block has ended, so a stream too short for its blocks is reported as the stream
// kernels report it (status 1).
struct IdxStep {
    uint32_t blk, dc, at, idx;  // idx: 0 at a DC symbol, else the AC position (walk_sync_bf's state)
    bool done = false;
    // one symbol; LDS: the window-only refill
    template <bool LDS>
    __device__ __forceinline__ void step(const EntParParams& p, const Lane& l, Reader& r, uint32_t* bpos, uint2* tiles,
                                         bool P) {
        if (LDS)
            r.refill_lds();
        else
            r.refill();
        const bool ac = idx != 0;
        const uint32_t hi = (uint32_t)(r.win >> 32), hi4 = hi >> 28, lo4 = (hi >> 24) & 15u;
        const uint32_t hdr = ac ? 8u : 4u, size = ac ? lo4 : hi4;
        const uint32_t v = __builtin_amdgcn_ubfe(hi, 32u - hdr - size, size);
        const uint32_t tot = hdr + size;
        r.win <<= tot;
        r.n -= tot;
        const uint32_t sym = at;  // this symbol's first bit
        at += tot;
        const int32_t e = huff_extend(v, size);
        const uint32_t tt = min(idx + hi4, 64u);
        const bool zrl = size == 0 && hi4 == 15, eob = size == 0 && hi4 != 15;
        const bool end = eob || (size != 0 && tt >= 63);
        // straight-line: the stores are predicated, the state updated by selects (the branchy form's
        // early returns put both paths and their exec bookkeeping on every symbol of the wave)
        const bool rec = !ac && blk < p.nblk;             // a DC symbol at `sym`: block `blk` starts
        const bool last = ac && end && blk == p.nblk;     // the plane's last block ends here
        if (rec) {
            bpos[blk] = sym;
            if (blk % kFuseTw == 0) tiles[blk / kFuseTw] = make_uint2(sym, P ? 0u : (dc & 0xffffu));
        }
        if (last) {
            bpos[p.nblk] = at;
            p.status[l.task] = at > 8u * l.t.nbytes ? 1u : 0u;
        }
        done = (!ac && !rec) || last;                      // (bits after the plane's last block, or its end)
        dc += rec ? (uint32_t)e : 0u;
        blk += rec ? 1u : 0u;
        const uint32_t nidx = zrl ? min(idx + 16, 64u) : tt + 1;
        idx = ac ? (end ? 0u : nidx) : 1u;
    }
};

__global__ void __launch_bounds__(256) entidx_kernel(const EntParParams p) {
    __shared__ uint32_t wins[256 * kWin];  // each lane's staged window, as in the synchronisation walk
    Lane l;
    const uint32_t g = p.g0 + blockIdx.x * 256 + threadIdx.x;
    if (!lane_of(p, g, l)) return;
    if (p.unsettled && p.tchg[l.task] == p.unsettled) return;  // left to entidx_serial_kernel
    if ((uint64_t)l.t.frame * 3 + l.t.plane >= p.ntasks) return;  // (never, with a consistent task table)
    const uint64_t st = p.start[g];
    IdxStep s;
    s.blk = p.nb[g];
    const bool ac = (st >> 32) & 1u;
    s.idx = ac ? (uint32_t)(st >> 33) & 127u : 0u;
    if (s.blk > p.nblk || (s.blk == p.nblk && !ac)) return;  // wholly past the plane's last block
    Walk w(p, l, (uint32_t)st, (lds_u32*)(wins + kWin * threadIdx.x));
    const uint64_t fp3 = (uint64_t)l.t.frame * 3 + l.t.plane;
    MJ423_BOUND(fp3 * (p.nblk + 1) + p.nblk, p.lim.bpos, "bpos (index)");
    MJ423_BOUND((fp3 + 1) * p.tiles_pp - 1, p.lim.tiles, "tiles (index)");
    MJ423_BOUND(l.task, p.lim.status, "status (index)");
    uint32_t* bpos = p.bpos + fp3 * (p.nblk + 1);
    uint2* tiles = p.tiles + fp3 * p.tiles_pp;
    const bool P = l.t.ptype != 0;
    s.dc = p.dcs[g];
    s.at = w.at();  // (kept alongside the reader, as in walk_sync_bf)
    const uint32_t stop = (l.k + 1) * kSubBits;
    while (s.at < stop && !s.done) s.step<true>(p, l, w.r, bpos, tiles, P);
    if (l.k + 1 == l.nsub)  // the plane's last lane: on until its last block has ended
        while (!s.done && w.guard-- != 0) s.step<false>(p, l, w.r, bpos, tiles, P);
}

// The streams still changing after the last synchronisation iteration (tchg == unsettled: a
// periodic bit pattern, e.g. dense blocks that end only at index 63): one lane walks the whole
// plane from its first bit.
__global__ void __launch_bounds__(64) entidx_serial_kernel(const EntParParams p) {
    const uint32_t task = blockIdx.x * 64 + threadIdx.x;
    if (task < p.ntasks) MJ423_BOUND(task, p.lim.tchg, "tchg (serial index)");
    if (task >= p.ntasks || p.tchg[task] != p.unsettled) return;
    MJ423_BOUND(task, p.lim.tasks, "tasks (serial index)");
    Lane l;
    l.task = task;
    l.k = 0;
    l.nsub = 1;
    l.t = p.tasks[task];
    p.status[task] = 2u;
    Walk w(p, l, 0u);
    index_plane(p, l.t, task, w, 0u, 0u, 0xffffffffu);
}

// ---------------------------------------------------------------------------------------------
// Multi-class resolution of the streams the synchronisation leaves unsettled.
//
// A parse that enters a periodic stretch out of phase stays out of phase until the pattern breaks:
// DC-only blocks (SIZE + VLI + EOB) in a flat or static region, all-zero-block runs broken by a few
// coded blocks.  The reference encoder writes exactly that for static P-frames (tools/real_mpg.py:
// every P-plane of a clean static scene still changing after 200 iterations), and then the iteration
// moves the true parse one subsequence per round.  But only a few parses survive to a lane's end
// whatever state it is entered in: the lane's exits from all states at its start form a small set
// (1-12 on the reference's files).  So, for the lanes of those streams only:
//   classes : one wave per lane walks it from 46 seed states -- every bit offset 0-22 at which its
//             first symbol can start (a symbol takes <= 23 bits), DC or AC (index 1) -- and keeps the
//             distinct exits (<= 15, in order of the lowest seed reaching each): mc_x;
//   maps    : 16 threads per lane walk it from each of its predecessor's classes and look the exit up
//             among its own: a map class -> class (15: none) per lane, and the blocks / DC sum of each
//             walk (lane 0: from the stream's first bit, class 0);
//   resolve : per stream, a prefix composition of the maps from class 0 gives every lane's entry
//             and exit class; a lane's start, exit, nb and dcs are then its walk from the entry class.
// Exact: every walk is an exact parse from an exact state, and the chain starts at the stream's first
// bit; only the lookups can fail (the true exit not among the classes: a seed set that missed it, or
// more than 15 classes) -- a stream with any failed lookup on its path keeps tchg == unsettled and goes
// to the serial fallback as before.  Resolved streams get tchg = 1.
constexpr uint32_t kMcClasses = 15;  // classes kept per lane (nibble 15 = none)
constexpr uint32_t kMcNone = 15;
constexpr uint32_t kMcSeedOffsets = 23;  // a symbol is at most 8 + 15 bits

// The lane's window [w0, w0 + kWin) dwords, masked at the stream's end and byte-swapped (the same
// words Walk's staging writes), by nt threads (t = 0 .. nt-1).  Returns w0.
__device__ __forceinline__ uint64_t mc_stage(const EntParParams& p, const Lane& l, lds_u32* lw, uint32_t t, uint32_t nt) {
    const uint32_t* dw = reinterpret_cast<const uint32_t*>(p.bytes);
    const uint64_t dw_max = (p.bytes_len + 60) / 4, end = l.t.byte_off + l.t.nbytes;
    MJ423_BOUND(dw_max, p.lim.bytes_dw, "bytes (mc window)");
    const uint64_t b = l.t.byte_off * 8 + (uint64_t)l.k * kSubBits;
    const uint64_t w0 = (b >> 5) - ((b >> 5) ? 1 : 0);
    for (uint32_t j = t; j < kWin; j += nt) {
        const uint64_t i = w0 + j;
        const uint32_t v = dw[i < dw_max ? i : dw_max];
        const uint64_t a = 4 * i;
        const uint32_t m = a + 4 <= end ? 0xffffffffu : a >= end ? 0u : (1u << (8 * (uint32_t)(end - a))) - 1u;
        lw[j] = __builtin_bswap32(v & m);
    }
    return w0;
}

// walk_sync_bf's walk from (pos, idx: 0 = DC) to the first symbol boundary at or past `stop`, reading
// a window staged by mc_stage (from any start in the lane's first 23 bits: the walk ends <= 23 bits
// past the lane, inside the window).  Returns the packed exit state.
__device__ __forceinline__ uint64_t mc_walk(const EntParParams& p, const Lane& l, const lds_u32* lw, uint64_t w0, uint32_t pos,
                                            uint32_t idx, uint32_t stop, uint32_t& nb, uint32_t& dcs) {
    Reader r;
    r.dw = reinterpret_cast<const uint32_t*>(p.bytes);
    r.dw_max = (p.bytes_len + 60) / 4;
    r.end = l.t.byte_off + l.t.nbytes;
    r.lw = lw;
    r.w0 = w0;
    r.lds = true;
    r.init(l.t.byte_off * 8 + pos);
    uint32_t at = pos;
    nb = 0;
    dcs = 0;
    while (at < stop) {
        r.refill_lds();
        const bool A = idx != 0;
        const uint32_t hi = (uint32_t)(r.win >> 32), hi4 = hi >> 28, lo4 = (hi >> 24) & 15u;
        const uint32_t hdr = A ? 8u : 4u, size = A ? lo4 : hi4;
        const uint32_t v = __builtin_amdgcn_ubfe(hi, 32u - hdr - size, size);
        const uint32_t tot = hdr + size;
        r.win <<= tot;
        r.n -= tot;
        at += tot;
        const int32_t e = huff_extend(v, size);
        dcs += A ? 0u : (uint32_t)e;
        nb += A ? 0u : 1u;
        const uint32_t t = min(idx + hi4, 64u);
        const bool zrl = size == 0 && hi4 == 15, eob = size == 0 && hi4 != 15;
        const bool end = eob || (size != 0 && t >= 63);
        const uint32_t nidx = zrl ? min(idx + 16, 64u) : t + 1;
        idx = A ? (end ? 0u : nidx) : 1u;
    }
    return pack(at, idx != 0 ? 1u : 0u, idx);
}

__device__ __forceinline__ uint32_t mc_nib(uint64_t m, uint32_t i) { return (uint32_t)(m >> (4 * i)) & 15u; }
// "a, then b": nibble i = b[a[i]] (15 stays 15: nibble 15 of every map is 15)
__device__ __forceinline__ uint64_t mc_then(uint64_t a, uint64_t b) {
    uint64_t r = 0;
#pragma unroll
    for (uint32_t i = 0; i < 16; i++) r |= (uint64_t)mc_nib(b, mc_nib(a, i)) << (4 * i);
    return r;
}
constexpr uint64_t kMcIdentity = 0xfedcba9876543210ull;

// An all-zero lane (zrun != ~0) of subsequence k entered at state `en` (inside its first 23 bits): its
// exit and DC symbols in closed form, as zero_lane computes them -- the walk through zero bits
// alternates DC size 0 and EOB, whatever the entry's zig-zag index.
__device__ __forceinline__ uint64_t mc_zero_exit(uint64_t en, uint32_t k, uint32_t& nb) {
    const uint32_t q = (uint32_t)en, a_in = (uint32_t)(en >> 32) & 1u, d0 = q + (a_in ? 8u : 0u);
    const uint32_t end = (k + 1) * kSubBits;
    uint32_t ac, pos = zero_next(d0, end, ac);
    if (q >= end) {  // (never for an entry inside the lane)
        pos = q;
        ac = a_in;
    }
    nb = zero_dcs_between(d0, q, pos);
    return pack(pos, ac, 1);
}

// The lanes of the streams still changing in the last iteration, compacted; one workgroup per stream.
__global__ void __launch_bounds__(256) entmc_list_kernel(const EntParParams p) {
    const uint32_t task = blockIdx.x;
    MJ423_BOUND(task, p.lim.tchg, "tchg (mc list)");
    if (p.tchg[task] != p.unsettled) return;
    MJ423_BOUND(task + 1, p.lim.sub0, "sub0 (mc list)");
    const uint32_t s0 = p.sub0[task], s1 = p.sub0[task + 1];
    __shared__ uint32_t base;
    if (threadIdx.x == 0) base = atomicAdd(p.mc_count, s1 - s0);
    __syncthreads();
    for (uint32_t j = threadIdx.x; j < s1 - s0; j += 256) {
        MJ423_BOUND(base + j, p.lim.mc, "mc_list");
        p.mc_list[base + j] = s0 + j;
    }
}

// classes: one wave per listed lane, one seed per thread.
__global__ void __launch_bounds__(256) entmc_classes_kernel(const EntParParams p) {
    __shared__ uint32_t wins[4 * kWin];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint32_t count = __builtin_nontemporal_load(p.mc_count);
    lds_u32* lw = (lds_u32*)(wins + kWin * wave);
    for (uint32_t b0 = blockIdx.x * 4; b0 < count; b0 += gridDim.x * 4) {  // (uniform per workgroup)
        const uint32_t i = b0 + wave;
        Lane l;
        uint32_t g = 0;
        bool ok = false;
        if (i < count) {
            MJ423_BOUND(i, p.lim.mc, "mc_list (classes)");
            g = p.mc_list[i];
            ok = lane_of(p, g, l);
        }
        uint64_t w0 = 0;
        if (ok) w0 = mc_stage(p, l, lw, lane, 64);
        __syncthreads();
        if (ok) {  // (uniform per wave)
            const uint32_t s = lane >> 1, o = s < kMcSeedOffsets ? s : s - kMcSeedOffsets;  // lanes 46-63 repeat seeds
            const uint32_t pos = l.k == 0 ? 0u : l.k * kSubBits + o, idx = l.k == 0 ? 0u : (lane & 1u);
            uint32_t nb, dcs;
            const uint64_t e = mc_walk(p, l, lw, w0, pos, idx, (l.k + 1) * kSubBits, nb, dcs);
            uint64_t mine = ~0ull, active = __ballot(1);
            for (uint32_t c = 0; c < kMcClasses && active != 0; c++) {
                const uint32_t lead = (uint32_t)__builtin_ctzll(active);
                const uint64_t v = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(e >> 32), (int)lead) << 32) |
                                   (uint32_t)__shfl((int)(uint32_t)e, (int)lead);
                if (lane == c) mine = v;
                active &= ~__ballot(e == v);
            }
            MJ423_BOUND((uint64_t)(g - p.g0) * 16 + 15, p.lim.mc * 16, "mc_x (classes)");
            if (lane < 16) p.mc_x[(size_t)(g - p.g0) * 16 + lane] = mine;
        }
        __syncthreads();  // the windows are restaged in the next round
    }
}

// classes, in two phases: the wave walks each of four lanes' 46 seeds only until they have merged into
// at most 16 distinct parses (checkpoints every 64 bits; the seeds of a lane fall onto a few parses
// within its first symbols), then continues the four lanes' distinct parses to their ends at once,
// 16 threads per lane -- about 0.4 of a wave-walk per lane instead of one.
constexpr uint32_t kMcCheck = 64;  // bits between phase-1 checkpoints
__global__ void __launch_bounds__(256) entmc_classes2_kernel(const EntParParams p) {
    __shared__ uint32_t wins[16 * kWin];   // the 16 lanes' windows (4 per wave)
    __shared__ uint64_t part[16 * 16];     // per lane: its distinct phase-1 states (~0: none)
    __shared__ uint32_t fin[16];           // per lane: part[] holds exits (an all-zero lane)
    __shared__ uint32_t ckpt[16];          // per lane: the phase-1 checkpoint its states sit at (bits into it)
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6, jj = lane >> 4, sl = lane & 15;
    const uint64_t gmask = 0xffffull << (16 * jj);  // this thread's 16-lane group
    const uint32_t count = __builtin_nontemporal_load(p.mc_count);
    for (uint32_t b0 = blockIdx.x * 16; b0 < count; b0 += gridDim.x * 16) {  // (uniform per workgroup)
        // group jj of wave w stages (and later finishes) list entry b0 + 4w + jj
        const uint32_t me = wave * 4 + jj;
        lds_u32* lw = (lds_u32*)(wins + kWin * me);
        Lane l;
        uint32_t g = 0;
        bool ok = false;
        if (b0 + me < count) {
            MJ423_BOUND(b0 + me, p.lim.mc, "mc_list (classes)");
            g = p.mc_list[b0 + me];
            ok = lane_of(p, g, l);
        }
        uint64_t w0 = 0;
        if (ok) w0 = mc_stage(p, l, lw, sl, 16);
        __syncthreads();
        // phase 1: the wave takes its four lanes one after another, one seed per thread
        for (uint32_t j = 0; j < 4; j++) {
            const uint32_t e = b0 + wave * 4 + j;
            Lane lj;
            if (!(e < count && lane_of(p, p.mc_list[e], lj))) {  // (uniform per wave)
                if (lane < 16) part[(wave * 4 + j) * 16 + lane] = ~0ull;
                continue;
            }
            const lds_u32* lwj = (const lds_u32*)(wins + kWin * (wave * 4 + j));
            const uint64_t bj = lj.t.byte_off * 8 + (uint64_t)lj.k * kSubBits;
            const uint64_t w0j = (bj >> 5) - ((bj >> 5) ? 1 : 0);
            const uint32_t s = lane >> 1, o = s < kMcSeedOffsets ? s : s - kMcSeedOffsets;  // lanes 46-63 repeat seeds
            uint32_t pos = lj.k == 0 ? 0u : lj.k * kSubBits + o, idx = lj.k == 0 ? 0u : (lane & 1u);
            const uint32_t end = (lj.k + 1) * kSubBits;
            const bool zero = p.zrun[p.mc_list[e]] != ~0u;  // (uniform per wave)
            uint64_t st = 0, active = 0;
            uint32_t dck = kSubBits;  // the checkpoint reached
            if (zero) {  // an all-zero lane: every seed's exit in closed form, nothing to walk
                uint32_t nb;
                st = mc_zero_exit(pack(pos, idx != 0 ? 1u : 0u, idx), lj.k, nb);
            } else
            for (uint32_t d = kMcCheck;; d += kMcCheck) {  // (uniform per wave)
                const uint32_t stop = min(lj.k * kSubBits + d, end);
                dck = stop - lj.k * kSubBits;
                uint32_t nb, dcs;
                st = mc_walk(p, lj, lwj, w0j, pos, idx, stop, nb, dcs);
                pos = (uint32_t)st;
                idx = ((st >> 32) & 1u) ? (uint32_t)(st >> 33) & 127u : 0u;
                // distinct states: at most 16 by the end of the lane's bits, or stop at the lane's end anyway
                uint64_t left = __ballot(1);
                uint32_t n = 0;
                while (left != 0 && n <= 16) {
                    const uint32_t lead = (uint32_t)__builtin_ctzll(left);
                    const uint64_t v = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(st >> 32), (int)lead) << 32) |
                                       (uint32_t)__shfl((int)(uint32_t)st, (int)lead);
                    left &= ~__ballot(st == v);
                    n++;
                }
                active = left;  // (0: n <= 16 distinct)
                if ((active == 0 && n <= 16) || stop >= end) break;
            }
            // record up to 16 distinct states, lowest seed first
            uint64_t left = __ballot(1), mine = ~0ull;
            for (uint32_t c = 0; c < 16 && left != 0; c++) {
                const uint32_t lead = (uint32_t)__builtin_ctzll(left);
                const uint64_t v = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(st >> 32), (int)lead) << 32) |
                                   (uint32_t)__shfl((int)(uint32_t)st, (int)lead);
                if (lane == c) mine = v;
                left &= ~__ballot(st == v);
            }
            if (lane < 16) part[(wave * 4 + j) * 16 + lane] = mine;
            if (lane == 0) {
                fin[wave * 4 + j] = zero ? 1u : 0u;  // exits already: phase 2 has nothing to walk
                ckpt[wave * 4 + j] = dck;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");  // part[] written by this wave, read below by it
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        // phase 2: group jj finishes its lane's distinct parses, one per thread
        if (ok) {  // (uniform per group)
            const uint64_t x = part[me * 16 + sl];
            uint64_t e = ~0ull;
            uint32_t nb = 0, dcs = 0;
            if (x != ~0ull && fin[me]) {
                e = x;
            } else if (x != ~0ull) {
                e = mc_walk(p, l, lw, w0, (uint32_t)x, ((x >> 32) & 1u) ? (uint32_t)(x >> 33) & 127u : 0u, (l.k + 1) * kSubBits, nb,
                            dcs);
            }
            uint64_t left = __ballot(x != ~0ull) & gmask, mine = ~0ull;
            uint32_t mycls = 15;
            for (uint32_t c = 0; c < kMcClasses && left != 0; c++) {
                const uint32_t lead = (uint32_t)__builtin_ctzll(left);
                const uint64_t v = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(e >> 32), (int)lead) << 32) |
                                   (uint32_t)__shfl((int)(uint32_t)e, (int)lead);
                if (sl == c) mine = v;
                if (e == v) mycls = c;
                left &= ~__ballot(e == v);
            }
            MJ423_BOUND((uint64_t)(g - p.g0) * 16 + 15, p.lim.mc * 16, "mc_x (classes)");
            p.mc_x[(size_t)(g - p.g0) * 16 + sl] = mine;
            // the phase-1 states, each with its exit's class and the rest of its walk (for the maps)
            p.mc_st[(size_t)(g - p.g0) * 16 + sl] = x;
            p.mc_sfx[(size_t)(g - p.g0) * 16 + sl] = mycls | ((nb & 0xfffu) << 4) | (dcs << 16);
            if (sl == 0) p.mc_ck[g - p.g0] = fin[me] ? kSubBits : ckpt[me];
        }
        __syncthreads();  // windows and part[] are rewritten in the next round
    }
}

// maps: 16 threads per listed lane, one per predecessor class.
__global__ void __launch_bounds__(256) entmc_maps_kernel(const EntParParams p) {
    __shared__ uint32_t wins[16 * kWin];
    __shared__ uint64_t sst[16 * 16];  // per lane: the classes kernel's phase-1 states ...
    __shared__ uint32_t ssf[16 * 16];  // ... and their suffixes
    const uint32_t j = threadIdx.x & 15, slot = threadIdx.x >> 4;
    const uint32_t count = __builtin_nontemporal_load(p.mc_count);
    lds_u32* lw = (lds_u32*)(wins + kWin * slot);
    for (uint32_t b0 = blockIdx.x * 16; b0 < count; b0 += gridDim.x * 16) {  // (uniform per workgroup)
        const uint32_t i = b0 + slot;
        Lane l;
        uint32_t g = 0;
        bool ok = false;
        if (i < count) {
            MJ423_BOUND(i, p.lim.mc, "mc_list (maps)");
            g = p.mc_list[i];
            ok = lane_of(p, g, l);
        }
        uint64_t w0 = 0;
        if (ok) {
            w0 = mc_stage(p, l, lw, j, 16);
            sst[slot * 16 + j] = p.mc_st[(size_t)(g - p.g0) * 16 + j];
            ssf[slot * 16 + j] = p.mc_sfx[(size_t)(g - p.g0) * 16 + j];
        }
        __syncthreads();
        uint64_t m = 0;
        if (ok) {  // (uniform per 16 threads)
            const size_t r = (size_t)(g - p.g0) * 16;
            MJ423_BOUND(r + 15, p.lim.mc * 16, "mc_x / mc_rec (maps)");
            if (l.k > 0) MJ423_BOUND(r - 16, p.lim.mc * 16, "mc_x (maps, predecessor)");
            const uint64_t x = l.k == 0 ? (j == 0 ? pack(0, 0, 0) : ~0ull) : p.mc_x[r - 16 + j];
            const uint64_t own = p.mc_x[r + j];  // this lane's class j (thread j holds it)
            uint32_t cls = kMcNone, rec = 0;
            uint64_t y = ~0ull;
            if (x != ~0ull && p.zrun[g] != ~0u) {  // an all-zero lane: closed form (DC differences all 0)
                uint32_t nb;
                y = mc_zero_exit(x, l.k, nb);
                rec = nb & 0xffffu;
            } else if (x != ~0ull) {
                // walk to the lane's phase-1 checkpoint; where the parse has met one of the phase-1 states,
                // the rest of its walk is that state's (the classes kernel walked it)
                uint32_t nb, dcs;
                const uint64_t s1 = mc_walk(p, l, lw, w0, (uint32_t)x, ((x >> 32) & 1u) ? (uint32_t)(x >> 33) & 127u : 0u,
                                            l.k * kSubBits + p.mc_ck[g - p.g0], nb, dcs);
                uint32_t hit = 16;
                for (uint32_t q = 0; q < 16; q++)
                    if (sst[slot * 16 + q] != ~0ull && sst[slot * 16 + q] == s1) hit = q;
                const uint32_t sf = ssf[slot * 16 + (hit & 15u)];
                if (hit < 16) {
                    cls = sf & 15u;
                    rec = ((nb + ((sf >> 4) & 0xfffu)) & 0xffffu) | ((dcs + (sf >> 16)) << 16);
                } else {
                    uint32_t nb2, dcs2;
                    y = mc_walk(p, l, lw, w0, (uint32_t)s1, ((s1 >> 32) & 1u) ? (uint32_t)(s1 >> 33) & 127u : 0u, (l.k + 1) * kSubBits,
                                nb2, dcs2);
                    rec = ((nb + nb2) & 0xffffu) | ((dcs + dcs2) << 16);
                }
            }
#pragma unroll
            for (uint32_t c = 0; c < kMcClasses; c++) {
                const uint64_t xc = ((uint64_t)(uint32_t)__shfl((int)(uint32_t)(own >> 32), (int)c, 16) << 32) |
                                    (uint32_t)__shfl((int)(uint32_t)own, (int)c, 16);
                if (y != ~0ull && xc == y) cls = c;
            }
            p.mc_rec[r + j] = rec;
            m = (uint64_t)cls << (4 * j);
        }
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {  // OR the slot's 16 nibbles
            const uint64_t t = ((uint64_t)(uint32_t)__shfl_xor((int)(uint32_t)(m >> 32), o, 16) << 32) |
                               (uint32_t)__shfl_xor((int)(uint32_t)m, o, 16);
            m |= t;
        }
        if (ok && j == 0) p.mc_map[g - p.g0] = m;
        __syncthreads();
    }
}

// resolve: per listed stream, the classes along the true parse by a prefix composition of the maps.
__global__ void __launch_bounds__(kScanThreads) entmc_resolve_kernel(const EntParParams p) {
    constexpr uint32_t W = kScanThreads / 64;
    const uint32_t task = blockIdx.x;
    MJ423_BOUND(task, p.lim.tchg, "tchg (mc resolve)");
    if (p.tchg[task] != p.unsettled) return;
    MJ423_BOUND(task + 1, p.lim.sub0, "sub0 (mc resolve)");
    const uint32_t s0 = p.sub0[task], s1 = p.sub0[task + 1];
    if (s1 > s0) {
        MJ423_BOUND(s1 - 1, p.lim.lanes, "lanes (mc resolve)");
        MJ423_BOUND((uint64_t)(s1 - 1 - p.g0) * 16 + 15, p.lim.mc * 16, "mc (resolve)");
    }
    __shared__ uint64_t wmap[W];
    __shared__ uint32_t miss;
    if (threadIdx.x == 0) miss = 0;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t carry = 0;  // class of the exit before the chunk (lane 0 enters at the one "class" 0: bit 0, DC)
    for (uint32_t c = s0; c < s1; c += kScanThreads) {
        const uint32_t g = c + threadIdx.x;
        uint64_t f = g < s1 ? p.mc_map[g - p.g0] : kMcIdentity;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {  // inclusive: f = this lane's map after its predecessors' in the wave
            const uint64_t t = ((uint64_t)(uint32_t)__shfl_up((int)(uint32_t)(f >> 32), o) << 32) |
                               (uint32_t)__shfl_up((int)(uint32_t)f, o);
            if (lane >= (uint32_t)o) f = mc_then(t, f);
        }
        if (lane == 63) wmap[wave] = f;
        __syncthreads();
        uint32_t cin = carry, all = carry;
#pragma unroll
        for (uint32_t w = 0; w < W; w++) {
            if (w < wave) cin = mc_nib(wmap[w], cin);
            all = mc_nib(wmap[w], all);
        }
        const uint32_t cg = mc_nib(f, cin);  // the class of lane g's exit
        uint32_t eg = (uint32_t)__shfl_up((int)cg, 1);
        if (lane == 0) eg = cin;  // the class of its entry
        if (g < s1) {
            if (cg == kMcNone || eg == kMcNone) {
                miss = 1u;
            } else {
                const size_t r = (size_t)(g - p.g0) * 16;
                const uint32_t rec = p.mc_rec[r + eg];
                p.start[g] = g == s0 ? pack(0, 0, 0) : p.mc_x[r - 16 + eg];
                p.exit_[g] = p.mc_x[r + cg];
                p.nb[g] = rec & 0xffffu;
                p.dcs[g] = rec >> 16;
            }
        }
        carry = all;
        __syncthreads();
    }
    if (threadIdx.x == 0 && miss == 0) p.tchg[task] = 1u;  // settled; else left to the serial fallback
}

}  // namespace mj423

extern "C" hipError_t mj423_launch_entpar_index(const mj423::EntParParams* p, hipStream_t stream) {
    if (p->nsub <= p->g0) return hipSuccess;
    hipLaunchKernelGGL(mj423::entpar_scan_kernel, dim3(p->ntasks), dim3(mj423::kScanThreads), 0, stream, *p);
    hipLaunchKernelGGL(mj423::entidx_kernel, dim3((p->nsub - p->g0 + 255) / 256), dim3(256), 0, stream, *p);
    if (p->unsettled)
        hipLaunchKernelGGL(mj423::entidx_serial_kernel, dim3((p->ntasks + 63) / 64), dim3(64), 0, stream, *p);
    return hipGetLastError();
}

extern "C" hipError_t mj423_launch_entpar(const mj423::EntParParams* p, uint32_t max_iters, hipStream_t stream) {
    if (p->nsub <= p->g0) return hipSuccess;
    // every table the launches index, present (a null one would fault on the device, not here)
    if (!p->bytes || !p->tasks || !p->sub0 || !p->start || !p->exit_ || !p->nb || !p->dcs || !p->flags || !p->zrun || !p->zlast ||
        !p->lane_task || !p->tchg || !p->wcnt || !p->status || !p->qbits ||
        (p->mc_list && (!p->mc_count || !p->mc_x || !p->mc_map || !p->mc_rec || !p->mc_st || !p->mc_sfx || !p->mc_ck)))
        return hipErrorInvalidValue;
    const dim3 grid((p->nsub - p->g0 + 255) / 256);
    hipLaunchKernelGGL(mj423::entpar_map_kernel, dim3(p->ntasks), dim3(256), 0, stream, *p);
#if !MJ423_INIT_IN_IT0
    hipLaunchKernelGGL(mj423::entpar_init_kernel, grid, dim3(256), 0, stream, *p);
    hipLaunchKernelGGL(mj423::entpar_zrun_kernel, dim3(p->ntasks), dim3(mj423::kScanThreads), 0, stream, *p);
#endif
    // list iterations: chunks of 32 * kListWords lanes, grid-stride over at most MJ423_LIST_GRID
    // workgroups (an empty list costs a short launch: the dispatch of a few hundred workgroups)
#ifndef MJ423_LIST_GRID
#define MJ423_LIST_GRID 4096
#endif
    const dim3 lgrid(std::min<uint32_t>((p->nsub - p->g0 + 32 * mj423::kListWords - 1) / (32 * mj423::kListWords) + 1, MJ423_LIST_GRID));
    for (uint32_t it = 0; it < max_iters; it++) {
        if (it < 2)
            hipLaunchKernelGGL(mj423::entpar_sync_kernel, dim3((p->nsub - p->g0 + mj423::kSyncThreads - 1) / mj423::kSyncThreads),
                               dim3(mj423::kSyncThreads), 0, stream, *p, it);
        else
            hipLaunchKernelGGL(mj423::entpar_sync_list_kernel, lgrid, dim3(mj423::kListThreads), 0, stream, *p, it);
#if MJ423_INIT_IN_IT0
        if (it == 0)  // the zero runs, from iteration 0's all-zero tests
            hipLaunchKernelGGL(mj423::entpar_zrun_kernel, dim3(p->ntasks), dim3(mj423::kScanThreads), 0, stream, *p);
#endif
    }
    if (p->mc_list) {  // streams still changing: multi-class resolution (the grids loop over the list)
        const uint32_t lanes = p->nsub - p->g0;
        hipLaunchKernelGGL(mj423::entmc_list_kernel, dim3(p->ntasks), dim3(256), 0, stream, *p);
#ifndef MJ423_MC_CLASSES
#define MJ423_MC_CLASSES 2
#endif
        if (MJ423_MC_CLASSES == 2)
            hipLaunchKernelGGL(mj423::entmc_classes2_kernel, dim3(std::min<uint32_t>((lanes + 15) / 16, 512u)), dim3(256), 0, stream, *p);
        else
            hipLaunchKernelGGL(mj423::entmc_classes_kernel, dim3(std::min<uint32_t>((lanes + 3) / 4, 1024u)), dim3(256), 0, stream, *p);
        hipLaunchKernelGGL(mj423::entmc_maps_kernel, dim3(std::min<uint32_t>((lanes + 15) / 16, 512u)), dim3(256), 0, stream, *p);
        hipLaunchKernelGGL(mj423::entmc_resolve_kernel, dim3(p->ntasks), dim3(mj423::kScanThreads), 0, stream, *p);
    }
    return hipGetLastError();
}

extern "C" hipError_t mj423_launch_entpar_finish(const mj423::EntParParams* p, hipStream_t stream) {
    if (p->nsub <= p->g0) return hipSuccess;
    hipLaunchKernelGGL(mj423::entpar_scan_kernel, dim3(p->ntasks), dim3(mj423::kScanThreads), 0, stream, *p);
    hipLaunchKernelGGL(mj423::entpar_emit_kernel, dim3((p->nsub - p->g0 + 255) / 256), dim3(256), 0, stream, *p);
    return hipGetLastError();
}
