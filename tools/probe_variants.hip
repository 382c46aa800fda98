// tools/probe_variants.hip -- stream-kernel variants kept for tools/probe.hip A/B runs only
// (measured, not production).  Included by the probe after mj423_kernels.hip.
namespace mj423 {

// Stream decode, register-state form (kGopRegState).  Same walk as decode_gop_kernel, but
// the accumulated quantized coefficients live in the VGPRs of the lanes that stage them
// (chunk k of lane t: 16 B, CHUNKS * 4 VGPRs per lane -- 24 at 4:2:0), so the LDS holds only
// what the batch kernel's does: the frame's coefficient slots, overlaid by the plane tiles
// after the IDCT has read them.  A P-frame's deltas are added in registers as they arrive
// (lossless_decode.c:90-92,121-122 in the quantized domain, mod 2^16).  kGopEarly: the next
// frame's loads are issued right after the state has been staged (in flight during IDCT + CSC).
template <int MODE, int TW, int THREADS, int FLAGS = kDefaultFlags, int WPE = 1>
__global__ void __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(WPE)))
decode_gop_reg_kernel(const DecodeParams p) {
    using T = Tile<MODE, TW, THREADS>;
    __shared__ __attribute__((aligned(16))) uint8_t lds[T::LDS_BYTES + 256];
    uint32_t* lds_qt = reinterpret_cast<uint32_t*>(lds + T::LDS_BYTES);  // never overlaid by the planes
    const int tid0 = threadIdx.x;
    if (tid0 < 16)  // ordered before the first IDCT by the first staging barrier
        reinterpret_cast<uint4*>(lds_qt)[tid0] = reinterpret_cast<const uint4*>(p.qt_dev)[tid0];
    const uint32_t tiles_per_frame = p.tiles_per_frame;
    uint32_t tx, sy;
    if (!gop_job(p, tx, sy)) return;  // (whole workgroup, before any barrier)
    const uint32_t f0 = p.seg_start[sy], f1 = p.seg_start[sy + 1];
    const TileCoord cs = tile_coord<MODE>(p, tx);  // frame-0 coordinates (state buffers)
    auto st_off = [&](int k, int tid) -> int64_t {
        const int run = T::chunk_run(k);
        const int col = T::SLOTS_PER_CHUNK * k + (tid >> 3) - T::run_first_slot(run);
        const int colc = col < cs.run_len(run) ? col : 0;
        const int64_t o = cs.run_off(run) + colc * 64 + (tid & 7) * 8;
        return run < 2 ? o : run == 2 ? o - p.cb_off + p.st_cb_off : o - p.cr_off + p.st_cr_off;
    };
    u32x4 st[T::CHUNKS];
    if (p.ftype[f0] != 0) {  // the segment continues a GOP: seed the state from p.state
#pragma unroll
        for (int k = 0; k < T::CHUNKS; k++) st[k] = *reinterpret_cast<const u32x4*>(p.state + st_off(k, tid0));
    } else {
#pragma unroll
        for (int k = 0; k < T::CHUNKS; k++) st[k] = (u32x4){0u, 0u, 0u, 0u};
    }
    constexpr bool EARLY = (FLAGS & kGopEarly) != 0;
    u32x4 v[T::CHUNKS];
    TileCoord c;
    if (EARLY && f0 < f1) {
        c = tile_coord<MODE>(p, f0 * tiles_per_frame + tx);
        stage_load<MODE, TW, THREADS, FLAGS>(p, c, tid0, v);
    }
    for (uint32_t f = f0; f < f1; f++) {
        int tid = tid0;
        asm volatile("" : "+v"(tid));  // lane-derived addresses recomputed per frame, not kept live
        if (!EARLY) {
            c = tile_coord<MODE>(p, f * tiles_per_frame + tx);
            stage_load<MODE, TW, THREADS, FLAGS>(p, c, tid, v);
        }
        if (p.ftype[f] != 0) {  // P: deltas onto the state
#pragma unroll
            for (int k = 0; k < T::CHUNKS; k++)
                st[k] = (u32x4){add_u16x2(st[k].x, v[k].x), add_u16x2(st[k].y, v[k].y), add_u16x2(st[k].z, v[k].z),
                                add_u16x2(st[k].w, v[k].w)};
        } else {
#pragma unroll
            for (int k = 0; k < T::CHUNKS; k++) st[k] = v[k];
        }
        stage_store<MODE, TW, THREADS, kDefaultFlags>(lds, tid, st);
        __syncthreads();
        TileCoord cn = c;
        if (EARLY && f + 1 < f1) {
            cn = tile_coord<MODE>(p, (f + 1) * tiles_per_frame + tx);
            stage_load<MODE, TW, THREADS, FLAGS>(p, cn, tid, v);
        }
        decode_tile<MODE, TW, THREADS, FLAGS | kGopLdsQt>(p, c, lds, tid, lds_qt);
        __syncthreads();  // the CSC's plane reads finish before the next frame's staging overwrites them
        c = cn;
    }
    if (p.state_out && sy + 1 == p.nseg) {  // end state, for a batch that continues this GOP
#pragma unroll
        for (int k = 0; k < T::CHUNKS; k++) {
            const int run = T::chunk_run(k);
            const int col = T::SLOTS_PER_CHUNK * k + (tid0 >> 3) - T::run_first_slot(run);
            if (col < cs.run_len(run)) *reinterpret_cast<u32x4*>(p.state_out + st_off(k, tid0)) = st[k];
        }
    }
}

// Stream decode with loader waves (measured, not production: DESIGN §4.2).  A workgroup is two
// groups of THREADS lanes:
//   * loader waves (THREADS..2*THREADS-1): hold the tile's accumulated quantized coefficients
//     in VGPRs -- chunk k of loader lane t is the 16 B it stages, exactly the batch kernel's
//     staging pattern -- and keep the NEXT frame's loads in flight while the current frame
//     is transformed: after folding frame f's data into the state (I: replace, P: add mod
//     2^16, lossless_decode.c:90-92,121-122 in the quantized domain) they issue frame f+1's
//     loads at once, so a whole frame's time covers their latency;
//   * compute waves (0..THREADS-1): the batch kernel's IDCT + CSC on the staged slots (plane
//     tiles overlaying them).  They never load from HBM, so their vmcnt holds only stores
//     and nothing ever waits for a store to drain.
// LDS is the batch kernel's (24 KiB at 4:2:0, the state lives in registers) and no wave
// holds both the state and the IDCT's registers, so the kernel fits the batch kernel's
// register budget (<= 80 VGPRs: six waves per SIMD, three 8-wave workgroups per CU) --
// against four 4-wave workgroups per CU for the LDS-state kernel above, whose 36 KiB of LDS
// and ~120 VGPRs cost ~9 % at 4K (probe: the batch kernel given the same LDS).
// Barriers per frame: A (CSC of f-1 done: the slots may be refilled), B (slots staged),
// C (inside decode_tile_idct: every block is in registers, the slots become plane tiles),
// D (plane tiles written).
template <int MODE, int TW, int THREADS, int FLAGS = kDefaultFlags, int WPE = 6>
__global__ void __launch_bounds__(2 * THREADS) __attribute__((amdgpu_waves_per_eu(WPE)))
decode_gop_ws_kernel(const DecodeParams p) {
    using T = Tile<MODE, TW, THREADS>;
    __shared__ __attribute__((aligned(16))) uint8_t lds[T::LDS_BYTES];
    const uint32_t tiles_per_frame = p.tiles_per_frame;
    uint32_t tx, sy;
    if (!gop_job(p, tx, sy)) return;  // (whole workgroup, before any barrier)
    const uint32_t f0 = p.seg_start[sy], f1 = p.seg_start[sy + 1];
    const bool loader = __builtin_amdgcn_readfirstlane(threadIdx.x) >= THREADS;  // wave-uniform role
    if (!loader) {
        const int tid0 = threadIdx.x;
        const int tid = tid0;
        // The wave's dequantization table (luma or chroma: a wave's slots share a plane class,
        // and a lane keeps its slot in every frame) read once into SGPRs for the whole segment.
        const int wc = __builtin_amdgcn_readfirstlane(T::slot_run(tid) >= 2 ? 1 : 0);
        uint32_t qs[32];
#pragma unroll
        for (int i = 0; i < 32; i++) qs[i] = __builtin_amdgcn_readfirstlane(p.qt_dev[32 * wc + i]);
        for (uint32_t f = f0; f < f1; f++) {
            // lane-derived addresses are recomputed every frame (a few VALU ops) instead of
            // being hoisted out of the loop and kept live across the IDCT (~+40 VGPRs)
            int tid = tid0;
            asm volatile("" : "+v"(tid));
            __syncthreads();  // A
            __syncthreads();  // B: the loaders have staged frame f
            const TileCoord c = tile_coord<MODE>(p, f * tiles_per_frame + tx);
            decode_tile_idct<MODE, TW, THREADS, FLAGS, true>(p, c, lds, lds, tid, nullptr, qs);  // C inside
            __syncthreads();  // D
            if constexpr ((FLAGS & kWsCscAll) != 0)
                decode_tile_csc<MODE, TW, THREADS, FLAGS, 2 * THREADS>(p, c, lds, tid);
            else
                decode_tile_csc<MODE, TW, THREADS, FLAGS>(p, c, lds, tid);
        }
        return;
    }
    // ---- loader waves
    const int lt = threadIdx.x - THREADS;
    const TileCoord cs = tile_coord<MODE>(p, tx);  // frame-0 coordinates (state buffers)
    auto st_off = [&](int k) -> int64_t {
        const int run = T::chunk_run(k);
        const int col = T::SLOTS_PER_CHUNK * k + (lt >> 3) - T::run_first_slot(run);
        const int colc = col < cs.run_len(run) ? col : 0;
        const int64_t o = cs.run_off(run) + colc * 64 + (lt & 7) * 8;
        return run < 2 ? o : run == 2 ? o - p.cb_off + p.st_cb_off : o - p.cr_off + p.st_cr_off;
    };
    // A lane's chunks sit at the same byte offsets inside every frame's planes: 32-bit buffer
    // offsets from the lane index (recomputed per frame -- kept live they would cost a VGPR per
    // chunk), the frame's plane bases in SGPRs.  Slots past a short edge tile re-read block 0
    // of their run, as in stage_load.
    const int64_t in_plane[4] = {cs.off0, cs.off1, cs.off2 - p.cb_off, cs.off3 - p.cr_off};
    auto load_frame = [&](uint32_t f, u32x4 (&dst)[T::CHUNKS]) {
        int l = lt;
        asm volatile("" : "+v"(l));
        const int16_t* fy = p.coef + (int64_t)f * (int64_t)p.plane_fstride;
        const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(const_cast<int16_t*>(fy), 0, -1, 0x00020000);
        const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(const_cast<int16_t*>(fy + p.cb_off), 0, -1, 0x00020000);
        const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(const_cast<int16_t*>(fy + p.cr_off), 0, -1, 0x00020000);
        constexpr int aux = (FLAGS & kNtLoad) ? 2 : 0;
#pragma unroll
        for (int k = 0; k < T::CHUNKS; k++) {
            const int run = T::chunk_run(k);
            const int col = T::SLOTS_PER_CHUNK * k + (l >> 3) - T::run_first_slot(run);
            const int colc = col < cs.run_len(run) ? col : 0;
            const uint32_t voff = (uint32_t)(2 * in_plane[run]) + (uint32_t)(colc * 128 + (l & 7) * 16);
            dst[k] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(run < 2 ? ry : run == 2 ? rb : rr,
                                                                                     voff, 0, aux));
        }
    };
    u32x4 st[T::CHUNKS], v[T::CHUNKS];
    if (f0 < f1 && p.ftype[f0] != 0) {  // the segment continues a GOP: seed the state from p.state
#pragma unroll
        for (int k = 0; k < T::CHUNKS; k++) st[k] = *reinterpret_cast<const u32x4*>(p.state + st_off(k));
    } else {
#pragma unroll
        for (int k = 0; k < T::CHUNKS; k++) st[k] = (u32x4){0u, 0u, 0u, 0u};
    }
    uint32_t ft = 0;
    if (f0 < f1) {
        ft = p.ftype[f0];
        load_frame(f0, v);
    }
    for (uint32_t f = f0; f < f1; f++) {
        // I: state = v; P: state += v (mod 2^16) -- one branch-free form, so the state keeps
        // its registers across the loop (an if/else made the compiler carry two copies)
        const uint32_t keep = __builtin_amdgcn_readfirstlane(ft) != 0 ? 0xffffffffu : 0u;
#pragma unroll
        for (int k = 0; k < T::CHUNKS; k++)
            st[k] = (u32x4){add_u16x2(st[k].x & keep, v[k].x), add_u16x2(st[k].y & keep, v[k].y),
                            add_u16x2(st[k].z & keep, v[k].z), add_u16x2(st[k].w & keep, v[k].w)};
        if (f + 1 < f1) {  // v is free: frame f+1's loads fly while frame f is transformed
            ft = p.ftype[f + 1];
            load_frame(f + 1, v);
        }
        __syncthreads();  // A: the compute waves are done with frame f-1's plane tiles
        stage_store<MODE, TW, THREADS, kDefaultFlags>(lds, lt, st);
        __syncthreads();  // B
        __syncthreads();  // C
        __syncthreads();  // D
        if constexpr ((FLAGS & kWsCscAll) != 0) {
            // a fixed number of stores (kStaticStores) behind the loads just issued: the next
            // frame's wait for them is vmcnt(#stores), never a wait for the stores
            static_assert((FLAGS & kStaticStores) != 0, "loader waves store only with a static store count");
            int t = threadIdx.x;
            asm volatile("" : "+v"(t));
            decode_tile_csc<MODE, TW, THREADS, FLAGS, 2 * THREADS>(p, tile_coord<MODE>(p, f * tiles_per_frame + tx), lds, t);
        }
    }
    if (p.state_out && sy + 1 == p.nseg) {  // end state, for a batch that continues this GOP
#pragma unroll
        for (int k = 0; k < T::CHUNKS; k++) {
            const int run = T::chunk_run(k);
            const int col = T::SLOTS_PER_CHUNK * k + (lt >> 3) - T::run_first_slot(run);
            if (col < cs.run_len(run)) *reinterpret_cast<u32x4*>(p.state_out + st_off(k)) = st[k];
        }
    }
}

// LDS-state stream kernel with only STAGE of its THREADS lanes staging (the rest join the
// CSC) at WPE waves per SIMD: more waves per workgroup for the same LDS.
// STAGE < THREADS: only the first STAGE lanes stage (and hold the prefetched next frame in
// registers); the others take part in the CSC only (more waves per workgroup for the same LDS).
// WPE: amdgpu_waves_per_eu (the compiler keeps VGPRs <= 512 / WPE).
template <int MODE, int TW, int THREADS, int FLAGS = kDefaultFlags, int STAGE = THREADS, int WPE = 1>
__global__ void __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(WPE)))
decode_gop_wide_kernel(const DecodeParams p) {
    using T = Tile<MODE, TW, STAGE>;
    static_assert(STAGE % 64 == 0 && STAGE <= THREADS, "staging lanes: whole waves");
    constexpr bool LDSQT = (FLAGS & kGopLdsQt) != 0;
    __shared__ __attribute__((aligned(16))) uint8_t lds[T::COEF_BYTES + T::PLANE_BYTES + (LDSQT ? 256 : 0)];
    uint8_t* state = lds;                  // quantized coefficient slots, persistent
    uint8_t* planes = lds + T::COEF_BYTES;  // uint8 plane tiles, per frame
    uint32_t* lds_qt = reinterpret_cast<uint32_t*>(lds + T::COEF_BYTES + T::PLANE_BYTES);  // LDSQT only
    const int tid0 = threadIdx.x;
    const int tid = tid0;
    if (LDSQT && tid < 16)  // ordered before the first IDCT by the first staging barrier
        reinterpret_cast<uint4*>(lds_qt)[tid] = reinterpret_cast<const uint4*>(p.qt_dev)[tid];
    const uint32_t tiles_per_frame = p.tiles_per_frame;
    // Workgroup order: tile-major inside a segment, so the resident workgroups walk the same
    // frames together.  (Measured alternatives, tools/ab_env.sh: a contiguous tile range per
    // XCD -1 %; consecutive workgroups on consecutive segments of one tile -5 %; groups of 4
    // or 8 segments interleaved like the batch kernel's frame groups -1 % / -5 %.)
    uint32_t tx, sy;
    if (!gop_job(p, tx, sy)) return;  // (whole workgroup, before any barrier)
    const bool stager = STAGE == THREADS || __builtin_amdgcn_readfirstlane(tid0) < STAGE;  // wave-uniform
    const uint32_t f0 = p.seg_start[sy], f1 = p.seg_start[sy + 1];
    // Chunk k of this lane in the state buffers ([Y | Cb | Cr] per frame).
    const TileCoord cs = tile_coord<MODE>(p, tx);  // frame-0 coordinates: no frame offset
    auto st_off = [&](int k) -> int64_t {
        const int run = T::chunk_run(k);
        const int col = T::SLOTS_PER_CHUNK * k + (tid >> 3) - T::run_first_slot(run);
        const int colc = col < cs.run_len(run) ? col : 0;
        const int64_t o = cs.run_off(run) + colc * 64 + (tid & 7) * 8;
        return run < 2 ? o : run == 2 ? o - p.cb_off + p.st_cb_off : o - p.cr_off + p.st_cr_off;
    };
    if (stager && p.ftype[f0] != 0) {  // the segment continues a GOP: seed the slots from p.state
        u32x4 v[T::CHUNKS];
#pragma unroll
        for (int k = 0; k < T::CHUNKS; k++) v[k] = *reinterpret_cast<const u32x4*>(p.state + st_off(k));
        stage_store<MODE, TW, STAGE, kDefaultFlags>(state, tid, v);
    }
    // Frame loop.  kGopPrefetch: frame f+1's loads are issued after frame f's IDCT, so they
    // are in flight during its CSC (the IDCT's registers are dead by then).
    constexpr bool EARLY = (FLAGS & kGopEarly) != 0;
    constexpr bool PREFETCH = (FLAGS & (kGopPrefetch | kGopEarly)) != 0;
    u32x4 v[T::CHUNKS];
    TileCoord c;
    // kStaticStores: the next frame's type is loaded with its coefficients (before this frame's
    // stores), so reading it never waits for the stores either.
    constexpr bool STATIC = (FLAGS & kStaticStores) != 0;
    uint32_t ft = f0 < f1 ? p.ftype[f0] : 0u;
    if (PREFETCH && f0 < f1) {
        c = tile_coord<MODE>(p, f0 * tiles_per_frame + tx);
        if (stager) stage_load<MODE, TW, STAGE, FLAGS>(p, c, tid0, v);
    }
    for (uint32_t f = f0; f < f1; f++) {
        // Lane-derived addresses are recomputed every frame (a few VALU ops) instead of
        // being hoisted out of the loop and kept live across the IDCT (~+40 VGPRs).
        int tid = tid0;
        asm volatile("" : "+v"(tid));
        if (!PREFETCH) {
            c = tile_coord<MODE>(p, f * tiles_per_frame + tx);
            if (stager) stage_load<MODE, TW, STAGE, FLAGS>(p, c, tid, v);
        }
        if (stager) {
            if (!STATIC) ft = p.ftype[f];
            if (__builtin_amdgcn_readfirstlane(ft) != 0) {  // P: accumulate deltas onto the state (each chunk has one owner lane)
#pragma unroll
                for (int k = 0; k < T::CHUNKS; k++) {
                    const u32x4 o = *reinterpret_cast<const u32x4*>(
                                        state + coef_off(T::SLOTS_PER_CHUNK * k + (tid >> 3), tid & 7)),
                                d = v[k];
                    v[k] = (u32x4){add_u16x2(o.x, d.x), add_u16x2(o.y, d.y), add_u16x2(o.z, d.z), add_u16x2(o.w, d.w)};
                }
            }
            stage_store<MODE, TW, STAGE, kDefaultFlags>(state, tid, v);
        }
        __syncthreads();
        TileCoord cn = c;
        if (EARLY && f + 1 < f1) {  // v is free again: next frame's loads overlap the IDCT too
            cn = tile_coord<MODE>(p, (f + 1) * tiles_per_frame + tx);
            if (stager) {
                stage_load<MODE, TW, STAGE, FLAGS>(p, cn, tid, v);
                if (STATIC) ft = p.ftype[f + 1];
            }
        }
        decode_tile_idct<MODE, TW, STAGE, FLAGS, false>(p, c, state, planes, tid, lds_qt);
        __syncthreads();
        if (!EARLY && PREFETCH && f + 1 < f1) {
            cn = tile_coord<MODE>(p, (f + 1) * tiles_per_frame + tx);
            if (stager) {
                stage_load<MODE, TW, STAGE, FLAGS>(p, cn, tid, v);
                if (STATIC) ft = p.ftype[f + 1];
            }
        }
        decode_tile_csc<MODE, TW, STAGE, FLAGS, THREADS>(p, c, planes, tid);
        // no barrier here: the next frame's staging barrier orders these plane reads
        // before the next IDCT overwrites the planes (state slots and planes are disjoint)
        c = cn;
    }
    __syncthreads();  // the last frame's state writes are visible to the end-state copy
    if (stager && p.state_out && sy + 1 == p.nseg) {  // end state, for a batch that continues this GOP
#pragma unroll
        for (int k = 0; k < T::CHUNKS; k++) {
            const int run = T::chunk_run(k);
            const int col = T::SLOTS_PER_CHUNK * k + (tid >> 3) - T::run_first_slot(run);
            if (col < cs.run_len(run))
                *reinterpret_cast<u32x4*>(p.state_out + st_off(k)) =
                    *reinterpret_cast<const u32x4*>(state + coef_off(T::SLOTS_PER_CHUNK * k + (tid >> 3), tid & 7));
        }
    }
}

// LDS-state stream kernel with dedicated loader waves.  A workgroup = THREADS compute lanes
// (IDCT + CSC exactly as decode_gop_kernel, never a load from HBM) + 64 * LW loader lanes.
// The accumulated quantized coefficients stay in LDS (as in decode_gop_kernel); the loader
// waves hold the NEXT frame's deltas in VGPRs and fold them into the LDS state while the
// compute waves run the previous frame's CSC, then issue the following frame's loads at once.
// Per frame f (barriers B_f, A_f):
//   compute: B_f  IDCT(f): state -> planes  A_f  CSC(f): planes -> HBM
//   loader :      fold v(f) into state, load v(f+1) ...  B_f  A_f
// so v(f+1) is in flight from the middle of CSC(f-1) through IDCT(f), the fold is off the
// compute waves' critical path, and the compute waves' vmcnt holds stores only.
// Loader chunk k of loader lane t: slot 16k + t/8, row t%8 (a wave reads 1 KiB contiguous).
template <int MODE, int TW, int THREADS, int FLAGS, int LW, int WPE, int D = 1>
__global__ void __launch_bounds__(THREADS + 64 * LW) __attribute__((amdgpu_waves_per_eu(WPE)))
decode_gop_lw_kernel(const DecodeParams p) {
    using T = Tile<MODE, TW, THREADS>;
    constexpr int LL = 64 * LW;                 // loader lanes
    constexpr int SPC = LL / 8;                 // slots per loader chunk
    constexpr int LCH = T::NSLOT / SPC;         // loader chunks per lane
    static_assert(T::NSLOT % SPC == 0 && (T::YRUN % SPC) == 0 && (TW % SPC) == 0, "loader chunks align to runs");
    __shared__ __attribute__((aligned(16))) uint8_t lds[T::COEF_BYTES + T::PLANE_BYTES + 256];
    uint8_t* state = lds;
    uint8_t* planes = lds + T::COEF_BYTES;
    uint32_t* lds_qt = reinterpret_cast<uint32_t*>(lds + T::COEF_BYTES + T::PLANE_BYTES);
    const uint32_t tiles_per_frame = p.tiles_per_frame;
    uint32_t tx, sy;
    if (!gop_job(p, tx, sy)) return;  // (whole workgroup, before any barrier)
    const uint32_t f0 = p.seg_start[sy], f1 = p.seg_start[sy + 1];
    const bool loader = __builtin_amdgcn_readfirstlane((int)threadIdx.x) >= THREADS;  // wave-uniform role
    if (!loader) {
        const int tid0 = threadIdx.x;
        if (tid0 < 16)  // ordered before the first IDCT by B_f0
            reinterpret_cast<uint4*>(lds_qt)[tid0] = reinterpret_cast<const uint4*>(p.qt_dev)[tid0];
        for (uint32_t f = f0; f < f1; f++) {
            int tid = tid0;
            asm volatile("" : "+v"(tid));
            const TileCoord c = tile_coord<MODE>(p, f * tiles_per_frame + tx);
            __syncthreads();  // B_f: state(f) staged; CSC(f-1)'s plane reads done
            decode_tile_idct<MODE, TW, THREADS, FLAGS | kGopLdsQt, false>(p, c, state, planes, tid, lds_qt);
            __syncthreads();  // A_f: planes written; the state may take frame f+1
            decode_tile_csc<MODE, TW, THREADS, FLAGS>(p, c, planes, tid);
        }
        return;
    }
    const int lt = threadIdx.x - THREADS;
    const TileCoord cs = tile_coord<MODE>(p, tx);  // frame-0 coordinates (state buffers)
    auto chunk = [&](int k, int l, int& slot, int& col_ok) -> int64_t {  // element offset inside a frame
        slot = SPC * k + (l >> 3);
        const int run = T::slot_run_c(SPC * k);
        const int col = slot - T::run_first_slot(run);
        col_ok = col < cs.run_len(run);
        return cs.run_off(run) + (col_ok ? col : 0) * 64 + (l & 7) * 8;
    };
    auto st_conv = [&](int k, int64_t o) -> int64_t {  // frame-plane offset -> state-buffer offset
        const int run = T::slot_run_c(SPC * k);
        return run < 2 ? o : run == 2 ? o - p.cb_off + p.st_cb_off : o - p.cr_off + p.st_cr_off;
    };
    auto load_frame = [&](uint32_t f, u32x4 (&dst)[LCH]) {
        int l = lt;
        asm volatile("" : "+v"(l));
        const int16_t* fb = p.coef + (int64_t)f * (int64_t)p.plane_fstride;
#pragma unroll
        for (int k = 0; k < LCH; k++) {
            int slot, ok;
            const int64_t o = chunk(k, l, slot, ok);
            dst[k] = load16(reinterpret_cast<const u32x4*>(fb + o), (FLAGS & kNtLoad) != 0);
        }
    };
    // D frames in flight: buffer j holds frame fb + j of the current group of D
    u32x4 v[D][LCH];
    uint32_t ft[D];
    if (f0 < f1 && p.ftype[f0] != 0) {  // the segment continues a GOP: seed the slots from p.state
#pragma unroll
        for (int k = 0; k < LCH; k++) {
            int slot, ok;
            const int64_t o = chunk(k, lt, slot, ok);
            *reinterpret_cast<u32x4*>(state + coef_off(slot, lt & 7)) = *reinterpret_cast<const u32x4*>(p.state + st_conv(k, o));
        }
    }
#pragma unroll
    for (int j = 0; j < D; j++) {
        ft[j] = 0;
        if (f0 + j < f1) {
            ft[j] = p.ftype[f0 + j];
            load_frame(f0 + j, v[j]);
        }
    }
    for (uint32_t fb = f0; fb < f1; fb += D) {
#pragma unroll
        for (int j = 0; j < D; j++) {
            const uint32_t f = fb + j;
            if (f >= f1) break;  // (uniform)
            int l = lt;
            asm volatile("" : "+v"(l));
            // fold v(f) into the state: I replaces, P adds mod 2^16 (each chunk has one owner lane)
            if (__builtin_amdgcn_readfirstlane(ft[j]) != 0) {
#pragma unroll
                for (int k = 0; k < LCH; k++) {
                    const int slot = SPC * k + (l >> 3);
                    const u32x4 o = *reinterpret_cast<const u32x4*>(state + coef_off(slot, l & 7));
                    v[j][k] = (u32x4){add_u16x2(o.x, v[j][k].x), add_u16x2(o.y, v[j][k].y), add_u16x2(o.z, v[j][k].z),
                                      add_u16x2(o.w, v[j][k].w)};
                }
            }
#pragma unroll
            for (int k = 0; k < LCH; k++) *reinterpret_cast<u32x4*>(state + coef_off(SPC * k + (l >> 3), l & 7)) = v[j][k];
            if (f + D < f1) {  // buffer j is free: frame f+D's loads
                ft[j] = p.ftype[f + D];
                load_frame(f + D, v[j]);
            }
            __syncthreads();  // B_f
            __syncthreads();  // A_f
        }
    }
    if (p.state_out && sy + 1 == p.nseg) {  // end state (this lane's own chunks: no barrier needed)
#pragma unroll
        for (int k = 0; k < LCH; k++) {
            int slot, ok;
            const int64_t o = chunk(k, lt, slot, ok);
            if (ok)
                *reinterpret_cast<u32x4*>(p.state_out + st_conv(k, o)) =
                    *reinterpret_cast<const u32x4*>(state + coef_off(slot, lt & 7));
        }
    }
}

// LDS-state stream kernel with the plane tiles overlaying the last OVL staging chunks of the
// state (whose values every lane keeps in OVL * 4 VGPRs instead): LDS = COEF_BYTES +
// PLANE_BYTES - OVL * THREADS * 16 (4:2:0 / 4:4:4: 32 KiB at OVL = 1, five workgroups per CU;
// 24 KiB at OVL = 3, six), dequantization table in SGPRs.  Per frame: fold v(f) into the state
// (LDS chunks < KEEP0, register chunks >= KEEP0), stage every chunk, barrier, IDCT (its own
// barrier between reading the slots and writing the planes), barrier, issue v(f+1), CSC,
// barrier (the next staging overwrites the overlaid planes).
template <int MODE, int TW, int THREADS, int FLAGS, int OVL, int WPE>
__global__ void __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(WPE)))
decode_gop_ovl_kernel(const DecodeParams p) {
    using T = Tile<MODE, TW, THREADS>;
    constexpr int CHB = THREADS * 16;  // LDS bytes of one staging chunk (slots SLOTS_PER_CHUNK*k ..)
    constexpr int KEEP0 = T::CHUNKS - OVL;
    constexpr int POFF = T::COEF_BYTES - OVL * CHB;
    static_assert(OVL >= 1 && KEEP0 >= 0 && T::SLOTS_PER_CHUNK * 128 == CHB, "chunk k = LDS bytes [k*CHB, (k+1)*CHB)");
    constexpr int LDSB = POFF + T::PLANE_BYTES > T::COEF_BYTES ? POFF + T::PLANE_BYTES : T::COEF_BYTES;
    __shared__ __attribute__((aligned(16))) uint8_t lds[LDSB];
    uint8_t* state = lds;
    uint8_t* planes = lds + POFF;
    const int tid0 = threadIdx.x;
    const uint32_t tiles_per_frame = p.tiles_per_frame;
    uint32_t tx, sy;
    if (!gop_job(p, tx, sy)) return;  // (whole workgroup, before any barrier)
    const uint32_t f0 = p.seg_start[sy], f1 = p.seg_start[sy + 1];
    const int wc = __builtin_amdgcn_readfirstlane(T::slot_run(tid0) >= 2 ? 1 : 0);
    uint32_t qs[32];
#pragma unroll
    for (int i = 0; i < 32; i++) qs[i] = __builtin_amdgcn_readfirstlane(p.qt_dev[32 * wc + i]);
    const TileCoord cs = tile_coord<MODE>(p, tx);
    auto st_off = [&](int k, int tid) -> int64_t {
        const int run = T::chunk_run(k);
        const int col = T::SLOTS_PER_CHUNK * k + (tid >> 3) - T::run_first_slot(run);
        const int colc = col < cs.run_len(run) ? col : 0;
        const int64_t o = cs.run_off(run) + colc * 64 + (tid & 7) * 8;
        return run < 2 ? o : run == 2 ? o - p.cb_off + p.st_cb_off : o - p.cr_off + p.st_cr_off;
    };
    u32x4 sr[OVL];
#pragma unroll
    for (int j = 0; j < OVL; j++) sr[j] = (u32x4){0u, 0u, 0u, 0u};
    if (f0 < f1 && p.ftype[f0] != 0) {  // the segment continues a GOP: seed the state from p.state
#pragma unroll
        for (int k = 0; k < T::CHUNKS; k++) {
            const u32x4 x = *reinterpret_cast<const u32x4*>(p.state + st_off(k, tid0));
            if (k < KEEP0)
                *reinterpret_cast<u32x4*>(state + coef_off(T::SLOTS_PER_CHUNK * k + (tid0 >> 3), tid0 & 7)) = x;
            else
                sr[k - KEEP0] = x;
        }
    }
    // kGopPrefetch: frame f+1's loads during CSC(f); otherwise at the top of frame f+1
    constexpr bool PF = (FLAGS & kGopPrefetch) != 0;
    u32x4 v[T::CHUNKS];
    TileCoord c = tile_coord<MODE>(p, f0 * tiles_per_frame + tx);
    uint32_t ft = f0 < f1 ? p.ftype[f0] : 0u;
    if (PF && f0 < f1) stage_load<MODE, TW, THREADS, FLAGS>(p, c, tid0, v);
    for (uint32_t f = f0; f < f1; f++) {
        int tid = tid0;
        asm volatile("" : "+v"(tid));
        if (!PF) {
            c = tile_coord<MODE>(p, f * tiles_per_frame + tx);
            stage_load<MODE, TW, THREADS, FLAGS>(p, c, tid, v);
            ft = p.ftype[f];
        }
        const uint32_t keep = __builtin_amdgcn_readfirstlane(ft) != 0 ? 0xffffffffu : 0u;
#pragma unroll
        for (int k = 0; k < T::CHUNKS; k++) {
            u32x4 o;
            if (k < KEEP0)
                o = keep ? *reinterpret_cast<const u32x4*>(state + coef_off(T::SLOTS_PER_CHUNK * k + (tid >> 3), tid & 7))
                         : (u32x4){0u, 0u, 0u, 0u};
            else
                o = sr[k - KEEP0];
            v[k] = (u32x4){add_u16x2(o.x & keep, v[k].x), add_u16x2(o.y & keep, v[k].y), add_u16x2(o.z & keep, v[k].z),
                           add_u16x2(o.w & keep, v[k].w)};
            if (k >= KEEP0) sr[k - KEEP0] = v[k];
        }
        stage_store<MODE, TW, THREADS, kDefaultFlags>(state, tid, v);
        __syncthreads();
        decode_tile_idct<MODE, TW, THREADS, FLAGS, true>(p, c, state, planes, tid, nullptr, qs);
        __syncthreads();
        TileCoord cn = c;
        if (PF && f + 1 < f1) {
            cn = tile_coord<MODE>(p, (f + 1) * tiles_per_frame + tx);
            stage_load<MODE, TW, THREADS, FLAGS>(p, cn, tid, v);
            ft = p.ftype[f + 1];
        }
        decode_tile_csc<MODE, TW, THREADS, FLAGS>(p, c, planes, tid);
        __syncthreads();  // the planes overlay state chunks >= KEEP0, restaged by the next frame
        c = cn;
    }
    if (p.state_out && sy + 1 == p.nseg) {  // end state, for a batch that continues this GOP
#pragma unroll
        for (int k = 0; k < T::CHUNKS; k++) {
            const int run = T::chunk_run(k);
            const int col = T::SLOTS_PER_CHUNK * k + (tid0 >> 3) - T::run_first_slot(run);
            if (col < cs.run_len(run))
                *reinterpret_cast<u32x4*>(p.state_out + st_off(k, tid0)) =
                    k < KEEP0 ? *reinterpret_cast<const u32x4*>(state + coef_off(T::SLOTS_PER_CHUNK * k + (tid0 >> 3), tid0 & 7))
                              : sr[k - KEEP0];
        }
    }
}

// Pipelined stream kernel: IDCT waves and CSC waves of one workgroup work on consecutive
// frames at the same time.  Waves 0-2 (192 lanes, one per block: 4:2:0 / 4:4:4 tiles) run the
// IDCT of frame k from the LDS state into plane buffer k % 2 while waves 3-6 (256 lanes) run
// the CSC of frame k-1 from buffer (k-1) % 2, fold the prefetched deltas of frame k+1 into the
// state (I: replace, P: add mod 2^16, lossless_decode.c:90-92,121-122 in the quantized domain)
// and issue frame k+2's loads.  Phase k: IDCT waves: read blocks(k)  M_k  IDCT -> planes  B_k+1;
// CSC waves: M_k  CSC(k-1)  fold v(k+1)  load v(k+2)  B_k+1.  The fold follows M_k (every
// block of frame k is in registers) and precedes B_k+1; planes are double-buffered.
// LDS 24 + 2 x 12 KiB: three 7-wave workgroups per CU; stores issue throughout every phase.
template <int MODE, int TW, int FLAGS, int WPE>
__global__ void __launch_bounds__(448) __attribute__((amdgpu_waves_per_eu(WPE)))
decode_gop_pipe_kernel(const DecodeParams p) {
    using T = Tile<MODE, TW, 256>;  // CSC / staging layout of the 256 CSC lanes
    static_assert(T::NSLOT == 192, "three IDCT waves");
    constexpr int IL = 192;
    __shared__ __attribute__((aligned(16))) uint8_t lds[T::COEF_BYTES + 2 * T::PLANE_BYTES];
    uint8_t* state = lds;
    const uint32_t tiles_per_frame = p.tiles_per_frame;
    uint32_t tx, sy;
    if (!gop_job(p, tx, sy)) return;  // (whole workgroup, before any barrier)
    const uint32_t f0 = p.seg_start[sy], f1 = p.seg_start[sy + 1];
    if (__builtin_amdgcn_readfirstlane((int)threadIdx.x) < IL) {  // ---- IDCT waves
        const int tid0 = threadIdx.x;
        const int wc = __builtin_amdgcn_readfirstlane(T::slot_run(tid0) >= 2 ? 1 : 0);
        uint32_t qs[32];
#pragma unroll
        for (int i = 0; i < 32; i++) qs[i] = __builtin_amdgcn_readfirstlane(p.qt_dev[32 * wc + i]);
        __syncthreads();  // B_f0: the state holds frame f0
        for (uint32_t k = f0; k <= f1; k++) {
            int tid = tid0;
            asm volatile("" : "+v"(tid));
            if (k < f1) {  // M_k inside (after the blocks are read)
                const TileCoord c = tile_coord<MODE>(p, k * tiles_per_frame + tx);
                decode_tile_idct<MODE, TW, 256, FLAGS, true>(p, c, state, lds + T::COEF_BYTES + (k & 1) * T::PLANE_BYTES, tid,
                                                             nullptr, qs);
            } else {
                __syncthreads();  // M_f1
            }
            __syncthreads();  // B_k+1
        }
        return;
    }
    // ---- CSC waves (lane t of 256): CSC, deltas in flight, fold
    const int t0 = threadIdx.x - IL;
    const TileCoord cs = tile_coord<MODE>(p, tx);
    auto st_off = [&](int k, int t) -> int64_t {
        const int run = T::chunk_run(k);
        const int col = T::SLOTS_PER_CHUNK * k + (t >> 3) - T::run_first_slot(run);
        const int colc = col < cs.run_len(run) ? col : 0;
        const int64_t o = cs.run_off(run) + colc * 64 + (t & 7) * 8;
        return run < 2 ? o : run == 2 ? o - p.cb_off + p.st_cb_off : o - p.cr_off + p.st_cr_off;
    };
    u32x4 v[T::CHUNKS];
    auto fold = [&](int t, uint32_t ft) {  // v -> state (this lane's chunks)
        const uint32_t keep = __builtin_amdgcn_readfirstlane(ft) != 0 ? 0xffffffffu : 0u;
#pragma unroll
        for (int k = 0; k < T::CHUNKS; k++) {
            u32x4* sp = reinterpret_cast<u32x4*>(state + coef_off(T::SLOTS_PER_CHUNK * k + (t >> 3), t & 7));
            const u32x4 o = keep ? *sp : (u32x4){0u, 0u, 0u, 0u};
            *sp = (u32x4){add_u16x2(o.x, v[k].x), add_u16x2(o.y, v[k].y), add_u16x2(o.z, v[k].z), add_u16x2(o.w, v[k].w)};
        }
    };
    if (f0 < f1) {
        if (p.ftype[f0] != 0) {  // the segment continues a GOP: seed the slots from p.state
#pragma unroll
            for (int k = 0; k < T::CHUNKS; k++)
                *reinterpret_cast<u32x4*>(state + coef_off(T::SLOTS_PER_CHUNK * k + (t0 >> 3), t0 & 7)) =
                    *reinterpret_cast<const u32x4*>(p.state + st_off(k, t0));
        }
        stage_load<MODE, TW, 256, FLAGS>(p, tile_coord<MODE>(p, f0 * tiles_per_frame + tx), t0, v);
        fold(t0, p.ftype[f0]);
    }
    uint32_t ft = 0;
    if (f0 + 1 < f1) {
        stage_load<MODE, TW, 256, FLAGS>(p, tile_coord<MODE>(p, (f0 + 1) * tiles_per_frame + tx), t0, v);
        ft = p.ftype[f0 + 1];
    }
    __syncthreads();  // B_f0
    for (uint32_t k = f0; k <= f1; k++) {
        int t = t0;
        asm volatile("" : "+v"(t));
        __syncthreads();  // M_k: the IDCT waves hold frame k's blocks in registers
        if (k > f0)
            decode_tile_csc<MODE, TW, 256, FLAGS>(p, tile_coord<MODE>(p, (k - 1) * tiles_per_frame + tx),
                                                  lds + T::COEF_BYTES + ((k - 1) & 1) * T::PLANE_BYTES, t);
        if (k + 1 < f1) {
            fold(t, ft);
            if (k + 2 < f1) {
                stage_load<MODE, TW, 256, FLAGS>(p, tile_coord<MODE>(p, (k + 2) * tiles_per_frame + tx), t, v);
                ft = p.ftype[k + 2];
            }
        }
        __syncthreads();  // B_k+1
    }
    if (p.state_out && sy + 1 == p.nseg) {  // end state (this lane's own chunks, unchanged since its last fold)
#pragma unroll
        for (int k = 0; k < T::CHUNKS; k++) {
            const int run = T::chunk_run(k);
            const int col = T::SLOTS_PER_CHUNK * k + (t0 >> 3) - T::run_first_slot(run);
            if (col < cs.run_len(run))
                *reinterpret_cast<u32x4*>(p.state_out + st_off(k, t0)) =
                    *reinterpret_cast<const u32x4*>(state + coef_off(T::SLOTS_PER_CHUNK * k + (t0 >> 3), t0 & 7));
        }
    }
}

// Global-state stream kernel (probe only): the batch kernel's 24 KiB LDS footprint (coefficient
// slots aliased with the plane tiles) so six 4-wave workgroups fit per CU, with the tile's
// accumulated coefficients kept in a per-(segment, tile) record in global memory instead of
// LDS: each frame's deltas (HBM) are added to the record (written by the same lane one frame
// earlier: reuse distance ~one frame of the whole GPU's traffic, inside the 256 MiB Infinity
// Cache) and written back unless it is the segment's last frame.  p.state_out = the records,
// CHUNKS x THREADS x 16 B each, lane-interleaved so a wave moves 1 KiB contiguous.
template <int MODE, int TW, int THREADS, int FLAGS, int WPE>
__global__ void __launch_bounds__(THREADS) __attribute__((amdgpu_waves_per_eu(WPE)))
decode_gop_gs_kernel(const DecodeParams p) {
    using T = Tile<MODE, TW, THREADS>;
    __shared__ __attribute__((aligned(16))) uint8_t lds[T::LDS_BYTES];
    const int tid0 = threadIdx.x;
    const uint32_t tx = blockIdx.x, sy = blockIdx.y;
    const uint32_t f0 = p.seg_start[sy], f1 = p.seg_start[sy + 1];
    u32x4* rec = reinterpret_cast<u32x4*>(p.state_out) + (size_t)(sy * p.tiles_per_frame + tx) * T::CHUNKS * THREADS;
    for (uint32_t f = f0; f < f1; f++) {
        int tid = tid0;
        asm volatile("" : "+v"(tid));
        const TileCoord c = tile_coord<MODE>(p, f * p.tiles_per_frame + tx);
        u32x4 v[T::CHUNKS];
        stage_load<MODE, TW, THREADS, FLAGS>(p, c, tid, v);
        if (__builtin_amdgcn_readfirstlane(p.ftype[f]) != 0) {
#pragma unroll
            for (int k = 0; k < T::CHUNKS; k++) {
                const u32x4 o = rec[k * THREADS + tid], d = v[k];
                v[k] = (u32x4){add_u16x2(o.x, d.x), add_u16x2(o.y, d.y), add_u16x2(o.z, d.z), add_u16x2(o.w, d.w)};
            }
        }
        if (f + 1 < f1) {
#pragma unroll
            for (int k = 0; k < T::CHUNKS; k++) rec[k * THREADS + tid] = v[k];
        }
        stage_store<MODE, TW, THREADS, FLAGS>(lds, tid, v);
        __syncthreads();
        decode_tile<MODE, TW, THREADS, FLAGS>(p, c, lds, tid);
        __syncthreads();  // the CSC's plane reads finish before the next frame's staging
    }
}

// Compact block records (probe only): per 8x8 block 64 B = 16 words: word 0 = the count n of
// nonzero coefficients (<= 15), or 0xffff when there are more (the block is then read from the
// dense plane); words 1..n = natural index << 16 | uint16 value.  Same order as the dense planes:
// the block at int16 element X (a multiple of 64) has words [X / 4, X / 4 + 16).
__global__ void __launch_bounds__(256) make_records_kernel(const int16_t* coef, uint32_t* rec, uint64_t nblocks,
                                                           unsigned long long* dense_blocks) {
    const uint64_t b = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (b >= nblocks) return;
    const int16_t* c = coef + b * 64;
    uint32_t* w = rec + b * 16;
    uint32_t n = 0;
    for (int i = 0; i < 64; i++) {
        const int16_t v = c[i];
        if (v != 0) {
            if (n < 15) w[1 + n] = ((uint32_t)i << 16) | (uint16_t)v;
            n++;
        }
    }
    for (uint32_t i = n; i < 15; i++) w[1 + i] = 0u;
    w[0] = n > 15 ? 0xffffu : n;
    if (n > 15) atomicAdd(dense_blocks, 1ull);
}

// The stream kernel reading compact records instead of dense planes (probe only; records passed in
// p.state).  One lane per block slot stages its block: an I-frame clears the slot and writes the
// entries, a P-frame adds them (mod 2^16); a dense-marked block is read whole from p.coef.  The
// next frame's record (64 B, 16 VGPRs) is loaded right after the staging barrier (kGopEarly-like).
template <int MODE, int TW, int THREADS, int FLAGS>
__global__ void __launch_bounds__(THREADS) decode_gop_rec_kernel(const DecodeParams p) {
    using T = Tile<MODE, TW, THREADS>;
    __shared__ __attribute__((aligned(16))) uint8_t lds[T::COEF_BYTES + T::PLANE_BYTES + 256];
    uint8_t* state = lds;
    uint8_t* planes = lds + T::COEF_BYTES;
    uint32_t* lds_qt = reinterpret_cast<uint32_t*>(lds + T::COEF_BYTES + T::PLANE_BYTES);
    const uint32_t* rec = reinterpret_cast<const uint32_t*>(p.state);
    const int tid0 = threadIdx.x;
    if (tid0 < 16) reinterpret_cast<uint4*>(lds_qt)[tid0] = reinterpret_cast<const uint4*>(p.qt_dev)[tid0];
    const uint32_t tx = blockIdx.x, sy = blockIdx.y;
    const uint32_t f0 = p.seg_start[sy], f1 = p.seg_start[sy + 1];
    const int s = tid0;
    const int run = T::slot_run(s < T::NSLOT ? s : 0);
    const int col = s - (run == 0 ? T::run_first_slot(0) : run == 1 ? T::run_first_slot(1)
                         : run == 2 ? T::run_first_slot(2) : T::run_first_slot(3));
    auto blk_off = [&](const TileCoord& c) -> int64_t {  // int16 element of this lane's block
        const int colc = col < c.run_len(run) ? col : 0;
        return (run == 0 ? c.off0 : run == 1 ? c.off1 : run == 2 ? c.off2 : c.off3) + (int64_t)colc * 64;
    };
    u32x4 r[4];
    TileCoord c = tile_coord<MODE>(p, f0 * p.tiles_per_frame + tx);
    if (s < T::NSLOT) {
        const u32x4* rp = reinterpret_cast<const u32x4*>(rec + blk_off(c) / 4);
#pragma unroll
        for (int k = 0; k < 4; k++) r[k] = __builtin_nontemporal_load(rp + k);
    }
    for (uint32_t f = f0; f < f1; f++) {
        int tid = tid0;
        asm volatile("" : "+v"(tid));
        const uint32_t ft = __builtin_amdgcn_readfirstlane(p.ftype[f]);
        const bool active = s < T::NSLOT && col < c.run_len(run);
        if (active) {
            const uint32_t n = r[0].x & 0xffffu;
            if (n == 0xffffu) {  // dense block
                const u32x4* dp = reinterpret_cast<const u32x4*>(p.coef + blk_off(c));
#pragma unroll
                for (int row = 0; row < 8; row++) {
                    u32x4 d = __builtin_nontemporal_load(dp + row);
                    u32x4* sp = reinterpret_cast<u32x4*>(state + coef_off(s, row));
                    if (ft != 0) {
                        const u32x4 o = *sp;
                        d = (u32x4){add_u16x2(o.x, d.x), add_u16x2(o.y, d.y), add_u16x2(o.z, d.z), add_u16x2(o.w, d.w)};
                    }
                    *sp = d;
                }
            } else {
                if (ft == 0) {
#pragma unroll
                    for (int row = 0; row < 8; row++) *reinterpret_cast<u32x4*>(state + coef_off(s, row)) = (u32x4){0u, 0u, 0u, 0u};
                }
                const uint32_t wv[15] = {r[0].y, r[0].z, r[0].w, r[1].x, r[1].y, r[1].z, r[1].w, r[2].x,
                                         r[2].y, r[2].z, r[2].w, r[3].x, r[3].y, r[3].z, r[3].w};
#pragma unroll
                for (int i = 0; i < 15; i++) {
                    if ((uint32_t)i < n) {
                        const uint32_t e = wv[i], ni = e >> 16;
                        uint16_t* a = reinterpret_cast<uint16_t*>(state + coef_off(s, (int)(ni >> 3)) + 2 * (ni & 7));
                        *a = (uint16_t)(ft != 0 ? (uint32_t)*a + e : e);
                    }
                }
            }
        }
        __syncthreads();
        TileCoord cn = c;
        if (f + 1 < f1) {
            cn = tile_coord<MODE>(p, (f + 1) * p.tiles_per_frame + tx);
            if (s < T::NSLOT) {
                const u32x4* rp = reinterpret_cast<const u32x4*>(rec + blk_off(cn) / 4);
#pragma unroll
                for (int k = 0; k < 4; k++) r[k] = __builtin_nontemporal_load(rp + k);
            }
        }
        decode_tile_idct<MODE, TW, THREADS, FLAGS, false>(p, c, state, planes, tid, lds_qt);
        __syncthreads();
        decode_tile_csc<MODE, TW, THREADS, FLAGS>(p, c, planes, tid);
        c = cn;
    }
}

// One-shot chain stream kernel (probe only, round 3): one workgroup per (tile, frame) like the batch
// kernel (its 24 KiB of LDS: six per CU), the accumulated coefficients handed from the workgroup of
// frame k to the one of frame k + 1 through a per-(segment, tile) record in global memory.  Jobs are
// ordered so that a chain stays on one XCD (workgroup b runs on XCD b % 8) and its hand-off is
// L2-local: XCD x takes units (segment, band of B tiles) x, x + 8, ...; inside a unit, frame-major,
// so frame k + 1 of a tile is dispatched B workgroups of its XCD after frame k.  Hand-off: plain
// record stores, every wave's vmcnt(0), a barrier, one lane's relaxed agent-scope flag store; the
// consumer's lane 0 polls the flag (L1-bypassing sc1 loads), a barrier, then sc1 record loads.
// Segments of exactly L frames starting with an I-frame (the probe's GOP setup).
template <int MODE, int TW, int THREADS, int FLAGS>
__global__ void __launch_bounds__(THREADS, 6) decode_chain_kernel(const DecodeParams p, u32x4* rec, uint32_t* flags,
                                                                  uint32_t B, uint32_t L, uint32_t nb, uint32_t U) {
    using T = Tile<MODE, TW, THREADS>;
    __shared__ __attribute__((aligned(16))) uint8_t lds[T::LDS_BYTES];
    const int tid = threadIdx.x;
    const uint32_t x = blockIdx.x % 8, j = blockIdx.x / 8, per = L * B;
    const uint32_t u = x + 8 * (j / per);
    if (u >= U) return;
    const uint32_t r = j % per, k = r / B, s = u / nb, beta = u % nb, t = beta * B + r % B;
    if (t >= p.tiles_per_frame) return;
    const uint32_t f = s * L + k;
    const TileCoord c = tile_coord<MODE>(p, f * p.tiles_per_frame + t);
    u32x4 v[T::CHUNKS];
    stage_load<MODE, TW, THREADS, FLAGS>(p, c, tid, v);
    const size_t chain = (size_t)s * p.tiles_per_frame + t;
    u32x4* my = rec + chain * T::CHUNKS * THREADS;
    if (k > 0) {  // P-frame: frame k - 1's record, then its deltas added mod 2^16
        if (tid == 0) {  // bounded: a hand-off that never arrives gives wrong pixels (the probe compares), not a hang
            for (uint32_t n = 0; n < (1u << 22); n++) {
                if (__hip_atomic_load(flags + chain, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= k) break;
                __builtin_amdgcn_s_sleep(1);
            }
        }
        __syncthreads();
        u32x4 o[T::CHUNKS];
#pragma unroll
        for (int q = 0; q < T::CHUNKS; q++)
            asm volatile("global_load_dwordx4 %0, %1, off sc1" : "=v"(o[q]) : "v"(my + q * THREADS + tid) : "memory");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
        for (int q = 0; q < T::CHUNKS; q++)
            v[q] = (u32x4){add_u16x2(o[q].x, v[q].x), add_u16x2(o[q].y, v[q].y), add_u16x2(o[q].z, v[q].z), add_u16x2(o[q].w, v[q].w)};
    }
    if (k + 1 < L) {  // hand the state to frame k + 1
#pragma unroll
        for (int q = 0; q < T::CHUNKS; q++) my[q * THREADS + tid] = v[q];
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) __hip_atomic_store(flags + chain, k + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    stage_store<MODE, TW, THREADS, FLAGS>(lds, tid, v);
    __syncthreads();
    decode_tile<MODE, TW, THREADS, FLAGS>(p, c, lds, tid);
}

// Round 3 diagnostic (PROBE_ORDERS): the one-shot batch kernel's body under workgroup orders that
// mimic where the stream kernel's resident workgroups are in the frames, to split the stream
// kernel's gap to the batch kernel into "loop" and "order".  Workgroup b runs on XCD x = b % 8,
// i = b / 8; T tiles per frame, E = ceil(T / 8), NF frames:
//   order 2 (bands): XCD x takes the x-th eighth of every frame's tiles, frame after frame (the
//     stream kernel's eighths order with every XCD in the same frame);
//   order 3 (frames per XCD): XCD x takes whole frames x, x + 8, ... (eight frames in flight);
//   order 4 (band walks): XCD x takes the x-th eighth of the tiles, in groups of G tiles that walk
//     frames 0 .. NF-1 before the next group (the stream kernel's tile x walking its segment's
//     frames, G = the XCD's resident workgroups);
//   order 5 (distant band walks): XCD x takes the x-th contiguous eighth of the frames, and in it
//     groups of G tiles (of the whole frame) walk its frames (the stream kernel in XCD-contiguous
//     job order: eight XCDs in eight distant parts of the batch, each holding tiles across frames).
template <int MODE, int TW, int THREADS, int FLAGS>
__global__ void __launch_bounds__(THREADS, (lds_waves(kBatchLds<MODE, TW, THREADS, FLAGS>, THREADS)))
    decode_order_kernel(const DecodeParams p, uint32_t order, uint32_t nf, uint32_t G) {
    using T = Tile<MODE, TW, THREADS>;
    __shared__ __attribute__((aligned(16))) uint8_t lds[kBatchLds<MODE, TW, THREADS, FLAGS>];
    const int tid = threadIdx.x;
    const uint32_t Tf = p.tiles_per_frame, E = (Tf + 7) / 8, x = blockIdx.x % 8, i = blockIdx.x / 8;
    uint32_t f, t;
    if (order == 2) {
        f = i / E;
        t = x * E + i % E;
    } else if (order == 3) {
        f = 8 * (i / Tf) + x;
        t = i % Tf;
    } else if (order == 4) {
        const uint32_t gi = i / (G * nf), r = i % (G * nf);
        f = r / G;
        t = x * E + gi * G + r % G;
        if (gi * G + r % G >= E) return;
    } else {  // 5: XCD x takes the x-th contiguous eighth of the frames; in it, groups of G tiles walk its frames
        const uint32_t nfx = (nf + 7) / 8, gi = i / (G * nfx), r = i % (G * nfx);
        f = x * nfx + r / G;
        t = gi * G + r % G;
        if (r / G >= nfx) return;
    }
    if (f >= nf || t >= Tf) return;
    const TileCoord c = tile_coord<MODE>(p, f * Tf + t);
    u32x4 v[T::CHUNKS];
    stage_load<MODE, TW, THREADS, FLAGS>(p, c, tid, v);
    stage_store<MODE, TW, THREADS, FLAGS>(lds, tid, v);
    __syncthreads();
    decode_tile_idct<MODE, TW, THREADS, FLAGS, true>(p, c, lds, lds, tid);
    __syncthreads();
    decode_tile_csc<MODE, TW, THREADS, FLAGS>(p, c, lds, tid);
}

}  // namespace mj423
