#!/usr/bin/env python3
"""Benchmark: fused dequant + 8x8 IDCT + YCbCr->BGRA on MI355X (BASELINE.json metric).

One step = one fused-decode launch over this rank's whole batch of synthetic
frames (default: BASELINE configs[2]/[3], 3840x2160 4:2:0, 300 frames per GPU),
coefficients already resident in HBM.  Frames are sharded across ranks (weak
scaling: 300 frames per GPU); the only collective is the RCCL broadcast of the
256-byte quantization tables at start-up plus the timing reductions.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c2|c5|c1]
    torchrun --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line (see the contract in the task description).
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "mjpeg423-video-decoder-software_amd")
ORACLE = os.path.join(REPO, "oracle")
PROFILES = os.path.join(REPO, "profiles")
for p in (PKG, ORACLE):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402


WARMUP_AUTO_S = 0.25


def warm_up(step, n, sync):
    """Untimed warm-up: exactly n steps if n >= 0, else steps until WARMUP_AUTO_S seconds of
    them have run (at least 3).  Returns the number of steps run."""
    if n >= 0:
        for _ in range(n):
            step()
        sync()
        return n
    done, t0 = 0, time.perf_counter()
    while done < 3 or time.perf_counter() - t0 < WARMUP_AUTO_S:
        step()
        done += 1
        if done % 4 == 0:
            sync()  # bound the queue so the wall clock tracks the GPU
    sync()
    return done


def _launch_ranks_if_needed(argv):
    """`--gpus N` must mean N ranks.  Under a torch.distributed launcher WORLD_SIZE has to
    equal N (else exit 2).  Run bare with N > 1, this parent -- which has imported neither
    torch nor the HIP library, so it made no GPU call -- starts N ranks (one per GPU) as a
    child `torch.distributed.run` on 127.0.0.1 and exits with the child's status."""
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    n = ap.parse_known_args(argv)[0].gpus
    if n < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    ws = os.environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != n:
            raise SystemExit(f"bench.py: --gpus {n} but WORLD_SIZE={ws}: refusing to report a "
                             f"{ws}-rank run as {n} GPUs")
        return
    if n == 1:
        return
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + list(argv)
    print(f"bench.py: launching {n} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    raise SystemExit(subprocess.call(cmd))


if __name__ == "__main__":
    _launch_ranks_if_needed(sys.argv[1:])

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import mj423  # noqa: E402
import shard  # noqa: E402

CONFIGS = {
    # name: (w, h, chroma, frames per GPU, BASELINE.json configs index)
    "c1": (640, 480, 444, 300, 0),
    "c2": (1920, 1080, 420, 300, 1),
    "c3": (3840, 2160, 420, 300, 2),
    "c5": (7680, 4320, 422, 15, 4),
    # --mode file only (the .mpg format is 4:4:4): a 1080p stream through the whole decoder
    "f2": (1920, 1080, 444, 240, None),
}
HBM_PEAK_GBPS = 8000.0  # MI355X spec (MI355X_MICROARCH.md, chip-level parameters)
SEED = 0x4D4A3432


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=-1,
                    help="untimed warm-up steps (default: as many as fill %.2f s, at least 3 -- short launches "
                         "read up to 15 %% low until the GPU's clocks have ramped under sustained load, "
                         "DESIGN §6); an explicit value is used exactly" % WARMUP_AUTO_S)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--frames", type=int, default=0, help="frames per GPU (default: the config's)")
    ap.add_argument("--total-frames", type=int, default=0,
                    help="strong scaling: this many frames in total, split into contiguous per-rank ranges "
                         "(SURVEY §8(d) C4: 2400 4K frames at N = 1, 2, 4, 8); default: weak scaling")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget for the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--verify", default="all", choices=["all", "ends"],
                    help="frames checked against the oracle after timing: all of every rank's, or first+last")
    ap.add_argument("--mode", default="batch", choices=["batch", "stream", "file"],
                    help="batch: every frame absolute (decode_kernel); stream: I/P GOPs with P-frame "
                         "deltas accumulated on chip (decode_gop_kernel, SURVEY §8(f) row 3); file: a "
                         "synthetic 4:4:4 .mpg through the whole streaming decoder (front end on host "
                         "threads + PCIe + GPU; never the headline number)")
    ap.add_argument("--threads", type=int, default=16, help="file mode: front-end host threads")
    ap.add_argument("--chunk", type=int, default=0, help="file mode: frames per pipeline chunk (0: the library's default)")
    ap.add_argument("--sink", default="host", choices=["host", "device"],
                    help="file mode: frames downloaded to host memory, or left in HBM (decode-to-device)")
    ap.add_argument("--frontend", default="host", choices=["host", "gpu"],
                    help="file mode: entropy decode on host threads (pipeline) or on the GPU "
                         "(mj423_mpg_decode_gpu, one wave per bitstream; frames left in HBM)")
    ap.add_argument("--frame0", type=int, default=-1,
                    help="global index of this rank's first frame (default rank*frames); lets one GPU rehearse "
                         "what a later rank of a multi-GPU run decodes (e.g. a stream range starting mid-GOP)")
    ap.add_argument("--gop", type=int, default=24, help="stream mode: I-frame interval (mj/sample_main.c:30)")
    ap.add_argument("--mpg", default="", help="file mode: decode this .mpg (e.g. tools/real_mpg.py's reference-encoded "
                                              "files) instead of a synthetic one; its header gives the size")
    return ap.parse_args()


def pmc_traffic(workload_key, sources=None):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/pmc_traffic.json,
    written by tools/pmc_summary.py), with where they came from.  Returns (bytes or None, source):
    the bytes only while the entry's kernel-source digest equals this tree's -- an entry measured on
    other kernel sources is reported as stale and its bytes are not used."""
    path = os.path.join(PROFILES, "pmc_traffic.json")
    try:
        with open(path) as f:
            e = json.load(f).get(workload_key)
    except (OSError, ValueError):
        e = None
    if not e:
        return None, {"status": "absent", "file": "profiles/pmc_traffic.json", "key": workload_key}
    now = mj423.kernel_source_digest(sources or mj423.KERNEL_SOURCES)
    src = {"file": "profiles/pmc_traffic.json", "key": workload_key, "kernel_src_digest": e.get("kernel_src_digest"),
           "tree_kernel_src_digest": now, "git_commit": e.get("git_commit"), "date": e.get("date"),
           "traffic_over_algorithmic": e.get("traffic_over_algorithmic")}
    if now is None or e.get("kernel_src_digest") != now:
        src["status"] = ("unknown: this tree's kernel sources are absent" if now is None
                         else "stale: measured on other kernel sources")
        return None, src
    src["status"] = "current"
    return e.get("hbm_bytes_per_launch"), src


def copy_context(src, dst, reps=10):
    """SURVEY §8(d)'s context figure: a plain device-to-device copy of the coefficient buffer into
    the output buffer (every byte read once and written once) in the same process and on the same
    buffers as the timed launches, so the same HBM placement -- what a memory-bound kernel with no
    arithmetic reaches here.  Run after every use of `dst` (it is overwritten)."""
    n = min(src.numel() * src.element_size(), dst.numel() * dst.element_size())
    s = src.view(torch.uint8)[:n]
    d = dst.view(torch.uint8)[:n]
    for _ in range(3):
        d.copy_(s)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        d.copy_(s)
    e1.record()
    e1.synchronize()
    ms = e0.elapsed_time(e1) / reps
    moved = 2 * s.numel()
    gbps = moved / (ms * 1e-3) / 1e9
    return {"achieved": round(gbps, 1), "unit": "GB/s", "frac": round(gbps / HBM_PEAK_GBPS, 4), "ms": round(ms, 4),
            "bytes_moved": moved, "method": "torch Tensor.copy_ device-to-device, coefficient buffer -> output buffer (the smaller's bytes), "
                                            "%d repetitions after the parity check" % reps}


def stream_kernel_label(chroma):
    """The stream-decode kernels one launch runs (mj423_launch_decode_gop's selection)."""
    if chroma == 422 and os.environ.get("MJ423_GOP_OPT", "1") != "0":
        return "decode_gop_kernel<422> (optimistic) + exact re-run pass, one event pair"
    return "decode_gop_kernel<%d>" % chroma


def init_dist(world, local, want):
    """One process per GPU over RCCL.  MJ423_BENCH_BACKEND=gloo rehearses the multi-rank
    logic on a box with fewer GPUs (ranks share cuda:local % count; collectives on the
    host) -- a test aid, never how the driver runs, and the JSON says so.  Returns
    (device, collective device, {"backend", "world_size", "rehearsal"}) after checking that
    the process group really has `want` ranks."""
    backend = os.environ.get("MJ423_BENCH_BACKEND", "nccl")
    if world != want:
        raise SystemExit(f"bench.py: WORLD_SIZE={world} but --gpus {want}")
    if backend == "nccl" and world > torch.cuda.device_count():
        raise SystemExit(f"bench.py: {world} ranks but only {torch.cuda.device_count()} visible GPU(s)")
    idx = local if backend == "nccl" else local % max(1, torch.cuda.device_count())
    dev = torch.device("cuda", idx)
    torch.cuda.set_device(dev)
    info = {"backend": None, "world_size": 1, "rehearsal": backend != "nccl"}
    # MJ423_BENCH_FORCE_DIST=1: a process group even for one rank (under a launcher), so a
    # one-GPU box runs the RCCL start-up, broadcast and reductions of the multi-GPU path
    if world > 1 or os.environ.get("MJ423_BENCH_FORCE_DIST") == "1":
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)
        info["backend"] = dist.get_backend()
        info["world_size"] = dist.get_world_size()
        if info["world_size"] != want:
            raise SystemExit(f"bench.py: process group has {info['world_size']} ranks, --gpus {want}")
        if backend == "nccl" and info["backend"] != "nccl":
            raise SystemExit(f"bench.py: expected the nccl (RCCL) backend, got {info['backend']}")
    return dev, (dev if backend == "nccl" else None), info


def main():
    a = parse()
    if a.mode == "file":
        return main_file(a)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev, coll_dev, dinfo = init_dist(world, local, a.gpus)

    w, h, chroma, frames_cfg, cfg_idx = CONFIGS[a.config]
    nfr = a.frames or frames_cfg
    if a.total_frames:  # strong scaling: contiguous ranges of the fixed total (sizes differ by <= 1)
        if a.total_frames < world:
            raise SystemExit("--total-frames must be >= the number of ranks")
        t_first, t_stop = shard.frame_range(rank, world, a.total_frames)
        nfr = t_stop - t_first
    g = mj423.geometry(w, h, chroma)

    ctx = mj423.Context(dev.index)
    # A dedicated (non-null) stream shared by torch and the library: the kernel
    # launches and the timing events below are on the same stream.
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)

    # Quantization tables: rank 0's tables reach every GPU over RCCL (xGMI); 256 B.
    yq, cq = ctx.get_quant()
    ctx.set_quant(*shard.broadcast_quant_tables(yq, cq, device=coll_dev))

    # This rank's shard (weak scaling): global frames [rank*nfr, (rank+1)*nfr), generated on-device.
    first, _ = shard.weak_range(rank, nfr)
    if a.total_frames:
        first = t_first
    if a.frame0 >= 0:
        first = a.frame0 + rank * nfr
    coef = torch.empty(nfr * g.coef_per_frame, dtype=torch.int16, device=dev)
    out = torch.empty(nfr * w * h, dtype=torch.int32, device=dev)
    ctx.synth_frames_device(coef.data_ptr(), w, h, chroma, nfr, first, SEED)
    torch.cuda.synchronize(dev)

    if a.mode == "stream":
        # Global frame g is an I-frame iff g % gop == 0; P-frames carry A[g] - A[g-1] (mod 2^16),
        # so the decoded pixels equal the batch decode of the absolute frames A.  A rank whose
        # range starts inside a GOP gets the absolute coefficients of frame first-1 as state_in.
        types = np.array([0 if (first + i) % a.gop == 0 else 1 for i in range(nfr)], np.uint8)
        cv = coef.view(nfr, -1)
        stream_in = cv.clone()
        # deltas in chunks of frames: masked indexing over the whole batch would hold several
        # batch-sized temporaries (2400 4K frames, SURVEY §8(d) C4 on one GPU: 53 GiB each)
        pmask = torch.from_numpy(types.astype(bool)).to(dev)
        for s in range(1, nfr, 64):
            e = min(nfr, s + 64)
            stream_in[s:e] = torch.where(pmask[s:e, None], cv[s:e] - cv[s - 1:e - 1], cv[s:e])
        state_in = None
        if types[0] == 1:
            state_in = torch.empty(g.coef_per_frame, dtype=torch.int16, device=dev)
            ctx.synth_frames_device(state_in.data_ptr(), w, h, chroma, 1, first - 1, SEED)
            stream_in[0] = cv[0] - state_in
        del pmask
        torch.cuda.synchronize(dev)

        def step():
            ctx.decode_stream_device(stream_in.data_ptr(), out.data_ptr(), nfr, w, h, chroma, types,
                                     state_in.data_ptr() if state_in is not None else 0)
    else:
        def step():
            ctx.decode_batch_device(coef.data_ptr(), out.data_ptr(), nfr, w, h, chroma)

    a.warmup = warm_up(step, a.warmup, lambda: torch.cuda.synchronize(dev))

    starts = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        starts[i].record(stream)
        step()
        ends[i].record(stream)
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = [s.elapsed_time(e) for s, e in zip(starts, ends)]
    elapsed_max, kern_ms_max, kern_med_max = shard.max_over_ranks(
        [elapsed, float(np.mean(kern_ms)), float(np.median(kern_ms))], device=coll_dev)
    per_rank = shard.gather_over_ranks([elapsed * 1e3 / a.steps, float(np.mean(kern_ms)), float(nfr)],
                                       device=coll_dev)

    # Parity of the timed output against the oracle, after timing: every frame of this
    # rank (--verify all, in chunks) or its first and last (--verify ends).
    verified, checked = None, 0
    if not a.no_verify:
        frames = list(range(nfr)) if a.verify == "all" else sorted({0, nfr - 1})
        bad, checked = cpu_leg_check_frames(coef, out, nfr, w, h, chroma, frames)
        bad_all, checked_all = shard.sum_over_ranks([float(bad), float(checked)], device=coll_dev)
        verified = bad_all == 0.0
        checked = int(checked_all)

    cpu = rank0_cpu_baseline(rank, coef, out, nfr, w, h, chroma, g, a.cpu_seconds, skip=a.no_cpu)
    copy_ctx = copy_context(coef, out) if rank == 0 else None  # (after every use of `out`)

    if rank == 0:
        frames_all = a.total_frames if a.total_frames else world * nfr
        total_px = float(frames_all) * w * h * a.steps
        value = total_px / elapsed_max / 1e6
        fbytes = mj423.frame_bytes(w, h, chroma)
        launch_bytes = fbytes * nfr
        achieved = launch_bytes / (kern_ms_max / 1e3) / 1e9
        key = f"{w}x{h}_{chroma}_{nfr}f" + ("_stream" if a.mode == "stream" else "")
        traffic, traffic_src = pmc_traffic(key)
        res = {
            "metric": "Mpixels/s decoded (dequant+IDCT+CSC) at 1/2/4/8 GPUs; % HBM roofline",
            "value": round(value, 1),
            "unit": "Mpix/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed_max * 1e3 / a.steps, 4),
            "higher_is_better": True,
            "scaling": "strong" if a.total_frames else "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic: device-generated seeded quantized-coefficient stream (SURVEY §8(d)), resident in HBM"
                    + (f"; stream mode: I every {a.gop} frames, P-frames as deltas" if a.mode == "stream" else ""),
            "config": {"workload": f"{w}x{h} {chroma // 100}:{chroma // 10 % 10}:{chroma % 10}, "
                                   + (f"{a.total_frames} frames split over {world} GPU(s) "
                                      if a.total_frames else f"{nfr} frames per GPU ")
                                   + (f"(BASELINE.json configs[{cfg_idx}]" if a.config != "c1" else
                                      "(SURVEY §8(d) C1: the reference's own 640x480 4:4:4 geometry, c0/common/config.h:23-24; "
                                      "BASELINE.json configs[0] is a single 640x480 4:2:0 frame on the CPU oracle, covered by "
                                      "tests/test_gpu_parity.py::test_baseline_config0_640x480_420_single_frame")
                                   + (", configs[3] scaling" if a.config == "c3" else "") + ")"
                                   + (f", I/P stream, GOP {a.gop}, P-frames accumulated on chip" if a.mode == "stream" else ""),
                       "width": w, "height": h, "chroma": chroma, "frames_per_gpu": nfr,
                       "total_frames": frames_all,
                       "parallelism": f"frame-sharded x{world}", "bytes_per_frame": fbytes, "mode": a.mode},
            "distributed": dict(dinfo, per_rank=[{"rank": r, "ms_per_step": round(v[0], 4),
                                                  "kernel_ms_avg": round(v[1], 4), "frames": int(v[2])}
                                                 for r, v in enumerate(per_rank)] if world > 1 else None),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                         "traffic_source": traffic_src,
                         "kernel": stream_kernel_label(chroma) if a.mode == "stream" else "decode_kernel<%d>" % chroma,
                         "kernel_ms_avg": round(kern_ms_max, 4),
                         "kernel_ms_median": round(kern_med_max, 4),
                         "frac_median": round(launch_bytes / (kern_med_max / 1e3) / 1e9 / HBM_PEAK_GBPS, 4),
                         "bytes_per_launch": launch_bytes},
            "cpu_baseline": cpu,
            "copy_context": copy_ctx,
            "parity_verified": verified,
            "parity_frames_checked": checked,
        }
        if a.mode == "stream":  # (segment, tile) jobs the exact kernel re-ran for the optimistic 4:2:2 kernel
            res["stream_reruns"] = ctx.stream_reruns()
        print(json.dumps(res), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()
    ctx.close()


def main_file(a):
    """--mode file: the streaming whole-file decoder (mj423_decode_mpg_pipelined) on a
    seeded synthetic .mpg written by tools/mpg_synth (untimed).  One step = one pass over
    the whole file: entropy decode on host threads, H2D, stream kernel, D2H, a sink that
    touches every frame.  PCIe- and front-end-inclusive: reported beside the kernel-only
    metric, never as it."""
    sys.path.insert(0, os.path.join(REPO, "tools"))
    import tempfile
    import mpg_synth
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dev, coll_dev, dinfo = init_dist(world, local, a.gpus)
    cfg = a.config if CONFIGS[a.config][2] == 444 else "c1"
    w, h, chroma, frames_cfg, cfg_idx = CONFIGS[cfg]
    nfr = a.frames or frames_cfg
    tmp = tempfile.mkdtemp(prefix="mj423bench")
    if a.mpg:  # a given file, whole: its own size and frame count
        path = a.mpg
        m = mj423.Mpg(path)
        w, h, nfr = m.header.width, m.header.height, m.header.num_frames
        fbytes = os.path.getsize(path)
    else:
        path = os.path.join(tmp, f"synth_r{rank}.mpg")
        fbytes = mpg_synth.write(path, w, h, nfr, gop=a.gop, seed=SEED + rank, nthreads=a.threads)
        m = mj423.Mpg(path)
    ctx = mj423.Context(dev.index)
    yq, cq = ctx.get_quant()
    ctx.set_quant(*shard.broadcast_quant_tables(yq, cq, device=coll_dev))
    ctx.enable_timing(True)
    check = {0, nfr - 1}
    keep = {}
    acc = [0]

    def sink(fi, view):
        acc[0] ^= int(view[0, 0]) ^ int(view[-1, -1])  # touch the frame
        if fi in check:
            keep[fi] = view.copy()
        return 0

    pipe = mj423.Pipeline(ctx, w, h, chunk_frames=a.chunk, nthreads=a.threads)  # buffers + thread pool set up once, untimed
    dkeep = {}

    def dsink(first, frames):  # decode-to-device: keep the check frames (a device copy on the decode stream)
        for fi in check:
            if first <= fi < first + frames.count:
                with torch.cuda.stream(torch.cuda.ExternalStream(frames.stream)):
                    dkeep[fi] = torch.as_tensor(frames, device=dev)[fi - first].view(torch.int32).clone()
        return 0

    gpu_out = torch.empty((nfr, h, w), dtype=torch.int32, device=dev) if a.frontend == "gpu" else None

    def one_pass():
        if a.frontend == "gpu":
            t = time.perf_counter()
            m.decode_gpu(ctx, 0, nfr, gpu_out.data_ptr())
            st = mj423.PipelineStats()
            st.frames, st.chunks, st.wall_s = nfr, 1, time.perf_counter() - t
            return st  # (every pass writes the same frames: the checked ones are copied after timing)
        if a.sink == "device":
            st = pipe.decode_device(m, 0, nfr, dsink)
            ctx.synchronize()
            return st
        return pipe.decode(m, 0, nfr, sink)

    a.warmup = warm_up(one_pass, a.warmup if a.warmup >= 0 else 3, lambda: torch.cuda.synchronize(dev))
    if dist.is_initialized():
        dist.barrier()
    torch.cuda.synchronize(dev)
    ctx.enable_timing(True)  # log only the timed passes' stream-kernel launches
    t0 = time.perf_counter()
    stats = []
    for _ in range(a.steps):
        stats.append(one_pass())
    torch.cuda.synchronize(dev)
    if dist.is_initialized():
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if a.frontend == "gpu":  # the last timed pass's frames, for the parity check below
        for fi in check:
            dkeep[fi] = gpu_out[fi].clone()
    # every stream-kernel launch (one per chunk / window) of the timed passes, HIP events on the
    # context stream they run on
    kern_ms, kern_frames, kern_launches = ctx.kernel_totals()
    elapsed_max = shard.max_over_ranks([elapsed], device=coll_dev)[0]

    verified = None
    if not a.no_verify:
        ok = True
        if a.sink == "device" or a.frontend == "gpu":
            keep = {fi: v.cpu().numpy().view(np.uint32) for fi, v in dkeep.items()}
        for fi in sorted(check):
            ok &= bool(np.array_equal(keep[fi], cpu_leg_mpg_frame(m, fi, w, h)))
        verified = shard.max_over_ranks([0.0 if ok else 1.0], device=coll_dev)[0] == 0.0
    cpu = None
    if dist.is_initialized():
        dist.barrier()
    if rank == 0 and not a.no_cpu:
        last = nfr - 1  # a GPU-decoded frame for the reference to match (the parity check's copy)
        px = (dkeep[last].cpu().numpy().view(np.uint32) if last in dkeep
              else keep[last] if last in keep else None)
        cpu = cpu_baseline_file(m, path, w, h, nfr, a.cpu_seconds, None if px is None else (last, px))
    pmodel = None
    if rank == 0 and a.frontend == "gpu":
        pmodel = file_path_model(m, nfr, w, h, elapsed_max * 1e3 / a.steps, dev)
    if rank == 0:
        total_px = float(world) * nfr * w * h * a.steps
        fused = a.frontend == "gpu" and os.environ.get("MJ423_GPU_FE_FUSED", "1") != "0" \
            and os.environ.get("MJ423_GPU_FE") != "wave"
        # bytes the timed kernel must move per frame: the fused kernel reads the frame's bitstreams and
        # writes BGRA (its block index, 2 B per block + 8 B per tile, is reported in `path`); the
        # stream kernel reads dense int16 planes and writes BGRA
        fb = (pmodel["coded_bytes_per_frame"] + 4 * w * h) if fused else mj423.frame_bytes(w, h, 444)
        achieved = fb * kern_frames / (kern_ms / 1e3) / 1e9 if kern_ms > 0 else None
        fe = float(np.mean([s.frontend_busy_s for s in stats]))
        # the fused kernel's HBM bytes from the committed PMC passes (tools/pmc_file_summary.py
        # --traffic-entry), per launch of a pass, while its sources are unchanged
        traffic, traffic_src = (pmc_traffic(f"{w}x{h}_444_{nfr}f_file_fused", mj423.FUSED_SOURCES) if fused and not a.mpg
                                else (None, None))  # (the committed PMC passes are of the synthetic file)
        res = {
            "metric": "Mpixels/s decoded end to end from .mpg (entropy decode + PCIe + dequant+IDCT+CSC)"
                      + (", frames left in HBM" if a.sink == "device" or a.frontend == "gpu"
                         else ", frames downloaded to host"),
            "value": round(total_px / elapsed_max / 1e6, 1),
            "unit": "Mpix/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
            "ms_per_step": round(elapsed_max * 1e3 / a.steps, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int32",
            "data": (f"given .mpg {os.path.basename(a.mpg)}, " if a.mpg else
                     f"synthetic seeded 4:4:4 .mpg (tools/mpg_synth, SURVEY §8(d) statistics, I every {a.gop}), ")
                    + f"{fbytes / nfr / 1e6:.2f} MB/frame coded",
            "config": {"workload": f"{w}x{h} 4:4:4 .mpg, {nfr} frames per GPU, whole streaming decoder",
                       "width": w, "height": h, "chroma": 444, "frames_per_gpu": nfr, "mode": "file",
                       "frontend_threads": a.threads, "chunks": int(stats[-1].chunks), "sink": a.sink,
                       "frontend": a.frontend,
                       "parallelism": f"file-per-rank x{world}"},
            "distributed": dinfo,
            "breakdown": {"frontend_busy_s_per_pass": round(fe, 4),
                          "frontend_Mpix_s": round(nfr * w * h / fe / 1e6, 1) if fe > 0 else None,
                          "gpu_span_ms_per_pass": round(float(np.mean([s.gpu_span_ms for s in stats])), 3),
                          "sink_busy_s_per_pass": round(float(np.mean([s.sink_busy_s for s in stats])), 4)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1) if achieved else None, "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4) if achieved else None,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "limiter": ({"kind": "valu", "evidence": "SQ counters (profiles/r05/file/f2_pmc_per_kernel.json): "
                                      "VALU issued in ~0.22 of each wave's cycles at 4 waves per SIMD, the block transform "
                                      "~14 lane-ops per plane pixel; HBM bytes are a fifth of 8 TB/s"} if fused else None),
                         "kernel": ("mpg_fused_kernel (entropy decode + P accumulation + dequant + IDCT + CSC; bytes = "
                                    "the frames' bitstreams read + BGRA written)" if fused else "decode_gop_kernel<444>")
                                   + ", every launch of the timed passes",
                         "kernel_launches": kern_launches,
                         "kernel_ms_avg": round(kern_ms / max(1, kern_launches), 4),
                         "bytes_per_launch": round(fb * kern_frames / max(1, kern_launches))},
            "path": pmodel,
            "cpu_baseline": cpu,
            "parity_verified": verified,
        }
        print(json.dumps(res), flush=True)
    pipe.close()
    m.close()
    ctx.close()
    try:
        if not a.mpg:
            os.remove(path)
        os.rmdir(tmp)
    except OSError:
        pass
    if dist.is_initialized():
        dist.destroy_process_group()


def file_path_model(m, nfr, w, h, pass_ms, dev):
    """Byte model of one whole-file GPU pass (mj423_mpg_decode_gpu): the file's frame
    bytes cross PCIe once (host -> HBM), the pass must read them and write every BGRA frame once;
    the fused form's only intermediate is its block index.  The link's achievable rate is measured
    here, on this box, with pinned copies of the same byte count; the bound is whichever floor --
    PCIe at that rate, or HBM at 8 TB/s -- is higher."""
    f0, f1 = m.frame(0), m.frame(nfr - 1)
    upload = int(f1.position + f1.frame_size - f0.position)
    coded = sum(int(m.frame(i).y_size + m.frame(i).cb_size + m.frame(i).cr_size) for i in range(nfr))
    g = m.geometry()
    tiles = -(-g.y_blocks // 64)
    index_b = nfr * 3 * (2 * g.y_blocks + 8 * tiles)
    host = torch.empty(upload, dtype=torch.uint8, pin_memory=True)
    devb = torch.empty(upload, dtype=torch.uint8, device=dev)
    for _ in range(2):
        devb.copy_(host, non_blocking=True)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(5):
        devb.copy_(host, non_blocking=True)
    e1.record()
    e1.synchronize()
    h2d_gbps = upload * 5 / (e0.elapsed_time(e1) * 1e-3) / 1e9
    del host, devb
    hbm = coded + 4 * nfr * w * h
    pcie_ms = upload / (h2d_gbps * 1e9) * 1e3
    hbm_ms = hbm / (HBM_PEAK_GBPS * 1e9) * 1e3
    bound = "pcie" if pcie_ms >= hbm_ms else "hbm"
    return {"bound": bound, "pass_ms": round(pass_ms, 4),
            "pcie_bytes": upload, "pcie_GBps_measured": round(h2d_gbps, 2), "pcie_floor_ms": round(pcie_ms, 4),
            "hbm_bytes_algorithmic": hbm, "hbm_floor_ms_at_8TBps": round(hbm_ms, 4),
            "frac_of_bound": round(max(pcie_ms, hbm_ms) / pass_ms, 4),
            "coded_bytes_per_frame": coded / nfr, "index_bytes": index_b,
            "note": "pcie_bytes = the frames' bytes uploaded per pass; hbm_bytes_algorithmic = those bitstreams "
                    "read once + 4 B per pixel written; index_bytes = the fused form's block index (written "
                    "once, read once); H2D rate = 5 pinned copies of pcie_bytes on this box"}


# ------------------------------------------------------------------------- CPU leg
# The only code in bench.py that touches oracle/ (test infrastructure): the checker that
# compares the timed GPU output with the bit-exact CPU restatement, and the timed CPU
# baselines.  Both run after the GPU timing; nothing measured as `value` goes through here.

def rank0_cpu_baseline(rank, coef, out, nfr, w, h, chroma, g, budget_s, skip=False):
    """The CPU baseline on rank 0 at every world size (north_star: the reference's core0/core1 CPU
    path timed on the node's host cores in the same run), after every rank has finished its GPU
    timing and its verification (that sum is a collective; the barrier makes the ordering explicit),
    so no other rank's CPU work overlaps it.  Other ranks return None."""
    if dist.is_initialized():
        dist.barrier()
    if rank != 0 or skip:
        return None
    cpu = cpu_baseline_reference(coef, out, nfr, w, h, chroma, g, budget_s)
    if cpu is None:
        print("bench.py: WARNING oracle/_ref/libmjref.so (the reference's own build) is absent; "
              "timing the oracle port as the CPU baseline (cpu_baseline.kind = port)", file=sys.stderr, flush=True)
        cpu = cpu_baseline(coef, nfr, w, h, chroma, g, budget_s)
    cpu["world_size"] = dist.get_world_size() if dist.is_initialized() else 1
    return cpu


def cpu_leg_check_frames(coef, out, nfr, w, h, chroma, frames):
    """Frames (indices into this rank's batch) of the GPU output vs the oracle, 8 at a time.
    Returns (mismatched, checked)."""
    import oracle
    # ranks on one node share the host's CPUs: each checks with its share (N = 8 would otherwise
    # oversubscribe the job's CPUs eight times; this runs after timing, so only the wall clock grows)
    local = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1))
    threads = max(1, host_cpus()["threads"] // local)
    bad = checked = 0
    for k in range(0, len(frames), 8):
        pick = frames[k:k + 8]
        c_host = coef.view(nfr, -1)[pick].cpu().numpy()
        o_host = out.view(nfr, h, w)[pick].cpu().numpy().view(np.uint32)
        exp = oracle.decode_frames_mt(c_host, len(pick), w, h, chroma, nthreads=threads)
        bad += sum(0 if np.array_equal(o_host[i], exp[i]) else 1 for i in range(len(pick)))
        checked += len(pick)
    return bad, checked


def host_cpus():
    """What the host gives this process: nproc (os.cpu_count(), the whole machine), the CPUs in
    its affinity mask, the cgroup CPU quota, and the CPU model.  `threads` = the smallest of
    affinity, quota and the job's CPU share in OMP_NUM_THREADS when the launcher sets one (the
    GPU pool shows every CPU of a shared machine in nproc but grants each GPU job a share) --
    i.e. every core this run may use.  `limit` names what set it."""
    nproc = os.cpu_count() or 1
    try:
        allowed = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        allowed = nproc
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    # OMP_NUM_THREADS is a per-process share (the box sets it to the GPU job's CPUs; a launcher may
    # set it per rank): the job's share on this node is that times the ranks on the node
    share = None
    omp = os.environ.get("OMP_NUM_THREADS")
    # torch.distributed.run sets OMP_NUM_THREADS=1 per rank when the caller left it unset: that is the
    # launcher's default, not a CPU share the job was given, so it is not taken as one
    launcher_default = omp == "1" and os.environ.get("TORCHELASTIC_RUN_ID") is not None
    try:
        local = max(1, int(os.environ.get("LOCAL_WORLD_SIZE", "1") or 1))
        share = int(omp) * local if omp and not launcher_default else None
    except ValueError:
        pass
    cands = [("nproc", nproc), ("affinity", allowed)] + ([("cgroup cpu.max", quota)] if quota else []) + \
            ([("OMP_NUM_THREADS job share", share)] if share else [])
    limit, threads = min(cands, key=lambda kv: kv[1])
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"nproc": nproc, "cpus_allowed": allowed, "cgroup_cpus": quota, "job_cpu_share": share,
            "omp_num_threads_ignored": "torch.distributed.run's default of 1" if launcher_default else None,
            "threads": max(1, threads), "limit": limit, "cpu_model": model}


def _timed_parallel(fn, nitems, threads, budget_s, max_items=1 << 20):
    """Calls fn(item, slot) for items 0, 1, 2, ... on `threads` threads until about budget_s
    seconds have passed; each thread owns slot = its index (private scratch/output buffers).
    Returns (items done, wall seconds)."""
    import threading
    lock = threading.Lock()
    nxt = [0]
    deadline = [0.0]

    def worker(slot):
        while True:
            with lock:
                k = nxt[0]
                if k >= max_items or (k >= threads and time.perf_counter() > deadline[0]):
                    return
                nxt[0] += 1
            fn(k % nitems, slot)

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(threads)]
    t0 = time.perf_counter()
    deadline[0] = t0 + budget_s
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    return nxt[0], time.perf_counter() - t0


def cpu_baseline_reference(coef, out, nfr, w, h, chroma, g, budget_s):
    """The reference's OWN idct() + ycbcr_to_rgb() (mj/decoder/idct.c, ycbcr_to_rgb.c compiled
    in place into oracle/_ref by oracle/Makefile; travels with the snapshot) through its frame
    loop (mjpeg423_decoder.c:114-124 restated by oracle/ref_harness.c: ref_decode_frame_444, or
    ref_decode_frame_sub for 4:2:x, which adds only the A7 nearest-neighbour chroma gather),
    timed (i) on one thread and (ii) frame-parallel on every host core this job may use
    (host_cpus()).  Input dequantized like the reference's lossless_decode leaves it (done
    beforehand, untimed).  Frame 0's reference output is also compared with the GPU's (`out`)."""
    import ctypes
    import oracle
    ref = oracle.ref_lib()
    if ref is None:
        return None
    hc = host_cpus()
    threads = hc["threads"]
    ny, nc = g.y_blocks, g.c_blocks
    cw, ch = g.y_bw * 8, g.y_bh * 8  # coded size: the reference writes whole blocks
    n = int(min(nfr, 64, max(1, (1 << 30) // (2 * g.coef_per_frame))))  # <= 1 GiB of dequantized planes
    q = coef.view(nfr, -1)[:n].cpu().numpy()
    tab = np.concatenate([np.tile(oracle.YQUANT.astype(np.int32), ny), np.tile(oracle.CQUANT.astype(np.int32), 2 * nc)])
    deq = (q.astype(np.int32) * tab[None, :]).astype(np.int16)  # (int16)(Q*q), lossless_decode.c:94-95,124-125
    outs = [np.empty((ch, cw), np.uint32) for _ in range(threads)]
    scratch = [np.empty(64 * (ny + 2 * nc), np.uint8) for _ in range(threads)]
    P = ctypes.c_void_p

    def one(i, slot):
        d = deq[i]
        Y, Cb, Cr = d[:64 * ny], d[64 * ny:64 * (ny + nc)], d[64 * (ny + nc):]
        if chroma == 444:
            ref.ref_decode_frame_444(ctypes.c_uint32(cw), ctypes.c_uint32(ch), Y.ctypes.data_as(P), Cb.ctypes.data_as(P),
                                     Cr.ctypes.data_as(P), scratch[slot].ctypes.data_as(P), outs[slot].ctypes.data_as(P))
        else:
            ref.ref_decode_frame_sub(ctypes.c_uint32(cw), ctypes.c_uint32(ch), ctypes.c_int(chroma), Y.ctypes.data_as(P),
                                     Cb.ctypes.data_as(P), Cr.ctypes.data_as(P), scratch[slot].ctypes.data_as(P),
                                     outs[slot].ctypes.data_as(P))

    one(0, 0)
    gpu0 = out.view(nfr, h, w)[0].cpu().numpy().view(np.uint32)
    matches = bool(np.array_equal(outs[0][:h, :w], gpu0))
    single_budget = min(4.0, budget_s / 3)
    done1, dt1 = _timed_parallel(one, n, 1, single_budget)
    done, dt = _timed_parallel(one, n, threads, budget_s - single_budget)
    single = done1 * w * h / dt1 / 1e6
    return {"value": round(done * w * h / dt / 1e6, 2), "unit": "Mpix/s", "cores": threads, "kind": "reference",
            "threads": threads, "nproc": hc["nproc"], "cpus_allowed": hc["cpus_allowed"],
            "cgroup_cpus": hc["cgroup_cpus"], "job_cpu_share": hc["job_cpu_share"], "threads_limited_by": hc["limit"],
            "cpu_model": hc["cpu_model"], "single_thread_mpix_s": round(single, 2),
            "sample": f"{done} frames (cycling over {n} of the same synthetic frames) through the reference's own "
                      f"idct()+ycbcr_to_rgb() frame loop" + ("" if chroma == 444 else " (+ the A7 chroma gather)")
                      + f" on {threads} threads ({dt:.1f} s; threads = {hc['limit']}), input pre-dequantized; "
                      f"single thread: {done1} frames in {dt1:.1f} s = {single:.1f} Mpix/s; "
                      f"frame 0 equals the GPU output: {matches}",
            "reference_equals_gpu_frame0": matches}


def cpu_baseline(coef, nfr, w, h, chroma, g, budget_s):
    """The oracle (bit-exact C restatement of the reference's idct()+ycbcr_to_rgb(),
    compiled -O3 -std=c99 like the reference) over a bounded sample of the same synthetic
    frames, on one thread and frame-parallel on every host core this job may use.  Used only
    when oracle/_ref/libmjref.so (the reference's own build) is absent; the JSON says so."""
    import oracle
    hc = host_cpus()
    threads = hc["threads"]
    n = min(nfr, 64)
    sample = coef.view(nfr, -1)[:n].cpu().numpy()
    frames = [sample[i:i + 1] for i in range(n)]
    one = lambda i, slot: oracle.decode_frames_mt(frames[i], 1, w, h, chroma, nthreads=1)  # noqa: E731
    single_budget = min(4.0, budget_s / 3)
    done1, dt1 = _timed_parallel(one, n, 1, single_budget)
    done, dt = _timed_parallel(one, n, threads, budget_s - single_budget)
    single = done1 * w * h / dt1 / 1e6
    return {"value": round(done * w * h / dt / 1e6, 2), "unit": "Mpix/s", "cores": threads, "kind": "port",
            "threads": threads, "nproc": hc["nproc"], "cpus_allowed": hc["cpus_allowed"],
            "cgroup_cpus": hc["cgroup_cpus"], "job_cpu_share": hc["job_cpu_share"], "threads_limited_by": hc["limit"],
            "cpu_model": hc["cpu_model"], "single_thread_mpix_s": round(single, 2),
            "fallback": "oracle/_ref/libmjref.so (the reference's own build) is absent: the oracle port was timed",
            "sample": f"{done} frames (cycling over {n} of the same {w}x{h} {chroma} synthetic frames) on {threads} "
                      f"threads ({dt:.1f} s; threads = {hc['limit']}); single thread: {done1} frames in "
                      f"{dt1:.1f} s = {single:.1f} Mpix/s"}


def _oracle_planes(m, f, nb, state):
    """Oracle front end (quantized-domain lossless_decode) of frame f onto `state`."""
    import ctypes
    import oracle
    fr = m.frame(f)
    P = fr.frame_type != 0
    for pi, (ptr, size) in enumerate(((fr.y, fr.y_size), (fr.cb, fr.cb_size), (fr.cr, fr.cr_size))):
        bs = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint8)), shape=(size,))
        state[pi] = oracle.lossless_decode_q(nb, np.concatenate([bs, np.zeros(8, np.uint8)]), P,
                                             prev=state[pi] if P else None)


def cpu_leg_mpg_frame(m, fi, w, h):
    """Frame fi of an .mpg by the oracle alone: front end from its GOP start + pixel path."""
    import oracle
    state = [None, None, None]
    for f in range(m.gop_start(fi), fi + 1):
        _oracle_planes(m, f, (w // 8) * (h // 8), state)
    return oracle.decode_frame(state[0], state[1], state[2], w, h, 444)


def cpu_baseline_file(m, path, w, h, nfr, budget_s, gpu_frame=None):
    """The reference's OWN decoder loop (mjpeg423_decoder.c:90-124 minus the BMP write: per frame its
    lossless_decode() of the three planes, P-frames accumulating, then idct() + ycbcr_to_rgb(); all
    three compiled in place from /root/reference into oracle/_ref/libmjref.so, driven by
    oracle/ref_harness.c:ref_decode_mpg_frames) over the same .mpg's GOPs -- frames inside a GOP are
    serial, GOPs are independent -- timed (i) on one thread and (ii) GOP-parallel on every host CPU
    this job may use (host_cpus()), cycling over the file's GOPs until the budget is spent.
    gpu_frame = (index, pixels) of one GPU-decoded frame: the reference decodes its GOP up to it and
    the two are compared.  Without oracle/_ref, the oracle's restatement on one thread (kind "port")."""
    import ctypes
    import oracle
    ref = oracle.ref_lib()
    if ref is None:
        return cpu_baseline_file_port(m, w, h, nfr, budget_s)
    hc = host_cpus()
    threads = hc["threads"]
    data = np.fromfile(path, dtype=np.uint8)
    pos = np.array([m.frame(i).position for i in range(m.header.num_frames)], np.uint64)
    types = [m.frame(i).frame_type for i in range(nfr)]
    gops = [i for i in range(nfr) if types[i] == 0] + [nfr]
    gop_ranges = list(zip(gops[:-1], gops[1:]))
    P = ctypes.c_void_p
    fn = ref.ref_decode_mpg_frames
    fn.restype = ctypes.c_int
    frames_done = [0] * max(1, threads)
    bad = []

    def one(i, slot):
        f0, f1 = gop_ranges[i]
        r = fn(data.ctypes.data_as(P), pos.ctypes.data_as(P), ctypes.c_uint32(f0), ctypes.c_uint32(f1),
               ctypes.c_uint32(w), ctypes.c_uint32(h), None)
        if r != f1 - f0:
            bad.append((f0, f1, r))
        frames_done[slot] += max(0, r)

    matches = None
    if gpu_frame is not None:
        fi, px = gpu_frame
        g0 = max(f for f, _ in gop_ranges if f <= fi)
        rgb = np.empty((h, w), np.uint32)
        fn(data.ctypes.data_as(P), pos.ctypes.data_as(P), ctypes.c_uint32(g0), ctypes.c_uint32(fi + 1),
           ctypes.c_uint32(w), ctypes.c_uint32(h), rgb.ctypes.data_as(P))
        cw, ch = w & ~7, h & ~7  # the reference writes the coded (whole-block) region only
        matches = bool(np.array_equal(rgb[:ch, :cw], px[:ch, :cw]))
    single_budget = min(6.0, budget_s / 3)
    done1, dt1 = _timed_parallel(one, len(gop_ranges), 1, single_budget)
    f1 = sum(frames_done)
    frames_done[:] = [0] * len(frames_done)
    done, dt = _timed_parallel(one, len(gop_ranges), threads, budget_s - single_budget)
    fr = sum(frames_done)
    single = f1 * w * h / dt1 / 1e6
    glen = float(np.mean([b - a for a, b in gop_ranges]))
    return {"value": round(fr * w * h / dt / 1e6, 2), "unit": "Mpix/s", "cores": threads, "kind": "reference",
            "threads": threads, "nproc": hc["nproc"], "cpus_allowed": hc["cpus_allowed"],
            "cgroup_cpus": hc["cgroup_cpus"], "job_cpu_share": hc["job_cpu_share"], "threads_limited_by": hc["limit"],
            "cpu_model": hc["cpu_model"], "single_thread_mpix_s": round(single, 2),
            "sample": f"{fr} frames ({done} GOPs of ~{glen:.0f} frames, cycling over the file's {len(gop_ranges)} GOPs) "
                      f"through the reference's own decoder loop (lossless_decode x3 + idct + ycbcr_to_rgb per frame, "
                      f"mjpeg423_decoder.c:90-124 minus the BMP write), GOP-parallel on {threads} threads "
                      f"({dt:.1f} s; threads = {hc['limit']}); single thread: {f1} frames in {dt1:.1f} s = "
                      f"{single:.1f} Mpix/s" + ("" if matches is None else f"; frame {gpu_frame[0]} equals the GPU "
                                                f"output: {matches}")
                      + (f"; FAILED GOPs {bad[:3]}" if bad else ""),
            "reference_equals_gpu": matches}


def cpu_baseline_file_port(m, w, h, nfr, budget_s):
    """Without oracle/_ref: the reference's per-frame loop restated by the oracle on one core:
    quantized-domain lossless_decode of the three planes (P-frames accumulating) + idct +
    ycbcr_to_rgb, over the file's frames in order until the budget is spent."""
    import oracle
    nb = (w // 8) * (h // 8)
    state = [None, None, None]
    t0 = time.perf_counter()
    n = 0
    while n < nfr and time.perf_counter() - t0 < budget_s:
        _oracle_planes(m, n, nb, state)
        oracle.decode_frame(state[0], state[1], state[2], w, h, 444)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n * w * h / dt / 1e6, 2), "unit": "Mpix/s", "cores": 1, "kind": "port",
            "fallback": "oracle/_ref/libmjref.so (the reference's own build) is absent: the oracle port was timed",
            "sample": f"first {n} frames of the same .mpg, in order, one thread ({dt:.1f} s): front end + "
                      f"idct + ycbcr_to_rgb per frame (the reference's decoder loop minus BMP writes)"}


if __name__ == "__main__":
    main()
