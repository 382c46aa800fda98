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
}
HBM_PEAK_GBPS = 8000.0  # MI355X spec (MI355X_MICROARCH.md, chip-level parameters)
SEED = 0x4D4A3432


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--frames", type=int, default=0, help="frames per GPU (default: the config's)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget for the CPU baseline sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-verify", action="store_true")
    ap.add_argument("--mode", default="batch", choices=["batch", "stream"],
                    help="batch: every frame absolute (decode_kernel); stream: I/P GOPs with P-frame "
                         "deltas accumulated on chip (decode_gop_kernel, SURVEY §8(f) row 3)")
    ap.add_argument("--gop", type=int, default=24, help="stream mode: I-frame interval (mj/sample_main.c:30)")
    return ap.parse_args()


def pmc_traffic(workload_key):
    """HBM bytes per launch from the committed rocprofv3 PMC summary, if one exists."""
    path = os.path.join(PROFILES, "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        return d.get(workload_key, {}).get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    a = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    w, h, chroma, frames_cfg, cfg_idx = CONFIGS[a.config]
    nfr = a.frames or frames_cfg
    g = mj423.geometry(w, h, chroma)

    ctx = mj423.Context(local)
    # A dedicated (non-null) stream shared by torch and the library: the kernel
    # launches and the timing events below are on the same stream.
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)

    # Quantization tables: rank 0's tables reach every GPU over RCCL (xGMI); 256 B.
    yq, cq = ctx.get_quant()
    ctx.set_quant(*shard.broadcast_quant_tables(yq, cq, device=dev))

    # This rank's shard (weak scaling): global frames [rank*nfr, (rank+1)*nfr), generated on-device.
    first, _ = shard.weak_range(rank, nfr)
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
        pmask = torch.from_numpy(types[1:].astype(bool)).to(dev)
        stream_in[1:][pmask] = cv[1:][pmask] - cv[:-1][pmask]
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

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize(dev)

    starts = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps)]
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(a.steps):
        starts[i].record(stream)
        step()
        ends[i].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = [s.elapsed_time(e) for s, e in zip(starts, ends)]
    elapsed_max, kern_ms_max = shard.max_over_ranks([elapsed, float(np.mean(kern_ms))], device=dev)

    # Parity spot check of the timed output (two frames of this rank) against the oracle.
    verified = None
    if not a.no_verify:
        import oracle
        pick = sorted({0, nfr - 1})
        c_host = coef.view(nfr, -1)[pick].cpu().numpy()
        o_host = out.view(nfr, h, w)[pick].cpu().numpy().view(np.uint32)
        exp = oracle.decode_frames_mt(c_host, len(pick), w, h, chroma, nthreads=min(16, os.cpu_count() or 1))
        verified = shard.max_over_ranks([0.0 if np.array_equal(o_host, exp) else 1.0], device=dev)[0] == 0.0

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu:
        cpu = cpu_baseline(coef, nfr, w, h, chroma, g, a.cpu_seconds)

    if rank == 0:
        total_px = float(world) * nfr * w * h * a.steps
        value = total_px / elapsed_max / 1e6
        fbytes = mj423.frame_bytes(w, h, chroma)
        launch_bytes = fbytes * nfr
        achieved = launch_bytes / (kern_ms_max / 1e3) / 1e9
        key = f"{w}x{h}_{chroma}_{nfr}f" + ("_stream" if a.mode == "stream" else "")
        traffic = pmc_traffic(key)
        res = {
            "metric": "Mpixels/s decoded (dequant+IDCT+CSC) at 1/2/4/8 GPUs; % HBM roofline",
            "value": round(value, 1),
            "unit": "Mpix/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed_max * 1e3 / a.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic: device-generated seeded quantized-coefficient stream (SURVEY §8(d)), resident in HBM"
                    + (f"; stream mode: I every {a.gop} frames, P-frames as deltas" if a.mode == "stream" else ""),
            "config": {"workload": f"{w}x{h} {chroma // 100}:{chroma // 10 % 10}:{chroma % 10}, {nfr} frames per GPU "
                                   f"(BASELINE.json configs[{cfg_idx}]" + (", configs[3] scaling" if a.config == "c3" else "") + ")"
                                   + (f", I/P stream, GOP {a.gop}, P-frames accumulated on chip" if a.mode == "stream" else ""),
                       "width": w, "height": h, "chroma": chroma, "frames_per_gpu": nfr,
                       "parallelism": f"frame-sharded x{world}", "bytes_per_frame": fbytes, "mode": a.mode},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                         "kernel": ("decode_gop_kernel<%d>" if a.mode == "stream" else "decode_kernel<%d>") % chroma, "kernel_ms_avg": round(kern_ms_max, 4),
                         "bytes_per_launch": launch_bytes},
            "cpu_baseline": cpu,
            "parity_verified": verified,
        }
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()
    ctx.close()


def cpu_baseline(coef, nfr, w, h, chroma, g, budget_s):
    """The oracle (bit-exact C restatement of the reference's idct()+ycbcr_to_rgb(),
    compiled -O3 -std=c99 like the reference) on the host cores, frame-parallel, over a
    bounded sample of the same synthetic frames: whole passes over (up to) the rank's
    frames until about `budget_s` seconds of wall time have been spent."""
    import oracle
    threads = max(1, min(16, os.cpu_count() or 1))
    one = coef.view(nfr, -1)[:1].cpu().numpy()
    t = time.perf_counter()
    oracle.decode_frames_mt(one, 1, w, h, chroma, nthreads=1)
    t1 = time.perf_counter() - t
    n = min(nfr, max(threads, int(budget_s * threads / max(t1, 1e-6))))
    sample = coef.view(nfr, -1)[:n].cpu().numpy()
    passes, dt = 0, 0.0
    while dt < budget_s and passes < 1000:
        t = time.perf_counter()
        oracle.decode_frames_mt(sample, n, w, h, chroma, nthreads=threads)
        dt += time.perf_counter() - t
        passes += 1
    return {"value": round(passes * n * w * h / dt / 1e6, 2), "unit": "Mpix/s", "cores": threads, "kind": "port",
            "sample": f"{passes} pass(es) over {n} of the same {w}x{h} {chroma} synthetic frames, frame-parallel "
                      f"over {threads} threads ({dt:.1f} s); single-thread 1 frame: {w * h / t1 / 1e6:.1f} Mpix/s"}


if __name__ == "__main__":
    main()
