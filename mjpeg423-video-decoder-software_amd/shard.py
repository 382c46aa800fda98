"""Frame sharding across GPUs (one process per GPU, torch.distributed).

The decode path partitions by FRAME: given absolute quantized coefficients
 frames are independent, so rank r takes a contiguous frame range
and no coefficient or pixel ever crosses a GPU.  The reference's only inter-core
exchange -- the mailbox hand-offs of c0/playback.c:80-134 / c1/main.c:227-335 --
has no data-path counterpart here; what remains global is the decoder's
configuration: the quantization tables (mj/common/tables.c:13-32), which rank 0
broadcasts once over RCCL (xGMI) as 256 bytes.

For real P-frame streams a shard must start at an I-frame: P-frames accumulate
coefficients across frames (mj/decoder/lossless_decode.c:90-92,121-122), so
`gop_aligned_ranges` cuts at the I-frame indices of the .mpg trailer
(mj/common/mjpeg423_types.h:22-25, mj/encoder/mjpeg423_encoder.c:204-207).
"""
from __future__ import annotations

import numpy as np


def frame_range(rank: int, world: int, total: int) -> tuple[int, int]:
    """Contiguous [start, stop) of `total` frames for `rank` of `world`; sizes differ by <= 1."""
    if world <= 0 or not 0 <= rank < world or total < 0:
        raise ValueError("bad rank/world/total")
    base, extra = divmod(total, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def weak_range(rank: int, per_gpu: int) -> tuple[int, int]:
    """Weak scaling: every rank decodes `per_gpu` frames, global frames [rank*per_gpu, ...)."""
    return rank * per_gpu, (rank + 1) * per_gpu


def gop_aligned_ranges(iframe_indices, total: int, world: int) -> list[tuple[int, int]]:
    """Split [0, total) into `world` contiguous ranges that each start at an I-frame,
    balancing frame counts.  iframe_indices must contain 0 and be ascending."""
    idx = sorted(set(int(i) for i in iframe_indices if 0 <= int(i) < total))
    if not idx or idx[0] != 0:
        raise ValueError("the stream must start with an I-frame")
    cuts = [0]
    for r in range(1, world):
        target = r * total / world
        best = min(idx, key=lambda i: (abs(i - target), i))
        if best > cuts[-1]:
            cuts.append(best)
    cuts.append(total)
    ranges = [(a, b) for a, b in zip(cuts[:-1], cuts[1:])]
    while len(ranges) < world:  # fewer GOPs than ranks: idle ranks get empty ranges
        ranges.append((total, total))
    return ranges


def broadcast_quant_tables(yquant, cquant, device=None, src: int = 0):
    """Rank `src`'s tables to every rank (one 256-byte broadcast; RCCL on GPUs, gloo on CPU).
    Returns (yquant, cquant) as int16[64] numpy arrays on every rank."""
    import torch
    import torch.distributed as dist
    buf = torch.from_numpy(np.concatenate([np.asarray(yquant, np.int16), np.asarray(cquant, np.int16)])
                           .view(np.uint8).copy())
    if device is not None:
        buf = buf.to(device)
    if dist.is_available() and dist.is_initialized():
        dist.broadcast(buf, src=src)
    host = buf.cpu().numpy().view(np.int16)
    return host[:64].copy(), host[64:].copy()


def max_over_ranks(values, device=None):
    """Element-wise max of a list of floats over all ranks (timing reduction)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(x) for x in t.cpu()]


def sum_over_ranks(values, device=None):
    """Element-wise sum of a list of floats over all ranks (parity counts)."""
    import torch
    import torch.distributed as dist
    t = torch.tensor(list(values), dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [float(x) for x in t.cpu()]


def gather_over_ranks(values, device=None):
    """Every rank's list of floats, as a list indexed by rank (per-rank timing report)."""
    import torch
    import torch.distributed as dist
    vals = [float(v) for v in values]
    if not (dist.is_available() and dist.is_initialized()):
        return [vals]
    world, rank = dist.get_world_size(), dist.get_rank()
    t = torch.zeros((world, len(vals)), dtype=torch.float64, device=device)
    t[rank] = torch.tensor(vals, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return [[float(x) for x in row] for row in t.cpu()]
