"""CPU, world_size 2 over gloo: the N>1 path of bench.py -- quant-table broadcast,
frame sharding, max-over-ranks timing -- and that a frame-sharded decode equals the
single-process decode (the oracle stands in for the GPU kernel here; the GPU
kernel itself is pinned to the oracle by tests/test_gpu_parity.py)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, total, q):
    import sys
    from conftest import ORACLE, PKG
    for p in (PKG, ORACLE):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist
    import oracle
    import shard
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # rank 0 owns the tables; rank 1 starts from garbage and must receive them
        yq, cq = (oracle.YQUANT, oracle.CQUANT) if rank == 0 else (np.full(64, -7, np.int16), np.ones(64, np.int16))
        yq, cq = shard.broadcast_quant_tables(yq, cq)
        w, h, chroma = 48, 32, 420
        rng = np.random.default_rng(1234)
        coef = oracle.random_quantized_planes(rng, w, h, chroma, nframes=total)  # identical on every rank
        a, b = shard.frame_range(rank, world, total)
        out = oracle.decode_frames_mt(coef[a:b], b - a, w, h, chroma) if b > a else np.zeros((0, h, w), np.uint32)
        t = shard.max_over_ranks([float(rank), -float(rank)])
        n = shard.sum_over_ranks([float(b - a), 1.0])  # bench.py: frames checked over all ranks
        q.put((rank, a, b, yq.tolist(), cq.tolist(), out, t, n))
    finally:
        dist.destroy_process_group()


def test_two_rank_sharded_decode():
    world, total = 2, 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, total, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    import oracle
    for r in res:
        assert r[3] == oracle.YQUANT.tolist() and r[4] == oracle.CQUANT.tolist()
        assert r[6] == [1.0, 0.0]
        assert r[7] == [float(total), float(world)]
    assert [(r[1], r[2]) for r in res] == [(0, 3), (3, 5)]
    sharded = np.concatenate([r[5] for r in res])
    rng = np.random.default_rng(1234)
    coef = oracle.random_quantized_planes(rng, 48, 32, 420, nframes=total)
    assert np.array_equal(sharded, oracle.decode_frames_mt(coef, total, 48, 32, 420))


def test_frame_ranges_cover_exactly():
    import shard
    for world in (1, 2, 3, 4, 8):
        for total in (0, 1, 7, 300, 2400):
            rs = [shard.frame_range(r, world, total) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == total
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(b - a for a, b in rs) - min(b - a for a, b in rs) <= 1
    assert shard.weak_range(3, 300) == (900, 1200)


def test_gop_aligned_ranges():
    import shard
    iframes = [0, 24, 48, 72, 96, 120]
    rs = shard.gop_aligned_ranges(iframes, 130, 4)
    assert rs[0][0] == 0 and rs[-1][1] == 130
    assert all(a in iframes for a, _ in rs if a < 130)
    assert all(x[1] == y[0] for x, y in zip(rs, rs[1:]))
    with pytest.raises(ValueError):
        shard.gop_aligned_ranges([5, 10], 20, 2)
    assert shard.gop_aligned_ranges([0], 10, 3) == [(0, 10), (10, 10), (10, 10)]


def _bench_worker(rank, world, port, q):
    """One rank of bench.py's post-timing leg on CPU tensors: the rank-0 CPU baseline after a
    barrier (every world size, not only 1) and the provenance-checked PMC traffic lookup."""
    import sys
    from conftest import ORACLE, PKG, REPO
    for p in (PKG, ORACLE, REPO):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world))
    import torch
    import torch.distributed as dist
    import bench
    import mj423
    import oracle
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        w, h, chroma, nfr = 64, 48, 420, 3
        rng = np.random.default_rng(7 + rank)
        coef = oracle.random_quantized_planes(rng, w, h, chroma, nframes=nfr)
        out = oracle.decode_frames_mt(coef, nfr, w, h, chroma)
        g = mj423.geometry(w, h, chroma)
        cpu = bench.rank0_cpu_baseline(rank, torch.from_numpy(coef.reshape(-1)),
                                       torch.from_numpy(out.view(np.int32).reshape(-1)), nfr, w, h, chroma, g, 0.6)
        traffic, src = bench.pmc_traffic("3840x2160_420_300f")
        q.put((rank, cpu, traffic, src))
    finally:
        dist.destroy_process_group()


def test_bench_cpu_baseline_and_traffic_at_two_ranks():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=180) for _ in range(world)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (_, cpu0, t0, s0), (_, cpu1, _, _) = res
    assert cpu1 is None  # only rank 0 times the CPU path
    assert cpu0["value"] > 0 and cpu0["cores"] >= 1 and cpu0["world_size"] == world
    assert cpu0["kind"] in ("reference", "port")
    if cpu0["kind"] == "reference":
        assert cpu0["reference_equals_gpu_frame0"] is True  # `out` here is the oracle's decode
    # traffic: reported only from an entry measured on this tree's kernel sources
    import mj423
    assert s0["tree_kernel_src_digest"] == mj423.kernel_source_digest()
    assert (t0 is not None) == (s0["status"] == "current")
    if s0["status"] == "current":
        assert s0["kernel_src_digest"] == s0["tree_kernel_src_digest"] and s0["git_commit"]
