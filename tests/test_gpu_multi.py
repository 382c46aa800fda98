"""GPU: the multi-GPU group of the C ABI (include/mj423gpu.h section 5) and its plain-C
driver (csrc/apps/mj423_multigpu.c), checked frame by frame against the oracle.

On the one-GPU test box the RCCL group has one rank (ncclCommInitAll over every visible
device, so the same test covers 8 ranks on an 8-GPU node); the sharding itself is
exercised with MJ423_MULTI_NO_COMM groups that put several ranks on device 0 (RCCL refuses
two ranks on one GPU).  Bit-exact, zero tolerance.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLDEN, PKG

pytestmark = pytest.mark.gpu

DRIVER = os.path.join(PKG, "mj423_multigpu")


def _ndev():
    import torch
    return torch.cuda.device_count()


def _custom_tables():
    yq = (np.arange(64) % 13 + 3).astype(np.int16)
    cq = (np.arange(64)[::-1] % 11 + 5).astype(np.int16)
    return yq, cq


def test_rccl_group_spans_every_device_and_broadcasts_tables(orc):
    """ncclCommInitAll over all visible GPUs; rank 0's tables reach every rank by ncclBroadcast
    and decode with them matches the oracle given the same tables."""
    import mj423
    n = _ndev()
    with mj423.Multi(0) as g:
        assert g.size == n
        assert g.comm_ranks() == n
        yq, cq = _custom_tables()
        g.set_quant(yq, cq)
        for r in range(n):
            gy, gc = g.get_quant(r)
            assert np.array_equal(gy, yq) and np.array_equal(gc, cq), r
        w, h, chroma, nf = 48, 32, 420, 2 * n + 1
        rng = np.random.default_rng(77)
        coef = orc.random_quantized_planes(rng, w, h, chroma, nframes=nf)
        got = g.decode_frames(coef, nf, w, h, chroma)
        geo = orc.geometry(w, h, chroma)
        for f in range(nf):
            c = coef[f]
            Y, Cb, Cr = c[:geo.y_blocks], c[geo.y_blocks:geo.y_blocks + geo.c_blocks], c[geo.y_blocks + geo.c_blocks:]
            exp = orc.decode_frame(Y, Cb, Cr, w, h, chroma, yquant=yq, cquant=cq)
            assert np.array_equal(got[f], exp), f
        g.set_quant()  # NULL: back to the reference's tables on every rank
        assert np.array_equal(g.get_quant(n - 1)[0], orc.YQUANT)


def test_duplicate_device_needs_no_comm():
    import mj423
    with pytest.raises(mj423.Mj423Error) as e:
        mj423.Multi(devices=[0, 0])
    assert "appears twice" in str(e.value)
    with pytest.raises(mj423.Mj423Error):
        mj423.Multi(devices=[_ndev()])  # not visible


@pytest.mark.parametrize("ranks,nf", [(3, 7), (4, 3), (2, 1), (5, 0)])
def test_sharded_host_decode_matches_oracle(orc, ranks, nf):
    """Frame ranges of 7 over 3 ranks (3+2+2), fewer frames than ranks (idle ranks), empty job."""
    import mj423
    w, h, chroma = 40, 24, 422
    rng = np.random.default_rng(ranks * 100 + nf)
    coef = orc.random_quantized_planes(rng, w, h, chroma, nframes=max(nf, 1))
    with mj423.Multi(devices=[0] * ranks, flags=mj423.MULTI_NO_COMM) as g:
        assert g.comm_ranks() == 0
        got = g.decode_frames(coef, nf, w, h, chroma)
    assert got.shape == (nf, h, w)
    if nf:
        assert np.array_equal(got, orc.decode_frames_mt(coef[:nf], nf, w, h, chroma, nthreads=4))


def test_device_resident_shards_timed_and_exact(orc):
    """Each rank generates its own range of the global synthetic stream on its device, the
    group times start-aligned decode steps, and the union of the shards equals the oracle's
    decode of the whole stream (generated in one piece)."""
    import mj423
    import torch
    w, h, chroma, total, ranks = 256, 144, 420, 9, 3
    geo = mj423.geometry(w, h, chroma)
    with mj423.Multi(devices=[0] * ranks, flags=mj423.MULTI_NO_COMM) as g:
        rng_ = [mj423.frame_range(r, ranks, total) for r in range(ranks)]
        coefs = [torch.empty(max(c, 1) * geo.coef_per_frame, dtype=torch.int16, device="cuda:0") for _, c in rng_]
        outs = [torch.empty(max(c, 1) * w * h, dtype=torch.int32, device="cuda:0") for _, c in rng_]
        cp, op = [t.data_ptr() for t in coefs], [t.data_ptr() for t in outs]
        g.synth_frames_device(cp, [f for f, _ in rng_], [c for _, c in rng_], w, h, chroma, seed=4321)
        mx, per, wall = g.time_decode(cp, op, [c for _, c in rng_], w, h, chroma, steps=3)
        assert mx > 0 and len(per) == ranks and max(per) == pytest.approx(mx) and wall >= mx * 0.5
        g.synchronize()
        got = np.concatenate([o.view(-1)[:c * w * h].cpu().numpy().view(np.uint32).reshape(c, h, w)
                              for o, (_, c) in zip(outs, rng_)])
        # the same frames generated in one piece by one context
        whole = torch.empty(total * geo.coef_per_frame, dtype=torch.int16, device="cuda:0")
        ctx = g.ctx(0)
        ctx.synth_frames_device(whole.data_ptr(), w, h, chroma, total, 0, 4321)
        ctx.synchronize()
        c = whole.cpu().numpy()
        shard_c = np.concatenate([t.view(-1)[:n * geo.coef_per_frame].cpu().numpy() for t, (_, n) in zip(coefs, rng_)])
        assert np.array_equal(shard_c, c)
    assert np.array_equal(got, orc.decode_frames_mt(c, total, w, h, chroma, nthreads=8))


def _driver(*args, timeout=120):
    r = subprocess.run([DRIVER, *args], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr
    return json.loads(r.stdout.strip().splitlines()[-1])


def _oracle_hashes(orc, w, h, chroma, first, n, seed):
    import mj423
    import torch
    geo = mj423.geometry(w, h, chroma)
    with mj423.Context(0) as ctx:
        t = torch.empty(n * geo.coef_per_frame, dtype=torch.int16, device="cuda:0")
        ctx.synth_frames_device(t.data_ptr(), w, h, chroma, n, first, seed)
        ctx.synchronize()
        c = t.cpu().numpy()
    exp = orc.decode_frames_mt(c, n, w, h, chroma, nthreads=8)
    return [orc.fnv1a64(exp[i]) for i in range(n)]


def test_c_driver_rccl_all_devices_weak(orc):
    """The plain-C driver: RCCL group over every device, 3 frames per GPU (weak scaling)."""
    n = _ndev()
    d = _driver("--width", "96", "--height", "64", "--chroma", "420", "--frames-per-gpu", "3", "--steps", "2",
                "--warmup", "1", "--seed", "99", "--hashes")
    assert d["ranks"] == n and d["comm_ranks"] == n and d["total_frames"] == 3 * n and d["scaling"] == "weak"
    assert d["hashes"] == _oracle_hashes(orc, 96, 64, 420, 0, 3 * n, 99)
    assert all(p["frames"] == 3 for p in d["per_rank"])


def test_c_driver_no_comm_strong_shards(orc):
    """Strong scaling: 7 frames over 3 ranks on device 0 (rehearsal), every frame exact."""
    d = _driver("--no-comm", "--devices", "0,0,0", "--width", "136", "--height", "56", "--chroma", "422",
                "--total-frames", "7", "--steps", "2", "--warmup", "0", "--seed", "5", "--hashes")
    assert d["ranks"] == 3 and d["comm_ranks"] == 0 and d["scaling"] == "strong"
    assert [p["frames"] for p in d["per_rank"]] == [3, 2, 2]
    assert [p["first"] for p in d["per_rank"]] == [0, 3, 5]
    assert d["hashes"] == _oracle_hashes(orc, 136, 56, 422, 0, 7, 5)


@pytest.mark.parametrize("flags,devices,first", [(0, None, 0), (1, [0, 0, 0], 0), (1, [0, 0], 3)])
def test_multi_decode_reference_mpg(tmp_path, manifest, flags, devices, first):
    """The reference encoder's .mpg cut at I-frames over the ranks, entropy decode on each
    rank's GPU: every frame's BMP byte-identical (SHA-256) to the reference decoder's."""
    import hashlib
    import mj423
    import torch
    name = "stream_320x240"
    fx = manifest["fixtures"][name]
    m = mj423.Mpg(os.path.join(GOLDEN, f"{name}.mpg"))
    w, h, n = m.header.width, m.header.height, m.header.num_frames
    with mj423.Multi(0 if devices is None else len(devices), devices=devices, flags=flags) as g:
        ranges = mj423.mpg_gop_ranges(m, first, n - first, g.size)
        devs = devices if devices is not None else list(range(g.size))
        outs = [torch.empty((max(c, 1), h, w), dtype=torch.int32, device=f"cuda:{d}") for (_, c), d in zip(ranges, devs)]
        got_ranges = g.decode_mpg_gpu(m, first, n - first, [o.data_ptr() for o in outs])
        assert got_ranges == ranges
        for (f0, c), o in zip(ranges, outs):
            host = o.cpu().numpy().view(np.uint32)
            for i in range(c):
                p = tmp_path / f"m{f0 + i:04d}.bmp"
                mj423.write_bmp(str(p), host[i])
                assert hashlib.sha256(p.read_bytes()).hexdigest() == fx["decoded_bmp_sha256"][f0 + i], f0 + i


def test_c_driver_mpg_mode(orc, manifest):
    """The C driver's --mpg mode over every device: per-frame hashes equal the oracle's
    decode of the same file (front end + pixels, P-frames accumulated)."""
    import mj423
    path = os.path.join(GOLDEN, "stream_160x96.mpg")
    d = _driver("--mpg", path, "--steps", "2", "--warmup", "1", "--hashes")
    m = mj423.Mpg(path)
    w, h, n = m.header.width, m.header.height, m.header.num_frames
    assert d["frames"] == n and d["ranks"] == _ndev()
    nb = (w // 8) * (h // 8)
    state = [None, None, None]
    import ctypes
    exp = []
    for f in range(n):
        fr = m.frame(f)
        P = fr.frame_type != 0
        for pi, (ptr, size) in enumerate(((fr.y, fr.y_size), (fr.cb, fr.cb_size), (fr.cr, fr.cr_size))):
            bs = np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint8)), shape=(size,))
            state[pi] = orc.lossless_decode_q(nb, np.concatenate([bs, np.zeros(8, np.uint8)]), P,
                                              prev=state[pi] if P else None)
        exp.append(orc.fnv1a64(orc.decode_frame(state[0], state[1], state[2], w, h, 444)))
    assert d["hashes"] == exp


@pytest.mark.parametrize("mode", ["batch", "stream"])
def test_bench_under_launcher_with_rccl_group(mode):
    """bench.py as the driver launches it (torch.distributed.run, one rank per GPU) with an RCCL
    process group even at one rank (MJ423_BENCH_FORCE_DIST=1): the group's start-up, the table
    broadcast and the timing/parity reductions run through RCCL on the device, and every frame
    of the small run is verified against the oracle."""
    import socket
    repo = os.path.dirname(PKG)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, MJ423_BENCH_FORCE_DIST="1")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr=127.0.0.1",
           f"--master-port={port}", os.path.join(repo, "bench.py"), "--gpus", "1", "--config", "c1",
           "--frames", "30", "--steps", "2", "--warmup", "1", "--no-cpu", "--verify", "all", "--mode", mode]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=repo, env=env)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["n_gpus"] == 1
    assert d["distributed"]["backend"] == "nccl" and d["distributed"]["world_size"] == 1
    assert d["distributed"]["rehearsal"] is False
    assert d["parity_verified"] is True and d["parity_frames_checked"] == 30
