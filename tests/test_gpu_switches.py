"""GPU: the stream kernel's A/B switches keep every frame bit-exact.

Each switch is read once per process, so every case runs bench.py in a child process with the
switch set and checks its `parity_verified` (every decoded frame against the oracle).  The
ranges start mid-GOP (`--frame0`), so the first segment continues from `state_in`.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import PKG

pytestmark = pytest.mark.gpu

CASES = [
    ({"MJ423_GOP_ORDER": "eighths"}, "c2"),
    ({"MJ423_GOP_ORDER": "xcd"}, "c2"),
    ({"MJ423_GOP_JITTER": "1"}, "c2"),
    ({"MJ423_GOP_STATIC": "0"}, "c1"),
    ({"MJ423_GOP_ORDER": "xcd", "MJ423_GOP_JITTER": "1"}, "c1"),
    ({"MJ423_GOP_FAIR": "1"}, "c2"),  # priority by frames left forced on a grid of several rounds
    ({"MJ423_GOP_FAIR": "0"}, "c1"),  # ... and off on a one-round grid (default: on there)
    ({"MJ423_GOP_OPT": "0"}, "c5"),  # 4:2:2 with the exact kernel only (default: optimistic + re-run)
    ({"MJ423_GOP_ORDER": "eighths"}, "c5"),  # optimistic 4:2:2 kernel in the other job order
]


@pytest.mark.parametrize("env,config", CASES, ids=["-".join(f"{k[6:]}={v}" for k, v in e.items()) + f"-{c}"
                                                   for e, c in CASES])
def test_stream_switch_keeps_parity(env, config):
    repo = os.path.dirname(PKG)
    cmd = [sys.executable, os.path.join(repo, "bench.py"), "--config", config, "--mode", "stream", "--frames", "40",
           "--frame0", "5", "--gop", "12", "--steps", "2", "--warmup", "1", "--no-cpu", "--verify", "all"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=110, cwd=repo, env=dict(os.environ, **env))
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["parity_verified"] is True and d["parity_frames_checked"] == 40
