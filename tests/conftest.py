"""Shared test plumbing.

Markers: `gpu` tests need a real MI355X (run with `-m gpu`); everything else runs
on CPU.  The product binding (mjpeg423-video-decoder-software_amd/mj423.py) and
the checker (oracle/oracle.py) are put on sys.path here.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

try:  # load torch's HIP runtime before libmj423gpu.so (see mj423.lib())
    import torch  # noqa: F401
except ImportError:
    torch = None

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "mjpeg423-video-decoder-software_amd")
ORACLE = os.path.join(REPO, "oracle")
GOLDEN = os.path.join(REPO, "tests", "golden")
TOOLS = os.path.join(REPO, "tools")
for p in (PKG, ORACLE, REPO, TOOLS):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); run with -m gpu")


def _ensure_built():
    """Build the oracle and the product library in-tree if they are missing (build container)."""
    if not os.path.exists(os.path.join(ORACLE, "build", "liboracle.so")):
        subprocess.run(["make", "-C", ORACLE], check=True, capture_output=True)
    if not os.path.exists(os.path.join(PKG, "libmj423gpu.so")):
        subprocess.run(["make", "-C", PKG, "-j8"], check=True, capture_output=True)


_ensure_built()


def load_golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def manifest():
    import json
    with open(os.path.join(GOLDEN, "manifest.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def orc():
    import oracle
    return oracle


@pytest.fixture(scope="session")
def gpu_ctx():
    """One product context for the whole GPU session (single process on the card)."""
    import mj423
    ctx = mj423.Context(0)
    yield ctx
    ctx.close()
