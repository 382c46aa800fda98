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


# Order of the GPU suite.  The driver runs `pytest -x`, so a failure hides every later test:
# the BASELINE-config parity tests and the hot-path fixtures go first, the tests that start
# subprocesses (bench under torch.distributed.run, the C multi-GPU driver, native drop-in
# builds, env-switch reruns) last.  Within a group the file order stays.
_FIRST = (
    "test_baseline_config0_640x480_420_single_frame",  # BASELINE configs[0]
    "test_full_size_synthetic_vs_oracle",              # configs[1], [2], [4] sizes
    "test_decode_frame_golden_640x480",                # the reference's own 640x480 stream
    "test_stream_decode_baseline_sizes",               # I/P streams at BASELINE sizes
    "test_idct_blocks_fixtures",
    "test_decode_wrap_regime",
    "test_idct_width_test_mixed_waves",
    "test_decode_width_test_mixed_waves",
    "test_decode_frame_vs_oracle",
    "test_reference_idct_symbol",
    "test_reference_idct_symbol_deferred",
    "test_reference_ycbcr_to_rgb_symbol",
    "test_dropin_deferred_frame_loop",
    "test_accelerator_api_golden",
    "test_accelerator_rejects_bad_submissions",
    "test_accel_csc_buffer",
)
_LAST_FILES = ("test_gpu_multi.py", "test_gpu_switches.py")
_LAST_TESTS = ("test_native_dropin_builds_match_reference_bmps",)


def pytest_collection_modifyitems(config, items):
    def key(it):
        name = it.name.split("[")[0]
        fname = os.path.basename(str(it.fspath))
        if name in _FIRST:
            return (0, _FIRST.index(name))
        if fname in _LAST_FILES or name in _LAST_TESTS:
            return (2, 0)
        return (1, 0)
    items[:] = sorted(items, key=key)  # stable: file order kept inside each group


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
