"""Shared test setup: import paths, the `gpu` marker, common fixtures.

`-m "not gpu"` tests run on CPU only (oracle vs golden vectors, host logic,
C-ABI exports, multi-process gloo paths). `-m gpu` tests are the parity
tests proper: they call the HIP path through the C-ABI (librtx.so) and
check it against the oracle.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "raytrace-we-gpu_amd"), os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and librtx.so")


@pytest.fixture(scope="session")
def oracle():
    import oracle as orc
    orc.lib()
    return orc


@pytest.fixture(scope="session")
def rtx():
    import rtx as r
    r.load_library()
    return r


@pytest.fixture(scope="session")
def gpu_ctx(rtx):
    """One HIP context for the whole GPU session (tests run in one process)."""
    if rtx.device_count() < 1:
        pytest.fail("no HIP device visible: the gpu tests need an MI355X")
    ctx = rtx.Context(0)
    yield ctx
    ctx.close()
