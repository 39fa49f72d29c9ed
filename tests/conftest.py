import os
import sys

import pytest

# torch first: it bundles its own HIP runtime with the same soname as
# /opt/rocm's (libamdhip64.so.7), and whichever loads first serves the whole
# process.  The bench imports torch before libkano_hip.so; so do the tests
# (the shard tests use torch for device buffers, as the bench does for RCCL).
try:
    import torch  # noqa: F401
except ImportError:   # pragma: no cover
    torch = None

ROOT =os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "kubernetes-verification_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and libkano_hip.so")
    config.addinivalue_line("markers", "slow: larger CPU oracle runs")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
