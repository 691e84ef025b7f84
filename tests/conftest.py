"""Shared pytest setup: the `gpu` marker, repo paths, and loaders for the oracle / product."""
import os
import sys

import pytest

# Under pytest-xdist every worker would start a full OpenMP team for the C oracle: 8 workers x 8
# spinning threads on 8 cores turns a 1 s oracle test into ~10 min.  One worker = one thread.
if os.environ.get("PYTEST_XDIST_WORKER") and "OMP_NUM_THREADS" not in os.environ:
    os.environ["OMP_NUM_THREADS"] = "1"

try:  # torch first: libnkhip.so must bind the same HIP runtime torch uses (user residuals run torch code)
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    torch = None

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libnkhip.so on the GPU box)")


@pytest.fixture(scope="session")
def golden_dir():
    return os.path.join(ROOT, "tests", "golden")
