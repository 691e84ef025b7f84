"""Shared pytest setup: the `gpu` marker, repo paths, and loaders for the oracle / product."""
import os
import sys

import pytest

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
