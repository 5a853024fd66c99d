"""Shared test configuration.

Markers: ``gpu`` — needs an MI355X (run with ``-m gpu``); everything else runs on CPU.
The oracle (``/root/repo/oracle``) is importable from tests only.
"""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (ROOT, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
