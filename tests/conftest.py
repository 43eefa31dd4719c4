import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through liborbgpu.so)")


@pytest.fixture(scope="session")
def oracle():
    import oracle_py

    oracle_py.build()
    return oracle_py


def _gpu_available():
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu():
    """Skips cleanly on CPU-only hosts; on a GPU host the HIP library MUST load (no fallback)."""
    if not _gpu_available():
        pytest.skip("no GPU visible")
    import orbslam2_with_quadrics_amd as m
    from orbslam2_with_quadrics_amd import _lib

    _lib.lib()  # raises if liborbgpu.so is missing
    return m
