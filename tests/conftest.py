import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libeonhip.so)")
    config.addinivalue_line("markers", "slow: larger sizes")


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def gpu_ctx():
    if not gpu_available():
        pytest.skip("no GPU")
    from plonky3_eon_amd import Context

    return Context(0)
