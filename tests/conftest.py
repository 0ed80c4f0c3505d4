import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))

import amd_pkg  # noqa: E402

amd_pkg.load()

GOLDEN = ROOT / "tests" / "golden"
REFERENCE = Path("/root/reference")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device) and the built library")
    config.addinivalue_line("markers", "slow: long-running CPU oracle comparison")


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    return torch.device("cuda", 0)


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
