import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); parity tests proper")
    config.addinivalue_line("markers", "slow: long CPU-oracle runs")


@pytest.fixture(scope="session")
def hip_lib():
    """The HIP product library on a GPU box. Fails (never skips) when the
    device or the library is missing: -m gpu tests must exercise native code."""
    from cfd_amd import _native
    lib = _native.hip()
    assert lib.hip_projection_available() == 1, "no HIP device visible to libcfd_hip.so"
    return lib
