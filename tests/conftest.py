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
    _install_native_backtrace()
    return lib


def _install_native_backtrace():
    """On a host segfault, print the native frames before faulthandler's
    Python ones (tests/native/segv_bt.c, built into /tmp on first use)."""
    import ctypes
    import subprocess
    import tempfile

    src = ROOT / "tests" / "native" / "segv_bt.c"
    out = Path(tempfile.gettempdir()) / f"cfd_segv_bt_{os.getpid()}.so"
    try:
        subprocess.run(["gcc", "-shared", "-fPIC", "-O1", "-o", str(out), str(src)], check=True,
                       capture_output=True, timeout=60)
        ctypes.CDLL(str(out)).segv_bt_install()
    except (OSError, subprocess.SubprocessError):
        pass  # a diagnostic aid only
