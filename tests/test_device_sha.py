"""cfd_amd._sha.device_code_sha: the device-code identity PMC profiles are
keyed on (bench.pmc_profile). CPU only: reads the built library's bytes."""
import re

import pytest

from cfd_amd import _sha
from cfd_amd._native import HIP_LIB


def test_device_sha_of_built_library():
    if not HIP_LIB.exists():
        pytest.skip("libcfd_hip.so not built")
    d = _sha.device_code_sha(HIP_LIB)
    assert d is not None and re.fullmatch(r"[0-9a-f]{16}", d)
    assert _sha.device_code_sha(HIP_LIB) == d  # a pure function of the file


def test_device_sha_without_device_code(tmp_path):
    f = tmp_path / "plain.bin"
    f.write_bytes(b"not an ELF image")
    assert _sha.device_code_sha(f) is None
