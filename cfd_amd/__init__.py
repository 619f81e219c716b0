"""cfd_amd -- MI355X-native (HIP/gfx950) Chorin projection step for shaia/CFD.

The product is the in-tree shared library cfd_amd/lib/libcfd_hip.so (HIP
kernels + the C-ABI of include/cfd_hip/projection_hip.h + the
`projection_hip` solver plugin). This package is the Python-side mirror of the
reference's plugin interface (cfd_amd.api) plus the library loader.
"""
from . import _abi as abi  # noqa: F401
from . import api  # noqa: F401
from ._native import build  # noqa: F401

__all__ = ["abi", "api", "build"]
