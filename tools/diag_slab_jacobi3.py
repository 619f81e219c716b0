#!/usr/bin/env python3
"""Diagnostic: the in-process 3-rank Jacobi slab test (tests/test_gpu_slabs.py
test_slab_relaxation_projection_bitwise[2-3]) repeated REPEAT times in ONE
process, with the native segfault backtrace installed, to see whether its
intermittent host crash needs a fresh process (first concurrent launches) or
recurs on later runs. usage: REPEAT=12 python tools/diag_slab_jacobi3.py"""
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import faulthandler  # noqa: E402

faulthandler.enable()

import conftest  # noqa: E402
import test_gpu_slabs as T  # noqa: E402
from cfd_amd import _abi as A  # noqa: E402
from cfd_amd import _native  # noqa: E402

lib = _native.hip()
assert lib.hip_projection_available() == 1
conftest._install_native_backtrace()
for i in range(int(os.environ.get("REPEAT", "12"))):
    t0 = time.time()
    T.test_slab_relaxation_projection_bitwise(lib, A.HIP_POISSON_JACOBI, 3)
    print(f"run {i}: ok {time.time() - t0:.1f} s", flush=True)
