#!/usr/bin/env python3
"""Achievable HBM rate by stream mix (cfd_hip_stream_bench_nm): ni streamed
fp64 inputs and no streamed outputs, 2^27 elements each, one JSON line per
mix. The kernels' roofline fractions are read against the mix they move:
CG sweeps 2/1, predictor 3/3, corrector 4/3, energy 4/1 (+stencil)."""
import ctypes as C
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402,F401

from cfd_amd import _native  # noqa: E402


def main():
    lib = _native.hip()
    for ni, no in ((1, 1), (2, 1), (3, 1), (2, 2), (3, 3), (4, 3), (4, 4), (5, 3)):
        g = C.c_double()
        s = lib.cfd_hip_stream_bench_nm(0, 1 << 27, ni, no, 5, C.byref(g))
        print(json.dumps({"in": ni, "out": no, "status": s, "GBps": round(g.value, 1)}), flush=True)


if __name__ == "__main__":
    main()
