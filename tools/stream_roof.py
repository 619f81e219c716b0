#!/usr/bin/env python3
"""Measured HBM roof of the GPU: cfd_hip_stream_bench (copy / triad, 16-B
lanes, best over unroll depths) at a few array sizes."""
import ctypes as C
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: E402,F401
from cfd_amd import _native  # noqa: E402

lib = _native.hip()
for n in (1 << 25, 1 << 27, 1 << 28):
    cp, tr = C.c_double(), C.c_double()
    s = lib.cfd_hip_stream_bench(0, n, 5, C.byref(cp), C.byref(tr))
    print(json.dumps({"n": n, "array_MB": n * 8 / 1e6, "status": s,
                      "copy_GBps": round(cp.value, 1), "triad_GBps": round(tr.value, 1)}), flush=True)
