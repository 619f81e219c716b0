#!/usr/bin/env python3
"""CG sweep timing at n^3 for a list of context configurations.
usage: sweep_bench.py "sweep_rows=8" "sweep_rows=16,kchunk=32" ...
Each configuration runs 100 fixed CG iterations (no early exit) with
dispatch-packet timing; prints per-sweep averages and GB/s (24 / 24 / 64 B/cell)."""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from cfd_amd import api  # noqa: E402


def main():
    n = int(os.environ.get("N", "512"))
    nz = int(os.environ.get("NZ", str(n)))   # NZ = 66: one 8-rank Z-slab of 512^3
    iters = int(os.environ.get("ITERS", "100"))
    rhs = np.zeros((nz, n, n))
    rhs[1:-1, 1:-1, 1:-1] = np.cos(np.linspace(0, 3, n - 2))[None, None, :]
    d = 1.0 / (n - 1)
    cells = (n - 2) ** 2 * (nz - 2)
    for spec in sys.argv[1:] or ["sweep_rows=8"]:
        kw = {}
        for item in filter(None, spec.split(",")):
            k, v = item.split("=")
            kw[k] = int(v)
        ctx = api.HipProjection(n, n, nz, **kw)
        ctx.cg_fixed_iters(rhs, d, d, d, 10)
        ctx.reset_timing()
        ctx.enable_timing(True)
        ms = ctx.cg_fixed_iters(rhs, d, d, d, iters)
        kt = ctx.timing()
        ctx.enable_timing(False)
        ctx.close()
        a, b, bx = kt["cg_sweep_a"], kt["cg_sweep_b"], kt["cg_sweep_bx"]
        ua, ub, ubx = (t[0] / t[1] * 1e3 for t in (a, b, bx))
        print(json.dumps({"cfg": spec, "nz": nz, "iter_us": round(ms / iters * 1e3, 1),
                          "A_us": round(ua, 1), "B_us": round(ub, 1), "BX_us": round(ubx, 1),
                          "A_GBps": round(24 * cells / (ua * 1e-6) / 1e9, 1),
                          "B_GBps": round(24 * cells / (ub * 1e-6) / 1e9, 1),
                          "BX_GBps": round(64 * cells / (ubx * 1e-6) / 1e9, 1)}), flush=True)

if __name__ == "__main__":
    main()
