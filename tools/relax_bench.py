#!/usr/bin/env python3
"""RB-SOR / Jacobi iteration cost at n^3 (hip_proj_poisson_solve, zero
tolerance so exactly ITERS iterations run). Reports per-iteration ms, the
per-kernel split and GB/s against SURVEY.md §8d's 24 B/cell."""
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from cfd_amd import _abi as A  # noqa: E402
from cfd_amd import api  # noqa: E402


def main():
    n = int(os.environ.get("N", "512"))
    nx, ny, nz = (int(os.environ.get(k, str(n))) for k in ("NX", "NY", "NZ"))
    iters = int(os.environ.get("ITERS", "40"))
    methods = os.environ.get("METHODS", "rbsor,jacobi").split(",")
    rhs = np.zeros((nz, ny, nx))
    rhs[1:-1, 1:-1, 1:-1] = np.cos(np.linspace(0, 3, nx - 2))[None, None, :]
    rhs -= rhs[1:-1, 1:-1, 1:-1].mean() * (rhs != 0)
    d = 1.0 / (nx - 1)
    cells = (nx - 2) * (ny - 2) * (nz - 2)
    for name, method in (("rbsor", A.HIP_POISSON_REDBLACK), ("jacobi", A.HIP_POISSON_JACOBI)):
        if name not in methods:
            continue
        ctx = api.HipProjection(nx, ny, nz)
        x = np.zeros((nz, ny, nx))
        prm = A.PoissonParams(0.0, 0.0, 3, 0.0, 1, False, 0)
        ctx.poisson_solve(method, x, rhs, d, d, d, prm)   # warm-up
        prm = A.PoissonParams(0.0, 0.0, iters, 0.0, 1, False, 0)
        ctx.reset_timing()
        ctx.enable_timing(True)
        t0 = time.perf_counter()
        s, st = ctx.poisson_solve(method, x, rhs, d, d, d, prm)
        wall = time.perf_counter() - t0
        kt = ctx.timing()
        ctx.enable_timing(False)
        ctx.close()
        # one-iteration sweeps (k_rb1 / k_rx) and two-iteration sweeps (k_rb2)
        relax = (kt["relax"][0] + kt["relax2"][0], kt["relax"][1] + kt["relax2"][1])
        res = kt["residual"]
        per_it = (relax[0] + res[0]) / iters
        print(json.dumps({"method": name, "grid": [nx, ny, nz], "iters": st.iterations, "status": s,
                          "rb2": os.environ.get("CFD_HIP_RB2"),
                          "sweeps_1it": kt["relax"][1], "sweeps_2it": kt["relax2"][1],
                          "iter_ms_kernels": round(per_it, 4),
                          "relax_ms": round(relax[0] / iters, 4),
                          "residual_ms": round(res[0] / max(res[1], 1), 4),
                          "GBps_24B": round(24 * cells / (per_it * 1e-3) / 1e9, 1),
                          "wall_s_incl_transfers": round(wall, 2)}), flush=True)


if __name__ == "__main__":
    main()
