#!/usr/bin/env python3
"""configs[0]-sized cavity steps (N x N x 1, Re = 1000, dt = 5e-4, device
resident) with the persistent small-grid CG (k_cg_small) and with the sweep
kernels (CFD_HIP_CG_SMALL = 0 / 1): ms per step, CG iterations, us per CG
iteration. Env: N (128), STEPS (300), also NZ for a 3-D N^2 x NZ grid."""
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402,F401

from cfd_amd import _abi as A  # noqa: E402
from cfd_amd import api  # noqa: E402


def run(n, nz, steps, small):
    small = bool(small)
    os.environ["CFD_HIP_CG_SMALL"] = "1" if small else "0"
    g = api.Grid(n, n, nz, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0 if nz > 1 else 0.0)
    prm = api.validation_params(5e-4, 1e-3)
    c = api.HipProjection(n, n, nz, kchunk=int(os.environ.get("KCHUNK", "0")))
    for fid in (A.HIP_FIELD_U, A.HIP_FIELD_V, A.HIP_FIELD_W, A.HIP_FIELD_P):
        c.fill(fid, 0.0)
    c.set_density(1.0)
    c.apply_dirichlet(A.HIP_FIELD_U, api.dirichlet(top=1.0))
    c.apply_dirichlet(A.HIP_FIELD_V, api.dirichlet())
    c.apply_dirichlet(A.HIP_FIELD_W, api.dirichlet())
    c.apply_scalar_bc(A.HIP_FIELD_P, A.BC_TYPE_NEUMANN)
    for _ in range(20):
        assert c.step_device(g, prm) == A.CFD_SUCCESS
    c.synchronize()
    its = 0
    t0 = time.perf_counter()
    for _ in range(steps):
        assert c.step_device(g, prm) == A.CFD_SUCCESS
        its += c.poisson_stats().iterations
    c.synchronize()
    dt = time.perf_counter() - t0
    c.close()
    return {"grid": [n, n, nz], "small_cg": small, "kchunk": int(os.environ.get("KCHUNK", "0")),
            "steps": steps,
            "ms_per_step": round(dt / steps * 1e3, 4), "cg_iters_per_step": its / steps,
            "us_per_cg_iter": round(dt / its * 1e6, 3)}


def main():
    n = int(os.environ.get("N", "128"))
    nz = int(os.environ.get("NZ", "1"))
    steps = int(os.environ.get("STEPS", "300"))
    modes = [int(m) for m in os.environ.get("MODES", "0,1,0,1").split(",")]
    for small in modes:
        print(json.dumps(run(n, nz, steps, small)), flush=True)


if __name__ == "__main__":
    main()
