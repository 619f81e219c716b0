#!/usr/bin/env python3
"""BASELINE configs[4] on one device: natural convection (Boussinesq energy
equation coupled) on [0,1] x [0,1] x [0,0.5], 1024 x 1024 x 512 by default,
projection_hip with the Red-Black SOR pressure solve, fields resident in HBM.
Setup restates tests/validation/test_natural_convection.c (:50-61 constants,
:145-154 alpha / nu / dt, hot x = 0 and cold x = 1 Dirichlet walls, Neumann
elsewhere, no-slip velocity, linear initial T). Prints one JSON line: step
time, RB-SOR iterations per step, MLUPS, and the RB-SOR sweeps' algorithmic
GB/s (24 B/cell per iteration)."""
import json
import math
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from cfd_amd import _abi as A  # noqa: E402
from cfd_amd import _native, api  # noqa: E402


def main():
    nx = int(os.environ.get("NX", "1024"))
    nz = int(os.environ.get("NZ", str(nx // 2)))
    steps = int(os.environ.get("STEPS", "2"))
    maxit = int(os.environ.get("MAXIT", "20000"))
    Ra, Pr, beta, grav, dT, T_hot, T_cold, T_ref = 1e3, 0.71, 0.003333, 9.81, 20.0, 310.0, 290.0, 300.0
    nu_alpha = grav * beta * dT / Ra
    alpha = math.sqrt(nu_alpha / Pr)
    nu = Pr * alpha
    g = api.Grid(nx, nx, nz, 0.0, 1.0, 0.0, 1.0, 0.0, 0.5)
    dx = 1.0 / (nx - 1)
    dt = 0.5 * dx * dx / (2.0 * alpha * 3.0)  # below the thermal limit (:150-154)
    p = api.params_default()
    p.dt, p.mu, p.alpha, p.beta, p.T_ref = dt, nu, alpha, beta, T_ref
    p.gravity[0], p.gravity[1], p.gravity[2] = 0.0, -grav, 0.0
    p.source_amplitude_u = p.source_amplitude_v = 0.0
    tb = p.thermal_bc
    tb.left = tb.right = A.BC_TYPE_DIRICHLET
    tb.top = tb.bottom = tb.front = tb.back = A.BC_TYPE_NEUMANN
    tb.dirichlet_values.left, tb.dirichlet_values.right = T_hot, T_cold
    mode = int(os.environ.get("RELAX_MODE", "0"))  # hip_proj_config_t.relax_two_pass
    ctx = api.HipProjection(nx, nx, nz, poisson_method=A.HIP_POISSON_REDBLACK,
                             poisson_max_iter=maxit, relax_two_pass=mode)
    for fid in (A.HIP_FIELD_U, A.HIP_FIELD_V, A.HIP_FIELD_W, A.HIP_FIELD_P):
        ctx.fill(fid, 0.0)
    x = np.asarray(g.x)
    ctx.set_field(A.HIP_FIELD_T, np.broadcast_to((T_hot - dT * x)[None, None, :], (nz, nx, nx)))
    ctx.set_density(1.0)
    for fid in (A.HIP_FIELD_U, A.HIP_FIELD_V, A.HIP_FIELD_W):
        ctx.apply_dirichlet(fid, api.dirichlet())
    ctx.synchronize()
    ctx.reset_timing()
    ctx.enable_timing(True)
    its, t0 = [], time.perf_counter()
    for _ in range(steps):
        s = ctx.step_device(g, p)
        if s != A.CFD_SUCCESS:
            raise SystemExit(f"step failed {s}: {_native.last_error()}")
        its.append(ctx.poisson_stats().iterations)
    ctx.synchronize()
    el = time.perf_counter() - t0
    kt = ctx.timing()
    ctx.close()
    cells = (nx - 2) ** 2 * (nz - 2)
    rms, rn = kt["relax"]
    iters = sum(its)
    rb_iter_ms = rms / iters if iters else None   # red + black sweeps per iteration
    print(json.dumps({
        "workload": f"{nx}x{nx}x{nz} natural convection Ra=1e3, projection_hip RB-SOR, 1 GPU",
        "relax_mode": mode,
        "steps": steps, "rbsor_iters_per_step": its, "ms_per_step": round(el / steps * 1e3, 1),
        "MLUPS": round(cells * steps / el / 1e6, 3),
        "rbsor_iter_ms": round(rb_iter_ms, 4) if rb_iter_ms else None,
        "rbsor_GBps_24B": round(24 * cells / (rb_iter_ms * 1e-3) / 1e9, 1) if rb_iter_ms else None,
        "energy_ms": round(kt["energy"][0] / max(1, kt["energy"][1]), 3)}), flush=True)


if __name__ == "__main__":
    main()
