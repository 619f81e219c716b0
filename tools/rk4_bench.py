#!/usr/bin/env python3
"""RK4 step cost at n^3 (hip_rk4_step_device on HBM-resident fields):
per-stage kernel time and GB/s against the stage's algorithmic bytes
(reads u,v,w,p (stencil), rho, the stage base q0 x4 and the
running sum x4, writes the sum x4 and the stage state x4; 8 B each)."""
import ctypes as C
import json
import math
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from cfd_amd import _abi as A  # noqa: E402
from cfd_amd import _native, api  # noqa: E402


def main():
    n = int(os.environ.get("N", "512"))
    steps = int(os.environ.get("STEPS", "5"))
    L = 2.0 * math.pi
    g = api.Grid(n, n, n, 0.0, L, 0.0, L, 0.0, L)
    x = np.asarray(g.x)
    ctx = api.HipProjection(n, n, n)
    u = np.cos(x)[None, None, :] * np.sin(x)[None, :, None] * np.cos(x)[:, None, None]
    ctx.set_field(A.HIP_FIELD_U, u)
    ctx.set_field(A.HIP_FIELD_V, -np.transpose(u, (0, 2, 1)))
    ctx.fill(A.HIP_FIELD_W, 0.0)
    ctx.fill(A.HIP_FIELD_P, 0.0)
    ctx.set_field(A.HIP_FIELD_RHO, np.ones((n, n, n)))
    prm = api.validation_params(1e-4, 0.01)
    lib = _native.hip()
    st = A.SolverStats()
    assert lib.hip_rk4_step_device(ctx.ctx, g.ptr, C.byref(prm), C.byref(st)) == 0
    ctx.reset_timing()
    ctx.enable_timing(True)
    for _ in range(steps):
        assert lib.hip_rk4_step_device(ctx.ctx, g.ptr, C.byref(prm), C.byref(st)) == 0
    kt = ctx.timing()
    ctx.enable_timing(False)
    ctx.close()
    ms, cnt = kt["rk_stage"]
    cells = (n - 2) ** 3
    stage_ms = ms / cnt
    print(json.dumps({"n": n, "stage_ms": round(stage_ms, 4), "stages": cnt,
                      "GBps_at_168B": round(168 * cells / (stage_ms * 1e-3) / 1e9, 1),
                      "max_velocity": st.max_velocity}), flush=True)


if __name__ == "__main__":
    main()
