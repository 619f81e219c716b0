#!/usr/bin/env python3
"""Per-iteration device time of the two CG variants (hip_proj_config_t.cg_variant
0 = textbook, 1 = single-reduction Chronopoulos-Gear) on one GPU, at 512^3 and
on one 8-rank slab's worth of planes (512 x 512 x 66: 64 owned planes + the
two halo planes). Exactly ITERS iterations (tolerance 0), kernel times from the
context's event timers. One JSON line per (shape, variant).

usage: ITERS=100 python tools/cg_variant_bench.py
"""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from cfd_amd import _abi as A  # noqa: E402
from cfd_amd import api  # noqa: E402


def main():
    iters = int(os.environ.get("ITERS", "100"))
    shapes = [(512, 512, 512), (512, 512, 66)]
    if os.environ.get("SHAPES") == "512":  # profiling runs: the cube only
        shapes = shapes[:1]
    elif os.environ.get("SHAPES") == "thin":  # rank 0's slab of 512^3 on 2, 4, 8 ranks
        shapes = [(512, 512, 257), (512, 512, 130), (512, 512, 66)]
    elif os.environ.get("SHAPES") == "slabs":  # rank 0's slab of 512^3 on 1, 2, 4, 8 ranks
        shapes = [(512, 512, 512), (512, 512, 257), (512, 512, 130), (512, 512, 66)]
    elif os.environ.get("SHAPES") == "slab8":  # rank 0's slab of 512^3 on 8 ranks
        shapes = [(512, 512, 66)]
    elif os.environ.get("SHAPES") == "depth":  # 512^2 planes, 64 .. 510 interior planes
        shapes = [(512, 512, 66), (512, 512, 130), (512, 512, 257), (512, 512, 386),
                  (512, 512, 512)]
    elif os.environ.get("SHAPES") == "slab4":  # rank 0's slab of 512^3 on 4 ranks
        shapes = [(512, 512, 130)]
    elif os.environ.get("SHAPES") == "256":  # configs[1]'s grid on one device
        shapes = [(256, 256, 256)]
    variants = [int(v) for v in os.environ.get("VARIANTS", "0,1").split(",")]
    rng = np.random.default_rng(1)
    for nx, ny, nz in shapes:
        rhs = np.zeros((nz, ny, nx))
        rhs[1:-1, 1:-1, 1:-1] = rng.standard_normal((nz - 2, ny - 2, nx - 2))
        h = 1.0 / (nx - 1)
        for variant in variants:
            ctx = api.HipProjection(nx, ny, nz, cg_variant=variant)
            prm = api._native.host().poisson_solver_params_default()
            prm.max_iterations = iters
            prm.tolerance = 0.0
            prm.absolute_tolerance = 0.0
            x = np.zeros_like(rhs)
            ctx.poisson_solve(A.HIP_POISSON_CG, x, rhs, h, h, h, prm)  # warm-up
            ctx.reset_timing()
            ctx.enable_timing(True)
            x[...] = 0.0
            s, st = ctx.poisson_solve(A.HIP_POISSON_CG, x, rhs, h, h, h, prm)
            ctx.enable_timing(False)
            kt = ctx.timing()
            ctx.close()
            per = {k: round(v[0] / st.iterations, 4) for k, v in kt.items() if v[1]}
            loop = sum(v for k, v in per.items() if k != "cg_setup")
            cells = (nx - 2) * (ny - 2) * (nz - 2)
            print(json.dumps({"run": "cg_variant", "grid": [nx, ny, nz], "cg_variant": variant,
                              "iterations": st.iterations, "status": s,
                              "final_residual": st.final_residual,
                              "kernel_ms_per_iter": per,
                              "loop_ms_per_iter": round(loop, 4),
                              "MLUPS_cg_iter": round(cells / (loop * 1e-3) / 1e6, 1)}),
                  flush=True)


if __name__ == "__main__":
    main()
