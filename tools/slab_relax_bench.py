#!/usr/bin/env python3
"""RB-SOR on Z-slabs of one device (in-process group, every rank's slab on
the same GPU): wall time per iteration of the one-pass form (k_rb_edge_r +
R halo + k_rb1<DIST>, relax_two_pass 0) and the two colour sweeps (k_rx,
relax_two_pass 2). The ranks share the GPU, so the figure is the total
device work of an iteration of the decomposed solve, not a scaling number.
Env: NX NY NZ (global), RANKS, ITERS."""
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
    nx, ny, nz = (int(os.environ.get(k, "512")) for k in ("NX", "NY", "NZ"))
    nranks = int(os.environ.get("RANKS", "4"))
    iters = int(os.environ.get("ITERS", "40"))
    iters2 = 3 * iters  # per-iteration wall = (wall(iters2) - wall(iters)) / (iters2 - iters)
    d = 1.0 / (nx - 1)
    for two_pass in (0, 2, 0, 2):
        group = api.LocalGroup(nranks)
        ctx = [api.HipProjection(nx, ny, nz, comm=group.comm(r, 0), relax_two_pass=two_pass)
               for r in range(nranks)]

        def body(r, prm):
            c = ctx[r]
            x = np.zeros(c.shape)
            k = np.arange(c.k_offset, c.k_offset + c.nz_local)[:, None, None]
            rhs = np.cos(np.linspace(0, 3, nx))[None, None, :] * np.cos(0.01 * k) + 0 * x
            t0 = time.perf_counter()
            s, st = c.poisson_solve(A.HIP_POISSON_REDBLACK, x, rhs, d, d, d, prm)
            return time.perf_counter() - t0, st.iterations

        api.run_ranks(lambda r: body(r, A.PoissonParams(0.0, 0.0, 3, 0.0, 1, False, 0)), nranks)
        for c in ctx:
            c.reset_timing()
            c.enable_timing(True)
        res = api.run_ranks(lambda r: body(r, A.PoissonParams(0.0, 0.0, iters, 0.0, 1, False, 0)),
                            nranks)
        kt = [c.timing()["relax"] for c in ctx]
        res2 = api.run_ranks(
            lambda r: body(r, A.PoissonParams(0.0, 0.0, iters2, 0.0, 1, False, 0)), nranks)
        for c in ctx:
            c.close()
        group.close()
        wall = max(t for t, _ in res)
        print(json.dumps({"grid": [nx, ny, nz], "ranks": nranks, "relax_two_pass": two_pass,
                          "iters": res[0][1], "wall_s_incl_transfers": round(wall, 3),
                          "wall_ms_per_iter": round(
                              (max(t for t, _ in res2) - wall) / (iters2 - iters) * 1e3, 4),
                          "relax_kernel_ms_per_iter_sum_ranks":
                              round(sum(k[0] for k in kt) / iters, 4)}), flush=True)


if __name__ == "__main__":
    main()
