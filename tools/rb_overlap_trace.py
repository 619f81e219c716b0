#!/usr/bin/env python3
"""Workload for the RB-SOR slab-overlap trace: an
in-process group of RANKS Z-slab contexts on one device runs ITERS RB-SOR
iterations of the one-pass slab form (relax_two_pass 0) on an NX x NY x NZ
grid; run it under
  rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d DIR -- python3 tools/rb_overlap_trace.py
and summarise with tools/overlap_summary.py. With CFD_HIP_RB_SPLIT=1 (default)
each iteration is k_rb_edge_r -> [R halo on the side stream || k_rb1 interior
part 1] -> k_rb1 edge planes -> [Y halo on the side stream || k_rb1 interior
part 2]; the trace shows whether the halo copies run during the interior
launches. Two ranks by default, so each of the four streams gets its own
hardware queue (GPU_MAX_HW_QUEUES is 4 on the box)."""
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from cfd_amd import _abi as A  # noqa: E402
from cfd_amd import _native, api  # noqa: E402


def main():
    nx, ny, nz = (int(os.environ.get(k, d)) for k, d in (("NX", "1024"), ("NY", "1024"),
                                                          ("NZ", "130")))
    nranks = int(os.environ.get("RANKS", "2"))
    iters = int(os.environ.get("ITERS", "20"))
    d = 1.0 / (nx - 1)
    group = api.LocalGroup(nranks)
    ctx = [api.HipProjection(nx, ny, nz, comm=group.comm(r, 0), relax_two_pass=0)
           for r in range(nranks)]
    prm = _native.host().poisson_solver_params_default()
    prm.max_iterations, prm.tolerance, prm.absolute_tolerance = iters, 0.0, 0.0

    def body(r):
        c = ctx[r]
        x = np.zeros(c.shape)
        k = np.arange(c.k_offset, c.k_offset + c.nz_local)[:, None, None]
        rhs = np.cos(np.linspace(0, 3, nx))[None, None, :] * np.cos(0.01 * k) + 0 * x
        s, st = c.poisson_solve(A.HIP_POISSON_REDBLACK, x, rhs, d, d, d, prm)
        return s, st.iterations

    out = api.run_ranks(body, nranks)
    for c in ctx:
        c.close()
    group.close()
    print({"grid": [nx, ny, nz], "ranks": nranks, "result": out,
           "split": os.environ.get("CFD_HIP_RB_SPLIT", "1")}, flush=True)


if __name__ == "__main__":
    main()
