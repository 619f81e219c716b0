#!/usr/bin/env python3
"""Does the march's speed depend on where the allocator put the fields?
Creates COUNT single-reduction contexts at N^3 one after another in ONE
process, keeping every earlier one alive (so each gets other physical
pages), and times ITERS fixed CG iterations (x0 = 0, cos RHS) on each, twice.
A spread between contexts that repeats within a context is placement, not
noise. One JSON line per context, then a summary line.

usage: N=512 COUNT=6 ITERS=60 python tools/alloc_lottery.py
"""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from cfd_amd import api  # noqa: E402
from tests import cases  # noqa: E402


def relax_lottery(n, count, iters):
    """METHOD=rbsor: the same for the RB-SOR solve (k_rb2 sweeps: X, rhs
    in, the iterate out), per-iteration kernel time from the context's
    relaxation timers."""
    from cfd_amd import _abi as A
    rhs = np.zeros((n, n, n))
    rhs[1:-1, 1:-1, 1:-1] = np.cos(np.linspace(0, 3, n - 2))[None, None, :]
    rhs -= rhs[1:-1, 1:-1, 1:-1].mean() * (rhs != 0)
    d = 1.0 / (n - 1)
    keep, res = [], []
    for k in range(count):
        c = api.HipProjection(n, n, n, poisson_method=A.HIP_POISSON_REDBLACK)
        keep.append(c)
        x = np.zeros((n, n, n))
        c.poisson_solve(A.HIP_POISSON_REDBLACK, x, rhs, d, d, d,
                        A.PoissonParams(0.0, 0.0, 3, 0.0, 1, False, 0))
        t = []
        for _ in range(2):
            x[...] = 0.0
            c.reset_timing()
            c.enable_timing(True)
            c.poisson_solve(A.HIP_POISSON_REDBLACK, x, rhs, d, d, d,
                            A.PoissonParams(0.0, 0.0, iters, 0.0, 1, False, 0))
            kt = c.timing()
            c.enable_timing(False)
            t.append((kt["relax"][0] + kt["relax2"][0] + kt["residual"][0]) / iters)
        res.append(t)
        print(json.dumps({"run": "alloc_lottery", "method": "rbsor", "context": k,
                          "grid": [n, n, n], "ms_per_iter": [round(v, 4) for v in t]}), flush=True)
    return keep, res


def main():
    n = int(os.environ.get("N", "512"))
    count = int(os.environ.get("COUNT", "6"))
    iters = int(os.environ.get("ITERS", "60"))
    cgv = int(os.environ.get("CG_VARIANT", "1"))
    if os.environ.get("METHOD") == "rbsor":
        keep, res = relax_lottery(n, count, iters)
        flat = [min(t) for t in res]
        print(json.dumps({"run": "alloc_lottery_summary", "method": "rbsor",
                          "min": round(min(flat), 4), "max": round(max(flat), 4),
                          "spread": round(max(flat) / min(flat) - 1, 4)}), flush=True)
        for c in keep:
            c.close()
        return
    g, rhs = cases.cos_rhs(n, n)
    rhs = np.ascontiguousarray(rhs)
    keep = []
    res = []
    for k in range(count):
        c = api.HipProjection(n, n, n, cg_variant=cgv)
        keep.append(c)
        c.cg_fixed_iters(rhs, g.dx, g.dy, g.dz, 8)  # warm-up
        t = [c.cg_fixed_iters(rhs, g.dx, g.dy, g.dz, iters) / iters for _ in range(2)]
        res.append(t)
        print(json.dumps({"run": "alloc_lottery", "context": k, "grid": [n, n, n],
                          "cg_variant": cgv, "ms_per_iter": [round(v, 4) for v in t]}),
              flush=True)
    flat = [min(t) for t in res]
    print(json.dumps({"run": "alloc_lottery_summary", "min": round(min(flat), 4),
                      "max": round(max(flat), 4), "spread": round(max(flat) / min(flat) - 1, 4),
                      "within_context_max_diff": round(max(abs(a - b) / min(a, b) for a, b in res), 4)}),
          flush=True)
    for c in keep:
        c.close()


if __name__ == "__main__":
    main()
