#!/usr/bin/env python3
"""CG sweep timing at 512^3 for several field-base staggers
(CFD_HIP_FIELD_STAGGER, bytes between consecutive field allocations) or,
with --variants, for the sweep memory-hint variants (hip_proj_config_t
sweep_variant)."""
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
    args = sys.argv[1:]
    variants = "--variants" in args
    args = [a for a in args if a != "--variants"]
    staggers = [int(x) for x in (args or (["0", "1", "2", "3"] if variants else
                                          ["0", "256", "4096", "65536", "2097152"]))]
    rhs = np.zeros((n, n, n))
    rhs[1:-1, 1:-1, 1:-1] = np.cos(np.linspace(0, 3, n - 2))[None, None, :]
    d = 1.0 / (n - 1)
    for st in staggers:
        if variants:
            ctx = api.HipProjection(n, n, n, sweep_variant=st)
        else:
            os.environ["CFD_HIP_FIELD_STAGGER"] = str(st)
            ctx = api.HipProjection(n, n, n)
        ctx.cg_fixed_iters(rhs, d, d, d, 10)
        ctx.reset_timing()
        ctx.enable_timing(True)
        ms = ctx.cg_fixed_iters(rhs, d, d, d, 100)
        kt = ctx.timing()
        ctx.enable_timing(False)
        ctx.close()
        a = kt["cg_sweep_a"]
        b = kt["cg_sweep_b"]
        bx = kt["cg_sweep_bx"]
        cells = (n - 2) ** 3
        out = {("variant" if variants else "stagger"): st, "iter_us": round(ms / 100 * 1e3, 1),
               "A_us": round(a[0] / a[1] * 1e3, 1), "B_us": round(b[0] / b[1] * 1e3, 1),
               "BX_us": round(bx[0] / bx[1] * 1e3, 1),
               "A_GBps": round(24 * cells / (a[0] / a[1] * 1e-3) / 1e9, 1),
               "B_GBps": round(24 * cells / (b[0] / b[1] * 1e-3) / 1e9, 1),
               "BX_GBps": round(48 * cells / (bx[0] / bx[1] * 1e-3) / 1e9, 1)}
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
