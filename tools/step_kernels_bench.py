#!/usr/bin/env python3
"""Per-kernel times of the non-CG phases of the projection step (predictor,
CG setup with the fused divergence, corrector) on the 512^3 cavity, with the algorithmic bandwidth of each
(48 / 40 / 56 B per interior cell)."""
import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import torch  # noqa: E402,F401

from cfd_amd import _abi as A  # noqa: E402
from cfd_amd import api  # noqa: E402

BYTES = {"predictor": 48.0, "cg_setup": 40.0, "corrector": 56.0}


def main():
    n = int(os.environ.get("N", "512"))
    steps = int(os.environ.get("STEPS", "3"))
    g = api.Grid(n, n, n, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0)
    prm = api.validation_params(1e-4, 1e-3)
    ctx = api.HipProjection(n, n, n)
    for fid in (A.HIP_FIELD_U, A.HIP_FIELD_V, A.HIP_FIELD_W, A.HIP_FIELD_P):
        ctx.fill(fid, 0.0)
    ctx.set_density(1.0)
    ctx.apply_dirichlet(A.HIP_FIELD_U, api.dirichlet(top=1.0))
    assert ctx.step_device(g, prm) == A.CFD_SUCCESS
    cells = (n - 2) ** 3
    for v in ("default",):
        ctx.reset_timing()
        ctx.enable_timing(True)
        for _ in range(steps):
            assert ctx.step_device(g, prm) == A.CFD_SUCCESS
        kt = ctx.timing()
        ctx.enable_timing(False)
        out = {"variant": v, "n": n, "steps": steps}
        for k, b in BYTES.items():
            ms, cnt = kt[k]
            if cnt:
                avg = ms / cnt
                out[k] = {"avg_ms": round(avg, 4),
                          "GBps": round(b * cells / (avg * 1e-3) / 1e9, 1)}
        print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
