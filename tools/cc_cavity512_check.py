#!/usr/bin/env python3
"""The 512^3 cavity trajectory (tests/test_gpu_cavity512.py's driving) with
the single-reduction CG (cg_variant 1) against the textbook-CG oracle
fixture: per step the CG iterations of both, the initial / final residual
and the interior norms' relative deviations. One JSON line per step.

usage: STEPS=25 python tools/cc_cavity512_check.py
"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from cfd_amd import _abi as A  # noqa: E402
from cfd_amd import api  # noqa: E402
from tests.test_gpu_cavity512 import FIDS, _init  # noqa: E402

N = 512


def main():
    rec = json.loads((ROOT / "tests/golden/cavity512_re1000_steps.json").read_text())
    steps = rec["steps"][: int(os.environ.get("STEPS", "25"))]
    g = api.Grid(N, N, N, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0)
    params = api.validation_params(rec["dt"], 1.0 / rec["re"])
    ctx = api.HipProjection(N, N, N, cg_variant=int(os.environ.get("CG_VARIANT", "1")))
    _init(ctx)
    for row in steps:
        st = A.SolverStats()
        s = ctx.step_device(g, params, st)
        ps = ctx.poisson_stats()
        out = {"step": row["step"], "status": s, "iters": ps.iterations, "oracle_iters": row["cg_iters"],
               "res0_rel": abs(ps.initial_residual / row["initial_residual"] - 1),
               "res_rel": abs(ps.final_residual / row["final_residual"] - 1),
               "vmax_rel": abs(st.max_velocity / row["max_velocity"] - 1),
               "pmax_rel": abs(st.max_pressure / row["max_pressure"] - 1)}
        for k, fid in FIDS.items():
            a = torch.from_numpy(ctx.get_field(fid))[1:-1, 1:-1, 1:-1]
            l2 = float(torch.linalg.vector_norm(a))
            ol2 = row["norms"][k][0]
            out[f"{k}_l2_rel"] = abs(l2 - ol2) / ol2
        print(json.dumps(out), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
