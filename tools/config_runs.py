#!/usr/bin/env python3
"""BASELINE configs[0], [1] and [3] run through projection_hip on one device,
fields resident in HBM. One JSON line per run to stdout (and progress lines to
stderr so a long run is visibly alive).

  cavity128  configs[0]: 128x128x1 lid-driven cavity, Re=1000, dt=5e-4,
             100 000 steps (t = 50, test_cavity_backends.c:74-76), cavity BCs
             before every step (lid_driven_cavity_common.h:238-270). Ghia RMS
             (tests/ghia.py) against the oracle's fixture
             tests/golden/cavity128_re1000_t50.json: the reference requires
             RMS < 0.10 (GHIA_RMS_TARGET_PROJECTION, test_cavity_backends.c:50)
             and backends within 0.001 of each other (:43). Takes ~150 s on
             one MI355X (1.5 ms per step with the persistent small-grid CG).
  tg         configs[1]: Taylor-Green 3-D, nu = 0.01, dt = 1e-3, 100 steps,
             periodic BCs before every step (taylor_green_3d_reference.h:177-
             404); relative interior L2 of u, v against the reference's
             "analytic" decay e^{-3 nu t} at n = 32, 64, 128, 256 (SIZES),
             gated by the reference at TG3_L2_ERROR_TOL = 0.25
             (taylor_green_3d_reference.h:58). The 3-D field with w = 0 is not
             an exact Navier-Stokes solution, so the error levels off with n
             (order_u -> 0): it measures the model, not the discretisation.
  tgslabs    configs[3] on one device: 512^3 Taylor-Green (STEPS steps) on 1
             context and on in-process Z-slab groups of 2, 4, 8 ranks (the
             multi-rank driver with device-copy halos); the L2 errors must
             equal the 1-context result within 1e-10 relative.

usage: python tools/config_runs.py cavity128|tg|tgslabs
"""
import json
import math
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401  (one HIP runtime in the process)

from cfd_amd import _abi as A  # noqa: E402
from cfd_amd import _native, api  # noqa: E402
from tests import cases, ghia  # noqa: E402

FIELDS = {"u": A.HIP_FIELD_U, "v": A.HIP_FIELD_V, "w": A.HIP_FIELD_W, "p": A.HIP_FIELD_P}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cavity128():
    steps = int(os.environ.get("STEPS", "100000"))
    g, f, p = cases.cavity(128, 128, 1, Re=1000.0, dt=5e-4)
    api.cavity_bc(f, 1.0)
    ctx = api.HipProjection(128, 128, 1)
    ctx.upload(f)
    its, t0 = [], time.perf_counter()
    for n in range(1, steps + 1):
        # the cavity BCs are constants and the step preserves the boundary
        # faces (as tests/test_gpu_parity.py::test_ghia_33_re100_device_resident)
        s = ctx.step_device(g, p)
        if s != A.CFD_SUCCESS:
            raise RuntimeError(f"step {n}: {s} {_native.last_error()}")
        its.append(ctx.poisson_stats().iterations)
        if n % 10000 == 0:
            log(f"cavity128 step {n} iters {its[-1]} {time.perf_counter() - t0:.1f}s")
    ctx.synchronize()
    wall = time.perf_counter() - t0
    ctx.download(f)
    ctx.close()
    rms_u, rms_v = ghia.rms_errors(f, g, 1000)
    y, uc, x, vc = ghia.centerlines(f.u[0], f.v[0], g.x, g.y)
    out = {"run": "cavity128_re1000", "config": "BASELINE configs[0] on projection_hip",
           "steps": steps, "wall_s": round(wall, 2), "ms_per_step": round(wall / steps * 1e3, 4),
           "cg_iters_total": int(sum(its)), "cg_iters_last": its[-1],
           "rms_u": rms_u, "rms_v": rms_v, "u_centerline": uc, "v_centerline": vc}
    fx = ROOT / "tests" / "golden" / "cavity128_re1000_t50.json"
    if fx.exists() and steps == 100000:
        ref = json.loads(fx.read_text())
        out.update({"oracle_rms_u": ref["rms_u"], "oracle_rms_v": ref["rms_v"],
                    "oracle_cg_iters_total": ref["cg_iters_total"],
                    "d_rms_u": abs(rms_u - ref["rms_u"]), "d_rms_v": abs(rms_v - ref["rms_v"]),
                    "max_centerline_diff": max(
                        float(np.max(np.abs(np.array(uc) - ref["u_centerline"]))),
                        float(np.max(np.abs(np.array(vc) - ref["v_centerline"]))))})
        out["pass"] = bool(rms_u < 0.10 and rms_v < 0.10 and out["d_rms_u"] < 1e-3
                           and out["d_rms_v"] < 1e-3)
    print(json.dumps(out), flush=True)


def tg_run(n, steps, nranks=0):
    """Taylor-Green n^3 for `steps` steps; nranks = 0: one context, else an
    in-process Z-slab group. Returns (L2 u, L2 v, CG iterations, wall s)."""
    g, f, p = cases.tg3(n)
    if nranks:
        group = api.LocalGroup(nranks)
        ctxs = [api.HipProjection(n, n, n, comm=group.comm(r, 0)) for r in range(nranks)]
    else:
        group = None
        ctxs = [api.HipProjection(n, n, n)]
    for c in ctxs:
        sl = slice(c.k_offset, c.k_offset + c.nz_local)
        for k, fid in FIELDS.items():
            c.set_field(fid, getattr(f, k)[sl])
        c.set_density(1.0)
        c.synchronize()

    def body(r, c):
        its = []
        for _ in range(steps):
            for fid in FIELDS.values():
                c.apply_scalar_bc(fid, A.BC_TYPE_PERIODIC)
            s = c.step_device(g, p)
            if s != A.CFD_SUCCESS:
                raise RuntimeError(f"rank {r}: {s} {_native.last_error()}")
            its.append(c.poisson_stats().iterations)
        c.synchronize()
        return its

    t0 = time.perf_counter()
    its = api.run_ranks(lambda r: body(r, ctxs[r]), len(ctxs)) if nranks else [body(0, ctxs[0])]
    wall = time.perf_counter() - t0
    for c in ctxs:
        loc, glob = c.owned() if nranks else ((slice(None),), (slice(None),))
        f.u[glob] = c.get_field(A.HIP_FIELD_U)[loc]
        f.v[glob] = c.get_field(A.HIP_FIELD_V)[loc]
        c.close()
    if group is not None:
        group.close()
    eu, ev = cases.tg3_l2_errors(g, f, steps * 1e-3)
    return eu, ev, its[0], wall


def tg():
    steps = int(os.environ.get("STEPS", "100"))
    sizes = [int(s) for s in os.environ.get("SIZES", "32,64,128,256").split(",")]
    prev = None
    for n in sizes:
        eu, ev, its, wall = tg_run(n, steps)
        out = {"run": f"tg3d_{n}", "config": "BASELINE configs[1] (n=256) on projection_hip",
               "steps": steps, "rel_l2_u": eu, "rel_l2_v": ev, "cg_iters_total": int(sum(its)),
               "wall_s": round(wall, 2)}
        if prev is not None:
            out["order_u"] = math.log(prev[1] / eu) / math.log((n - 1) / (prev[0] - 1))
        prev = (n, eu)
        print(json.dumps(out), flush=True)
        log(f"tg {n} done {wall:.1f}s")


def tgslabs():
    n = int(os.environ.get("N", "512"))
    steps = int(os.environ.get("STEPS", "3"))
    base = None
    for nranks in (0, 2, 4, 8):
        eu, ev, its, wall = tg_run(n, steps, nranks)
        out = {"run": f"tg3d_{n}_slabs{max(nranks, 1)}", "config": "BASELINE configs[3] "
               "decomposition on one device (in-process group)", "steps": steps,
               "rel_l2_u": eu, "rel_l2_v": ev, "cg_iters": its, "wall_s": round(wall, 2)}
        if base is None:
            base = (eu, ev, its)
        else:
            out["d_rel_l2_u"] = abs(eu - base[0]) / base[0]
            out["d_rel_l2_v"] = abs(ev - base[1]) / base[1]
            out["pass"] = bool(out["d_rel_l2_u"] <= 1e-10 and out["d_rel_l2_v"] <= 1e-10)
        print(json.dumps(out), flush=True)
        log(f"tgslabs {nranks} done {wall:.1f}s")


if __name__ == "__main__":
    {"cavity128": cavity128, "tg": tg, "tgslabs": tgslabs}[sys.argv[1]]()
