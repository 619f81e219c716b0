#!/usr/bin/env python3
"""Regenerates the golden fixtures in tests/golden/ from the CPU oracle.

The oracle is itself pinned to the reference's own vectors
(tests/test_oracle_golden.py: test_ns_solver_3d.c:345-348 bit for bit, the
Ghia RMS of cavity-backends-validation.md:115, the CG iteration counts of a
reference build); these fixtures freeze its full-field outputs so the GPU
tests can check the HIP path against stored data as well as the live oracle.

usage: python tests/golden/make_golden.py      (writes *.npz next to this file)
"""
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent))

from cfd_amd import _abi as A  # noqa: E402
from cfd_amd import api  # noqa: E402
from oracle import oracle  # noqa: E402
from tests import cases  # noqa: E402


def fields(f):
    return {k: getattr(f, k).copy() for k in ("u", "v", "w", "p")}


def kat():
    g, f, p = cases.kat_2d()
    s, st, it = oracle.projection_step(f, g, p)
    assert s == A.CFD_SUCCESS
    np.savez_compressed(HERE / "kat16_projection_step1.npz", cg_iters=it, **fields(f))


def cavity_rbsor():
    g, f, p = cases.cavity(17, 17, 17, Re=100.0, dt=5e-4)
    oracle.set_projection_poisson_params(oracle.poisson_params(tolerance=1e-2))
    its = []
    for _ in range(3):
        api.cavity_bc(f, 1.0)
        s, st, it = oracle.projection_step(f, g, p, A.ORACLE_POISSON_REDBLACK)
        assert s == A.CFD_SUCCESS
        its.append(it)
    oracle.set_projection_poisson_params(None)
    np.savez_compressed(HERE / "cavity17_rbsor_tol1e-2_3steps.npz", iters=np.array(its),
                        **fields(f))


def cavity_cg():
    g, f, p = cases.cavity(17, 17, 17, Re=100.0, dt=5e-4)
    its = []
    for _ in range(3):
        api.cavity_bc(f, 1.0)
        s, st, it = oracle.projection_step(f, g, p, A.ORACLE_POISSON_CG)
        assert s == A.CFD_SUCCESS
        its.append(it)
    np.savez_compressed(HERE / "cavity17_cg_3steps.npz", iters=np.array(its), **fields(f))


def tg():
    g, f, p = cases.tg3(17)
    for _ in range(5):
        cases.tg3_bc(f)
        s, _, _ = oracle.projection_step(f, g, p)
        assert s == A.CFD_SUCCESS
    np.savez_compressed(HERE / "tg17_cg_5steps.npz", **fields(f))


def poisson():
    g, rhs = cases.cos_rhs(17)
    out = {}
    for name, fn in (("cg", oracle.cg_solve), ("rbsor", oracle.redblack_solve),
                     ("jacobi", oracle.jacobi_solve)):
        x = np.zeros_like(rhs)
        prm = oracle.poisson_params(max_iterations=3000) if name == "jacobi" else None
        s, st = fn(x, rhs, g.dx, g.dy, g.dz, prm)
        out[f"x_{name}"] = x
        out[f"iters_{name}"] = st.iterations
        out[f"status_{name}"] = s
    np.savez_compressed(HERE / "poisson17_cos.npz", rhs=rhs, **out)


def dvd_ra1e3():
    """de Vahl Davis Ra=1e3 on 41^2 (test_natural_convection.c:315-322)."""
    import json

    from tests import dvd
    g, f, p, alpha = dvd.setup(41, 1000.0, 0.002)
    r = dvd.run(lambda ff: oracle.projection_step(ff, g, p)[0], g, f, p, alpha, 30000)
    r = {k: (float(v) if not isinstance(v, bool) else v) for k, v in r.items()}
    (HERE / "dvd41_ra1e3.json").write_text(json.dumps(r, indent=1) + "\n")
    np.savez_compressed(HERE / "dvd41_ra1e3_fields.npz", u=f.u, v=f.v, p=f.p, T=f.T)


def cavity128_re1000(steps=100000, snap=1000):
    """BASELINE configs[0]: 128x128x1 lid-driven cavity, Re=1000, dt=5e-4,
    100 000 steps (t = 50, test_cavity_backends.c:74-76), scalar projection
    with the cavity BCs before every step (lid_driven_cavity_common.h:238-270).
    Writes the Ghia RMS (cavity_validation_utils.h:36-65 restated in
    tests/ghia.py), the centrelines, the per-step CG iteration counts and the
    fields after `snap` steps and at the end. About an hour on one core."""
    import json

    from tests import ghia
    g, f, p = cases.cavity(128, 128, 1, Re=1000.0, dt=5e-4)
    its = []
    for n in range(1, steps + 1):
        api.cavity_bc(f, 1.0)
        s, st, it = oracle.projection_step(f, g, p)
        assert s == A.CFD_SUCCESS
        its.append(it)
        if n == snap:
            np.savez_compressed(HERE / f"cavity128_re1000_{snap}steps.npz",
                                iters=np.array(its), **fields(f))
    api.cavity_bc(f, 1.0)
    y, uc, x, vc = ghia.centerlines(f.u[0], f.v[0], g.x, g.y)
    rms_u, rms_v = ghia.rms_errors(f, g, 1000)
    r = {"steps": steps, "dt": 5e-4, "re": 1000.0, "rms_u": rms_u, "rms_v": rms_v,
         "cg_iters_total": int(sum(its)), "cg_iters_last": int(its[-1]),
         "u_centerline": uc, "v_centerline": vc}
    (HERE / "cavity128_re1000_t50.json").write_text(json.dumps(r, indent=1) + "\n")
    np.savez_compressed(HERE / "cavity128_re1000_t50_fields.npz",
                        iters=np.array(its, dtype=np.int32), **fields(f))


if __name__ == "__main__":
    oracle.set_threads(1)
    if sys.argv[1:] == ["cavity128"]:
        cavity128_re1000()
        sys.exit(0)
    dvd_ra1e3()
    kat()
    cavity_rbsor()
    cavity_cg()
    tg()
    poisson()
    for f in sorted(HERE.glob("*.npz")):
        print(f.name, f.stat().st_size)
