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


CAV512_SNAP_STEPS = (1, 6, 25)
CAV512_PLANES = (1, 255, 510)
CAV512_ROWS = (1, 255, 509, 510)
CAV512_COLS = (1, 255, 510)


def plane_samples(a2: np.ndarray) -> dict:
    """What the 512^3 fixture keeps of one z plane: a stride-4 lattice (plus
    the last index), full rows j = 1, 255, 509, 510 (the lid's boundary layer
    sits at j = 510), full columns i = 1, 255, 510, and sum / L2 / max |.|
    of the whole plane."""
    n = a2.shape[0]
    idx = np.r_[np.arange(0, n, 4), n - 1] if (n - 1) % 4 else np.arange(0, n, 4)
    rows = [j for j in CAV512_ROWS if j < n]
    cols = [i for i in CAV512_COLS if i < a2.shape[1]]
    return {"lattice_idx": idx, "lattice": a2[np.ix_(idx, idx)].copy(),
            "rows_j": np.array(rows), "rows": a2[rows, :].copy(),
            "cols_i": np.array(cols), "cols": a2[:, cols].T.copy(),
            "stats": np.array([float(np.sum(a2)), float(np.sqrt(np.sum(a2 * a2))),
                               float(np.max(np.abs(a2)))])}


def field_norms(f) -> dict:
    """L2 (sqrt of the pairwise sum of squares) and max |.| of the interior
    of each field (the cells the step computes; the boundary u = 1 lid would
    dominate a whole-field norm)."""
    out = {}
    for k in ("u", "v", "w", "p"):
        a = np.ascontiguousarray(getattr(f, k)[1:-1, 1:-1, 1:-1])
        out[k] = [float(np.sqrt(np.sum(a * a))), float(np.max(np.abs(a)))]
    return out


def cavity512_re1000(n=512, steps=25, state_dir="/tmp/cav512_state", threads=8):
    """BASELINE configs[2] at its own size, on the bench's exact trajectory:
    n^3 lid-driven cavity, Re = 1000, dt = 1e-4, from rest, lid u = 1 on
    y = 1 and Neumann p before every step (bench.py make_ctx; the step keeps
    the boundary faces, so applying them before every step is the same as
    once), the reference's CG settings (rel 1e-6, abs 1e-10, 5000).
    The oracle runs its OpenMP twin (the reference's projection_omp /
    cg_omp_solve order of dot-product partials, solver_projection_omp.c:26-279)
    on `threads` cores: about 5 min per step here, so the state is saved to
    `state_dir` after every step and a rerun resumes.
    Writes cavity{n}_re1000_steps.json (per step: CG iterations, initial /
    final residual, L2 and max |.| of u, v, w, p) and, after the steps in
    CAV512_SNAP_STEPS, cavity{n}_re1000_step{s}_planes.npz (plane_samples of
    u, v, w, p at k in CAV512_PLANES)."""
    import json
    import time

    sd = Path(state_dir)
    sd.mkdir(parents=True, exist_ok=True)
    oracle.set_threads(threads)
    g, f, p = cases.cavity(n, n, n, Re=1000.0, dt=1e-4)
    out_json = HERE / f"cavity{n}_re1000_steps.json"
    rec = {"grid": [n, n, n], "re": 1000.0, "dt": 1e-4, "steps": [],
           "oracle": f"oracle_projection_step, CG, OpenMP {threads} threads",
           "generator": "tests/golden/make_golden.py cavity512"}
    prog = sd / "progress.json"
    if prog.exists():
        rec = json.loads(prog.read_text())
        for k in ("u", "v", "w", "p"):
            getattr(f, k)[...] = np.load(sd / f"{k}.npy")
        print(f"resumed after step {len(rec['steps'])}", flush=True)
    while len(rec["steps"]) < steps:
        s = len(rec["steps"]) + 1
        t0 = time.time()
        api.cavity_bc(f, 1.0)
        st, sts, it = oracle.projection_step(f, g, p)
        assert st == A.CFD_SUCCESS, st
        ps = oracle.last_poisson_stats()
        row = {"step": s, "cg_iters": it, "initial_residual": ps.initial_residual,
               "final_residual": ps.final_residual, "max_velocity": sts.max_velocity,
               "max_pressure": sts.max_pressure, "norms": field_norms(f),
               "seconds": round(time.time() - t0, 1)}
        rec["steps"].append(row)
        print(json.dumps(row), flush=True)
        if s in CAV512_SNAP_STEPS:
            planes = {}
            for k in ("u", "v", "w", "p"):
                for kz in CAV512_PLANES:
                    if kz < n:
                        for key, val in plane_samples(getattr(f, k)[kz]).items():
                            planes[f"{k}_k{kz}_{key}"] = val
            np.savez_compressed(HERE / f"cavity{n}_re1000_step{s}_planes.npz", **planes)
        out_json.write_text(json.dumps(rec, indent=1) + "\n")
        if s < steps:
            for k in ("u", "v", "w", "p"):
                np.save(sd / f"{k}.npy", getattr(f, k))
            prog.write_text(json.dumps(rec))


def field_sha(a: np.ndarray) -> str:
    """sha256 of a field's packed fp64 bytes (k, j, i order): the bitwise
    fingerprint the RB-SOR convection tests compare against."""
    import hashlib

    return hashlib.sha256(np.ascontiguousarray(a, dtype=np.float64).tobytes()).hexdigest()


# configs[4] at its own tolerance: bench.convection_setup
# (test_natural_convection.c:140-293 in 3-D) with the RB-SOR pressure solve at
# tol 1e-6 and the bench's cap of 20000 iterations. Grid sizes: at 96^2 x 48
# all three steps converge (~1.2-1.5k iterations each); at 32^2 x 16 step 2
# stalls on the singular Neumann problem and runs into the cap (20001
# iterations, CFD_ERROR_MAX_ITER): the long-iteration regime of the L-inf
# checked loop (linear_solver.c:397-485 driving linear_solver_redblack.c:80-147).
CONV_CASES = {"conv96": (96, 96, 48, 3), "conv32cap": (32, 32, 16, 2)}
CONV_TOL, CONV_CAP = 1e-6, 20000


def convection(name: str, threads: int = 8):
    """Writes convection_<name>.json: per step the projection status, the
    RB-SOR iterations / initial / final L-inf residual / status, and per field
    (u, v, w, p, T) the sha256 of its bytes plus sum, L2 and max |.|. RB-SOR
    and the energy step are per-cell arithmetic and an L-inf max, so the
    oracle's result does not depend on its thread count and the device's must
    be bitwise equal."""
    import json

    import bench

    nx, ny, nz, steps = CONV_CASES[name]
    oracle.set_threads(threads)
    g, p, T0 = bench.convection_setup(nx, ny, nz)
    f = api.FlowField(nx, ny, nz)
    f.u[...] = f.v[...] = f.w[...] = f.p[...] = 0.0
    f.rho[...] = 1.0
    f.T[...] = np.broadcast_to(T0[None, None, :], f.T.shape)
    oracle.set_projection_poisson_params(oracle.poisson_params(tolerance=CONV_TOL,
                                                               max_iterations=CONV_CAP))
    rec = {"grid": [nx, ny, nz], "tolerance": CONV_TOL, "max_iterations": CONV_CAP,
           "setup": "bench.convection_setup, fluid at rest, T linear in x",
           "generator": f"tests/golden/make_golden.py {name}", "steps": []}
    try:
        for s in range(1, steps + 1):
            st, _, it = oracle.projection_step(f, g, p, A.ORACLE_POISSON_REDBLACK)
            ps = oracle.last_poisson_stats()
            row = {"step": s, "status": int(st), "iterations": int(ps.iterations),
                   "initial_residual": ps.initial_residual,
                   "final_residual": ps.final_residual, "poisson_status": int(ps.status),
                   "fields": {}}
            for k in ("u", "v", "w", "p", "T"):
                a = getattr(f, k)
                row["fields"][k] = {"sha256": field_sha(a), "sum": float(np.sum(a)),
                                    "l2": float(np.sqrt(np.sum(a * a))),
                                    "max": float(np.max(np.abs(a)))}
            rec["steps"].append(row)
            print(s, st, it, ps.final_residual, flush=True)
    finally:
        oracle.set_projection_poisson_params(None)
    (HERE / f"convection_{name}.json").write_text(json.dumps(rec, indent=1) + "\n")


if __name__ == "__main__":
    oracle.set_threads(1)
    if sys.argv[1:2] and sys.argv[1] in CONV_CASES:
        convection(sys.argv[1])
        sys.exit(0)
    if sys.argv[1:] == ["cavity128"]:
        cavity128_re1000()
        sys.exit(0)
    if sys.argv[1:2] == ["cavity512"]:
        # optional: size steps state_dir (defaults: the bench's 512^3, 25 steps)
        a = sys.argv[2:]
        cavity512_re1000(int(a[0]) if a else 512, int(a[1]) if len(a) > 1 else 25,
                         a[2] if len(a) > 2 else "/tmp/cav512_state")
        sys.exit(0)
    dvd_ra1e3()
    kat()
    cavity_rbsor()
    cavity_cg()
    tg()
    poisson()
    for f in sorted(HERE.glob("*.npz")):
        print(f.name, f.stat().st_size)
