"""The committed fixtures in tests/golden/ against the oracle (CPU) and the
reference vectors they descend from."""
import json
from pathlib import Path

import numpy as np
import pytest

from cfd_amd import _abi as A
from cfd_amd import api
from oracle import oracle
from tests import cases

GOLD = Path(__file__).resolve().parent / "golden"
F4 = ("u", "v", "w", "p")


def load(name):
    return np.load(GOLD / name, allow_pickle=False)


def test_reference_vectors_match_cases():
    ref = json.loads((GOLD / "reference_vectors.json").read_text())["projection_kat16_l2"]
    assert (ref["u"], ref["v"], ref["p"]) == cases.KAT_PROJECTION_L2


def test_kat_fixture_reproduces_reference_l2():
    z = load("kat16_projection_step1.npz")
    l2 = (cases.l2_rms(z["u"]), cases.l2_rms(z["v"]), cases.l2_rms(z["p"]))
    assert l2 == cases.KAT_PROJECTION_L2


@pytest.mark.parametrize("name,kind,tol", [
    ("cavity17_rbsor_tol1e-2_3steps.npz", A.ORACLE_POISSON_REDBLACK, 1e-2),
    ("cavity17_cg_3steps.npz", A.ORACLE_POISSON_CG, None)])
def test_cavity_fixtures_regenerate_bitwise(name, kind, tol):
    z = load(name)
    g, f, p = cases.cavity(17, 17, 17, Re=100.0, dt=5e-4)
    oracle.set_threads(1)
    if tol:
        oracle.set_projection_poisson_params(oracle.poisson_params(tolerance=tol))
    try:
        for i in range(3):
            api.cavity_bc(f, 1.0)
            s, _, it = oracle.projection_step(f, g, p, kind)
            assert s == A.CFD_SUCCESS and it == z["iters"][i]
    finally:
        oracle.set_projection_poisson_params(None)
    for k in F4:
        np.testing.assert_array_equal(getattr(f, k), z[k], err_msg=k)


def test_poisson_fixture_regenerates_bitwise():
    z = load("poisson17_cos.npz")
    g, rhs = cases.cos_rhs(17)
    np.testing.assert_array_equal(rhs, z["rhs"])
    x = np.zeros_like(rhs)
    s, st = oracle.redblack_solve(x, rhs, g.dx, g.dy, g.dz)
    assert st.iterations == z["iters_rbsor"]
    np.testing.assert_array_equal(x, z["x_rbsor"])


def test_cavity128_re1000_fixture_consistent():
    """configs[0] oracle fixture (make_golden.py cavity128): the Ghia RMS the
    survey measured on a reference build (0.0299 / 0.0282),
    under the reference's 0.10 gate (test_cavity_backends.c:50), and the
    stored centrelines / fields agree with each other; the first 10 steps of
    the 1000-step snapshot are re-run on the oracle here."""
    from tests import ghia
    r = json.loads((GOLD / "cavity128_re1000_t50.json").read_text())
    assert round(r["rms_u"], 4) == 0.0299 and round(r["rms_v"], 4) == 0.0282
    assert r["rms_u"] < 0.10 and r["rms_v"] < 0.10
    z = load("cavity128_re1000_t50_fields.npz")
    g = api.Grid(128, 128, 1, 0.0, 1.0, 0.0, 1.0, 0.0, 0.0)
    y, uc, x, vc = ghia.centerlines(z["u"][0], z["v"][0], g.x, g.y)
    assert uc == r["u_centerline"] and vc == r["v_centerline"]
    assert int(z["iters"].sum()) == r["cg_iters_total"]
    snap = load("cavity128_re1000_1000steps.npz")
    assert np.array_equal(snap["iters"], z["iters"][:1000])
    g, f, p = cases.cavity(128, 128, 1, Re=1000.0, dt=5e-4)
    its = []
    for _ in range(10):
        api.cavity_bc(f, 1.0)
        s, _, it = oracle.projection_step(f, g, p)
        assert s == A.CFD_SUCCESS
        its.append(it)
    assert its == list(snap["iters"][:10])


@pytest.mark.parametrize("name,threads", [("conv32cap", 1), ("conv32cap", 3)])
def test_convection_fixture_regenerates_bitwise(name, threads):
    """convection_conv32cap.json (configs[4] at tol 1e-6, cap 20000: step 2
    runs 20001 RB-SOR iterations) from the oracle at 1 and 3 threads: the
    fingerprints do not depend on the thread count (the fixtures were written
    with 8)."""
    import hashlib

    import bench

    fx = json.loads((GOLD / f"convection_{name}.json").read_text())
    nx, ny, nz = fx["grid"]
    g, p, T0 = bench.convection_setup(nx, ny, nz)
    f = api.FlowField(nx, ny, nz)
    f.u[...] = f.v[...] = f.w[...] = f.p[...] = 0.0
    f.rho[...] = 1.0
    f.T[...] = np.broadcast_to(T0[None, None, :], f.T.shape)
    oracle.set_threads(threads)
    oracle.set_projection_poisson_params(oracle.poisson_params(
        tolerance=fx["tolerance"], max_iterations=fx["max_iterations"]))
    try:
        for want in fx["steps"]:
            s, _, it = oracle.projection_step(f, g, p, A.ORACLE_POISSON_REDBLACK)
            ps = oracle.last_poisson_stats()
            assert (s, ps.iterations, ps.final_residual) == (
                want["status"], want["iterations"], want["final_residual"])
            for k, w in want["fields"].items():
                a = np.ascontiguousarray(getattr(f, k))
                assert hashlib.sha256(a.tobytes()).hexdigest() == w["sha256"], k
    finally:
        oracle.set_projection_poisson_params(None)
        oracle.set_threads(1)
