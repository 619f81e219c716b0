"""Energy equation + Boussinesq coupling on the device (SURVEY.md §8a a9,
BASELINE config 5): thermal BCs bitwise, coupled steps vs the oracle, Z-slab
runs bitwise with RB-SOR, and the reference's de Vahl Davis Ra=1e3
validation (test_natural_convection.c:315-322) through the plugin."""
import json
from pathlib import Path

import numpy as np
import pytest

from cfd_amd import _abi as A
from cfd_amd import api
from oracle import oracle
from tests import cases, dvd

pytestmark = pytest.mark.gpu

GOLD = Path(__file__).resolve().parent / "golden"
P, N, D = A.BC_TYPE_PERIODIC, A.BC_TYPE_NEUMANN, A.BC_TYPE_DIRICHLET


def _thermal(p, types, vals=(310.0, 290.0, 301.0, 299.0, 305.0, 295.0)):
    tb = p.thermal_bc
    tb.left, tb.right, tb.bottom, tb.top, tb.back, tb.front = types
    dv = tb.dirichlet_values
    dv.left, dv.right, dv.bottom, dv.top, dv.back, dv.front = vals


def _convection_case(nx, ny, nz, alpha=2e-3, beta=3.333e-3):
    zmax = 1.0 if nz > 1 else 0.0
    g = api.Grid(nx, ny, nz, 0.0, 1.0, 0.0, 1.0, 0.0, zmax)
    f = api.FlowField(nx, ny, nz)
    rng = np.random.default_rng(3)
    f.u[...] = 0.01 * rng.standard_normal(f.u.shape)
    f.v[...] = 0.01 * rng.standard_normal(f.v.shape)
    f.w[...] = 0.01 * rng.standard_normal(f.w.shape) if nz > 1 else 0.0
    f.p[...] = 0.0
    f.rho[...] = 1.0
    f.T[...] = 310.0 - 20.0 * np.asarray(g.x)[None, None, :] + 0.1 * rng.standard_normal(f.T.shape)
    p = api.validation_params(1e-3, 1e-2)
    p.alpha = alpha
    p.beta = beta
    p.T_ref = 300.0
    p.gravity[1] = -9.81
    return g, f, p


@pytest.mark.parametrize("shape", [(17, 13, 11), (16, 16, 1)])
@pytest.mark.parametrize("types", [(D, D, N, N, N, N), (P, P, P, P, P, P), (N, D, P, P, D, N),
                                   (D, N, D, N, P, P)])
def test_thermal_bcs_bitwise(hip_lib, shape, types):
    nx, ny, nz = shape
    g, f, p = _convection_case(nx, ny, nz)
    _thermal(p, types)
    ctx = api.HipProjection(nx, ny, nz)
    ctx.set_field(A.HIP_FIELD_T, f.T)
    assert ctx._lib().hip_proj_apply_thermal_bcs(ctx.ctx, api.C.byref(p)) == A.CFD_SUCCESS
    got = ctx.get_field(A.HIP_FIELD_T)
    ctx.close()
    assert oracle.apply_thermal_bcs(f, p) == A.CFD_SUCCESS
    np.testing.assert_array_equal(got, f.T)


def _steps(g, f, p, n, method=A.HIP_POISSON_CG, **cfg):
    fo = api.FlowField(g.nx, g.ny, g.nz)
    fo.copy_from(f)
    ctx = api.HipProjection(g.nx, g.ny, g.nz, poisson_method=method, **cfg)
    okind = {A.HIP_POISSON_CG: A.ORACLE_POISSON_CG,
             A.HIP_POISSON_REDBLACK: A.ORACLE_POISSON_REDBLACK}[method]
    for _ in range(n):
        sto_ = oracle.projection_step(fo, g, p, okind)
        sth = A.SolverStats()
        assert ctx.step(f, g, p, sth) == A.CFD_SUCCESS, api._native.last_error()
        assert sto_[0] == A.CFD_SUCCESS
        assert sth.max_temperature == pytest.approx(float(np.max(fo.T)), rel=1e-12)
    ctx.close()
    return fo


@pytest.mark.parametrize("shape", [(17, 13, 11), (24, 20, 1)])
def test_energy_steps_cg_vs_oracle(hip_lib, shape):
    g, f, p = _convection_case(*shape)
    _thermal(p, (D, D, N, N, N, N))
    fo = _steps(g, f, p, 5)
    for k in ("u", "v", "w", "p", "T"):
        a, b = getattr(f, k), getattr(fo, k)
        assert float(np.max(np.abs(a - b))) / max(1.0, float(np.max(np.abs(b)))) <= 1e-10, k


def _at_rest(f):
    # RB-SOR runs the singular Neumann problem (linear_solver_redblack.c:139);
    # a random velocity field's divergence is far from compatible with it, so
    # these cases start at rest (buoyancy drives the flow) with the looser
    # tolerance the cavity RB tests use.
    f.u[...] = 0.0
    f.v[...] = 0.0
    f.w[...] = 0.0


RB_TOL = 1e-2


def test_energy_steps_rbsor_bitwise(hip_lib):
    g, f, p = _convection_case(17, 13, 11)
    _at_rest(f)
    _thermal(p, (D, D, N, N, P, P))
    oracle.set_projection_poisson_params(oracle.poisson_params(tolerance=RB_TOL))
    try:
        fo = _steps(g, f, p, 4, method=A.HIP_POISSON_REDBLACK, poisson_tolerance=RB_TOL)
    finally:
        oracle.set_projection_poisson_params(None)
    for k in ("u", "v", "w", "p", "T"):
        np.testing.assert_array_equal(getattr(f, k), getattr(fo, k), err_msg=k)


@pytest.mark.parametrize("nranks,zbc", [(2, P), (3, N)])
def test_slab_energy_rbsor_bitwise(hip_lib, monkeypatch, nranks, zbc):
    """Config 5 in miniature: Boussinesq + energy with RB-SOR on Z-slabs,
    bitwise the single-domain oracle (periodic thermal z faces wrap across
    the slabs)."""
    monkeypatch.setenv("CFD_HIP_GROUP_TIMEOUT_S", "60")
    g, f, p = _convection_case(17, 13, 11)
    _at_rest(f)
    _thermal(p, (D, D, N, N, zbc, zbc))
    grp = api.LocalGroup(nranks)
    ctxs = [api.HipProjection(17, 13, 11, comm=grp.comm(r, 0),
                              poisson_method=A.HIP_POISSON_REDBLACK, poisson_tolerance=RB_TOL)
            for r in range(nranks)]
    fid = {"u": A.HIP_FIELD_U, "v": A.HIP_FIELD_V, "w": A.HIP_FIELD_W, "p": A.HIP_FIELD_P,
           "T": A.HIP_FIELD_T}
    try:
        for c in ctxs:
            sl = slice(c.k_offset, c.k_offset + c.nz_local)
            for k, i in fid.items():
                c.set_field(i, getattr(f, k)[sl])
            c.set_density(1.0)

        def body(r, c):
            for _ in range(3):
                st = A.SolverStats()
                assert c.step_device(g, p, st) == A.CFD_SUCCESS, api._native.last_error()
            return st.max_temperature
        tmax = api.run_ranks(lambda r: body(r, ctxs[r]), nranks)
        got = {}
        for k, i in fid.items():
            out = np.full(f.u.shape, np.nan)
            for c in ctxs:
                loc, glob = c.owned()
                out[glob] = c.get_field(i)[loc]
            got[k] = out
    finally:
        for c in ctxs:
            c.close()
        grp.close()
    oracle.set_projection_poisson_params(oracle.poisson_params(tolerance=RB_TOL))
    try:
        for _ in range(3):
            assert oracle.projection_step(f, g, p, A.ORACLE_POISSON_REDBLACK)[0] == A.CFD_SUCCESS
    finally:
        oracle.set_projection_poisson_params(None)
    for k in fid:
        np.testing.assert_array_equal(got[k], getattr(f, k), err_msg=k)
    assert all(t == float(np.max(f.T)) for t in tmax)


def test_energy_rejects_heat_source_callback(hip_lib):
    g, f, p = _convection_case(9, 9, 9)
    cb = A.HeatSourceFunc(lambda x, y, z, t, ctx: 0.0)
    p.heat_source_func = api.C.cast(cb, api.C.c_void_p)
    ctx = api.HipProjection(9, 9, 9)
    assert ctx.step(f, g, p, A.SolverStats()) == A.CFD_ERROR_UNSUPPORTED
    ctx.close()


def test_de_vahl_davis_ra1e3(hip_lib):
    """test_natural_convection.c:315-322 through the projection_hip plugin:
    the reference's 10 % gate on (u_max*, v_max*, Nu) and agreement with the
    oracle's run (tests/golden/dvd41_ra1e3.json) to 1e-6."""
    g, f, p, alpha = dvd.setup(41, 1000.0, 0.002)
    reg = api.Registry()
    s = reg.create("projection_hip")
    assert s.init(g, p) == A.CFD_SUCCESS
    st = A.SolverStats()
    r = dvd.run(lambda ff: s.step(ff, g, p, st), g, f, p, alpha, 30000)
    s.close()
    assert r["converged"]
    for got, ref in zip((r["umax"], r["vmax"], r["nu"]), dvd.REF_RA1E3):
        assert abs(got - ref) / ref < dvd.GATE
    want = json.loads((GOLD / "dvd41_ra1e3.json").read_text())
    assert abs(r["steps"] - want["steps"]) <= 2
    for k in ("umax", "vmax", "nu"):
        assert r[k] == pytest.approx(want[k], rel=1e-6), k


def _seq_max(a):
    """compute_max_temperature's loop (solver_registry.c:52-62): m = T[0];
    m = T[i] if T[i] > m."""
    m = a[0]
    for v in a[1:]:
        if v > m:
            m = v
    return m


@pytest.mark.parametrize("plant", ["max_last_chunk", "nan_inside", "nan_first", "signed_zero"])
def test_host_step_max_temperature_threaded(hip_lib, plant):
    """The host-buffer step's stats.max_temperature (the full-transfer path
    computes it on the caller's T, now on up to 16 threads, r06) equals the
    reference's sequential loop bit for bit: a maximum in the last chunk, a
    NaN inside (skipped by the strict comparison), a NaN at T[0] (kept), and
    -0.0 / +0.0 ties (the first one kept). 130 x 130 x 66 = 1.1 M cells, so
    the threaded path runs."""
    g, f, p = cases.cavity(130, 130, 66, Re=100.0, dt=1e-4)
    t = f.T.reshape(-1)
    rng = np.random.default_rng(3)
    t[...] = rng.uniform(290.0, 310.0, t.size)
    if plant == "max_last_chunk":
        t[-5] = 400.0
    elif plant == "nan_inside":
        t[t.size // 3] = np.nan
        t[t.size // 2] = 350.0
    elif plant == "nan_first":
        t[0] = np.nan
    else:
        t[...] = -0.0
        t[t.size // 2] = 0.0
    want = _seq_max(t[: min(t.size, 8)]) if plant == "nan_first" else None
    reg = api.Registry()
    solver = reg.create("projection_hip")
    try:
        assert solver.init(g, p) == A.CFD_SUCCESS
        st = A.SolverStats()
        assert solver.step(f, g, p, st) == A.CFD_SUCCESS, api._native.last_error()
    finally:
        solver.close()
    got = st.max_temperature
    if plant == "nan_first":
        assert np.isnan(got) and np.isnan(want)
        return
    ref = float(np.max(t[~np.isnan(t)])) if plant != "signed_zero" else -0.0
    assert got == ref
    if plant == "signed_zero":
        assert np.signbit(got)  # -0.0 at T[0] stays: +0.0 > -0.0 is false
