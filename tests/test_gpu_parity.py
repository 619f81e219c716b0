"""Parity of the HIP product path (libcfd_hip.so via its C-ABI) with the CPU
oracle and the reference's golden vectors. Runs on an MI355X only."""
import ctypes as C
import math

import numpy as np
import pytest

from cfd_amd import _abi as A
from cfd_amd import api
from oracle import oracle
from tests import cases

pytestmark = pytest.mark.gpu

# CG dot products are summed in a different (blocked, deterministic) order on
# the GPU than the reference's sequential loop, so CG-based results agree to
# rounding, not bitwise. Tolerances below are relative to the field's scale.
CG_FIELD_RTOL = 1e-10
# The reference's own GPU-vs-CPU gate for CG (test_poisson_jacobi_gpu.c:303).
REF_GPU_CG_GATE = 1e-6


def _fields(f):
    return {k: getattr(f, k).copy() for k in ("u", "v", "w", "p")}


def _rel_maxdiff(a, b):
    scale = max(1.0, float(np.max(np.abs(b))))
    return float(np.max(np.abs(a - b))) / scale


def _clone(g, f):
    f2 = api.FlowField(g.nx, g.ny, g.nz)
    f2.copy_from(f)
    return f2


def test_plugin_projection_kat(hip_lib):
    """The `projection_hip` plugin through the registry on the reference KAT
    (test_ns_solver_3d.c:267-348): golden L2 norms within the reference's 1e-12."""
    g, f, p = cases.kat_2d()
    reg = api.Registry()
    assert reg.has("projection_hip")
    s = reg.create("projection_hip")
    assert s.init(g, p) == A.CFD_SUCCESS
    p.max_iter = 3  # the reference helper sets 3; the step wrapper does exactly one step
    st = A.SolverStats()
    assert s.step(f, g, p, st) == A.CFD_SUCCESS
    assert st.iterations == 1
    l2 = (cases.l2_rms(f.u), cases.l2_rms(f.v), cases.l2_rms(f.p))
    for got, want in zip(l2, cases.KAT_PROJECTION_L2):
        assert abs(got - want) <= 1e-12, (got, want)
    assert np.all(f.w == 0.0)
    s.close()


def _step_both(g, f, p, n_steps, bc=None, method=A.HIP_POISSON_CG, **cfg):
    """Advance a copy with the HIP context and a copy with the oracle."""
    fo = _clone(g, f)
    fh = _clone(g, f)
    ctx = api.HipProjection(g.nx, g.ny, g.nz, poisson_method=method, **cfg)
    okind = {A.HIP_POISSON_CG: A.ORACLE_POISSON_CG, A.HIP_POISSON_REDBLACK:
             A.ORACLE_POISSON_REDBLACK, A.HIP_POISSON_JACOBI: A.ORACLE_POISSON_JACOBI}[method]
    for _ in range(n_steps):
        if bc:
            bc(fo)
            bc(fh)
        so, sto, io = oracle.projection_step(fo, g, p, okind)
        sth = A.SolverStats()
        sh = ctx.step(fh, g, p, sth)
        assert so == A.CFD_SUCCESS, so
        assert sh == A.CFD_SUCCESS, (sh, api._native.last_error())
        ih = ctx.poisson_stats().iterations
        assert abs(ih - io) <= (0 if method != A.HIP_POISSON_CG else 1), (ih, io)
        assert sth.iterations == 1
        assert sth.max_velocity == pytest.approx(sto.max_velocity, rel=1e-9, abs=1e-300)
        assert sth.max_pressure == pytest.approx(sto.max_pressure, rel=1e-9, abs=1e-300)
    ctx.close()
    return fo, fh


def test_step_kat_fields_vs_oracle(hip_lib):
    g, f, p = cases.kat_2d()
    fo, fh = _step_both(g, f, p, 1)
    for k in ("u", "v", "w", "p"):
        assert _rel_maxdiff(getattr(fh, k), getattr(fo, k)) <= CG_FIELD_RTOL, k


def test_step_default_source_3d_vs_oracle(hip_lib):
    """ns_solver_params_default keeps the default source term on (trap 4)."""
    g = api.Grid(17, 13, 11, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0)
    f = api.FlowField(17, 13, 11)
    api._native.host().initialize_flow_field(f.ptr, g.ptr)
    p = api.params_default()
    p.dt = 1e-4
    fo, fh = _step_both(g, f, p, 2)
    for k in ("u", "v", "w", "p"):
        assert _rel_maxdiff(getattr(fh, k), getattr(fo, k)) <= CG_FIELD_RTOL, k


def test_tg3d_vs_oracle(hip_lib):
    g, f, p = cases.tg3(17)
    fo, fh = _step_both(g, f, p, 5, bc=cases.tg3_bc)
    for k in ("u", "v", "w", "p"):
        assert _rel_maxdiff(getattr(fh, k), getattr(fo, k)) <= CG_FIELD_RTOL, k


def test_cavity3d_vs_oracle(hip_lib):
    g, f, p = cases.cavity(33, 33, 33, Re=100.0, dt=5e-4)
    fo, fh = _step_both(g, f, p, 4, bc=lambda ff: api.cavity_bc(ff, 1.0))
    for k in ("u", "v", "w", "p"):
        assert _rel_maxdiff(getattr(fh, k), getattr(fo, k)) <= CG_FIELD_RTOL, k


@pytest.mark.parametrize("method", [A.HIP_POISSON_REDBLACK, A.HIP_POISSON_JACOBI])
def test_relaxation_projection_bitwise(hip_lib, method):
    """RB-SOR and Jacobi involve no summation (L-infinity residuals, in-place
    colour updates that read only the other colour), so the HIP step is
    bitwise the oracle's, iteration counts included."""
    # the cavity's discrete divergence is not Neumann-compatible, so the
    # relaxation methods cannot reach the default 1e-6 (the oracle fails too);
    # both sides use the same looser relative tolerance here.
    g, f, p = cases.cavity(17, 17, 17, Re=100.0, dt=5e-4)
    maxit = 2000 if method == A.HIP_POISSON_JACOBI else 5000
    oracle.set_projection_poisson_params(
        oracle.poisson_params(tolerance=1e-2, max_iterations=maxit))
    try:
        fo, fh = _step_both(g, f, p, 3, bc=lambda ff: api.cavity_bc(ff, 1.0), method=method,
                            poisson_tolerance=1e-2, poisson_max_iter=maxit)
    finally:
        oracle.set_projection_poisson_params(None)
    for k in ("u", "v", "w", "p"):
        np.testing.assert_array_equal(getattr(fh, k), getattr(fo, k), err_msg=k)


@pytest.mark.parametrize("shape", [(16, 16, 1), (17, 13, 11), (9, 33, 5)])
def test_device_bc_kernels_bitwise(hip_lib, shape):
    nx, ny, nz = shape
    rng = np.random.default_rng(7)
    ctx = api.HipProjection(nx, ny, nz)
    for mode in ("neumann", "periodic", "dirichlet"):
        a = rng.standard_normal((nz, ny, nx))
        ctx.set_field(A.HIP_FIELD_U, a)
        want = a.copy()
        if mode == "neumann":
            ctx.apply_scalar_bc(A.HIP_FIELD_U, A.BC_TYPE_NEUMANN)
            oracle.bc_neumann(want)
        elif mode == "periodic":
            ctx.apply_scalar_bc(A.HIP_FIELD_U, A.BC_TYPE_PERIODIC)
            oracle.bc_periodic(want)
        else:
            v = api.dirichlet(1.0, 2.0, 3.0, 4.0, 5.0, 6.0)
            ctx.apply_dirichlet(A.HIP_FIELD_U, v)
            oracle.bc_dirichlet(want, v)
        np.testing.assert_array_equal(ctx.get_field(A.HIP_FIELD_U), want, err_msg=mode)
    ctx.close()


@pytest.mark.parametrize("n,expected", [(33, 47), (65, 97)])
def test_poisson_cg_vs_oracle(hip_lib, n, expected):
    """Standalone CG: iteration count of the reference build
    and the reference's demeaned GPU-vs-CPU gate (test_poisson_jacobi_gpu.c:303)."""
    g, rhs = cases.cos_rhs(n)
    xo = np.zeros_like(rhs)
    so, sto = oracle.cg_solve(xo, rhs, g.dx, g.dy, g.dz)
    ctx = api.HipProjection(n, n, n)
    xh = np.zeros_like(rhs)
    sh, sth = ctx.poisson_solve(A.HIP_POISSON_CG, xh, rhs, g.dx, g.dy, g.dz)
    assert so == sh == A.CFD_SUCCESS
    assert sto.iterations == expected
    assert abs(sth.iterations - expected) <= 1
    d = (xh - xh.mean()) - (xo - xo.mean())
    assert np.max(np.abs(d)) < REF_GPU_CG_GATE
    assert np.max(np.abs(d)) / np.max(np.abs(xo)) < 1e-9
    ctx.close()


@pytest.mark.parametrize("iters", [1, 2, 3, 4, 5, 6, 7, 8, 9])
def test_poisson_cg_fixed_iterations_vs_oracle(hip_lib, iters):
    """CG stopped by max_iterations after every residue of the fold period:
    sweep B folds x every fourth iteration and the finalize kernel applies the
    up to three unfolded alpha p, so x must hold exactly `iters` updates
    (linear_solver_cg.c:379-380)."""
    g, rhs = cases.cos_rhs(17)
    prm = oracle.poisson_params(max_iterations=iters)
    xo = np.zeros_like(rhs)
    so, sto = oracle.cg_solve(xo, rhs, g.dx, g.dy, g.dz, prm)
    ctx = api.HipProjection(17, 17, 17)
    xh = np.zeros_like(rhs)
    sh, sth = ctx.poisson_solve(A.HIP_POISSON_CG, xh, rhs, g.dx, g.dy, g.dz, prm)
    ctx.close()
    assert sh == so
    assert sth.iterations == sto.iterations == iters
    assert _rel_maxdiff(xh, xo) < 1e-12


@pytest.mark.parametrize("rows", [8, 16])
def test_cg_sweep_variants_bitwise_equal(hip_lib, rows):
    """The sweep variants (memory hints, plane prefetch) change how bytes move,
    not the arithmetic or the reduction tree: bitwise equal solutions and
    iteration counts for one tile height, and within the CG gate of the oracle."""
    g, rhs = cases.cos_rhs(33)
    xo = np.zeros_like(rhs)
    oracle.cg_solve(xo, rhs, g.dx, g.dy, g.dz)
    outs = []
    for v in (0, 3, 4, 7, 15, 23, 31):
        ctx = api.HipProjection(33, 33, 33, sweep_rows=rows, sweep_variant=v)
        xh = np.zeros_like(rhs)
        sh, sth = ctx.poisson_solve(A.HIP_POISSON_CG, xh, rhs, g.dx, g.dy, g.dz)
        ctx.close()
        assert sh == A.CFD_SUCCESS
        outs.append((sth.iterations, xh))
    for it, xh in outs[1:]:
        assert it == outs[0][0]
        np.testing.assert_array_equal(xh, outs[0][1])
    assert _rel_maxdiff(outs[0][1], xo) < 1e-9


@pytest.mark.parametrize("method", [A.HIP_POISSON_REDBLACK, A.HIP_POISSON_JACOBI])
def test_poisson_relax_bitwise(hip_lib, method):
    g, rhs = cases.cos_rhs(17)
    xo = np.zeros_like(rhs)
    prm = oracle.poisson_params(max_iterations=3000 if method == A.HIP_POISSON_JACOBI else 5000)
    if method == A.HIP_POISSON_REDBLACK:
        so, sto = oracle.redblack_solve(xo, rhs, g.dx, g.dy, g.dz, prm)
    else:
        so, sto = oracle.jacobi_solve(xo, rhs, g.dx, g.dy, g.dz, prm)
    ctx = api.HipProjection(17, 17, 17)
    xh = np.zeros_like(rhs)
    sh, sth = ctx.poisson_solve(method, xh, rhs, g.dx, g.dy, g.dz, prm)
    assert sh == so
    assert sth.iterations == sto.iterations
    np.testing.assert_array_equal(xh, xo)
    ctx.close()


@pytest.mark.parametrize("method", [A.HIP_POISSON_REDBLACK, A.HIP_POISSON_JACOBI])
@pytest.mark.parametrize("shape,kw", [
    ((17, 17, 17), dict()),                                   # converges
    ((23, 19, 14), dict(max_iterations=7)),                   # capped: iterations = 8
    ((33, 29, 1), dict(check_interval=5)),                    # 2-D, sparse checks
    ((130, 20, 9), dict(max_iterations=40, check_interval=3)),  # two x tiles, odd ny
    ((17, 17, 17), dict(tolerance=1e-2)),                     # early stop, odd iterate
    ((250, 30, 40), dict(max_iterations=25)),                 # 3x3 one-pass tiles, z chunks
])
def test_poisson_relax_fused_loop_bitwise(hip_lib, method, shape, kw):
    """The device loop (one-pass RB k_rb1 or the two colour sweeps of k_rx,
    lagged residual, ping-pong buffers) and the host two-pass form all equal
    the oracle bit for bit: iterate, iteration
    count (max_iterations + 1 when capped, linear_solver.c:472), status,
    initial and final residual."""
    nx, ny, nz = shape
    rng = np.random.default_rng(nx * 7 + nz)
    rhs = rng.standard_normal((nz, ny, nx))
    x0 = 0.1 * rng.standard_normal((nz, ny, nx))
    d = 1.0 / (nx - 1)
    dz = 1.0 / (nz - 1) if nz > 1 else 0.0
    base = dict(max_iterations=3000 if method == A.HIP_POISSON_JACOBI else 2000)
    base.update(kw)
    prm = oracle.poisson_params(**base)
    xo = x0.copy()
    if method == A.HIP_POISSON_REDBLACK:
        so, sto = oracle.redblack_solve(xo, rhs, d, d, dz, prm)
    else:
        so, sto = oracle.jacobi_solve(xo, rhs, d, d, dz, prm)
    for two_pass in (0, 1, 2):  # one-pass RB (3-D) / host two-pass / device two-colour
        ctx = api.HipProjection(nx, ny, nz, relax_two_pass=two_pass)
        xh = x0.copy()
        sh, sth = ctx.poisson_solve(method, xh, rhs, d, d, dz, prm)
        ctx.close()
        assert sh == so, two_pass
        assert (sth.iterations, sth.status) == (sto.iterations, sto.status), two_pass
        assert sth.initial_residual == sto.initial_residual
        assert sth.final_residual == sto.final_residual
        np.testing.assert_array_equal(xh, xo)


def test_poisson_relax_initially_converged(hip_lib):
    """linear_solver.c:429-437: residual below the absolute tolerance before
    the loop -> 0 iterations, x untouched."""
    g, rhs = cases.cos_rhs(17)
    prm = oracle.poisson_params(absolute_tolerance=1e6)
    ctx = api.HipProjection(17, 17, 17)
    x = np.full_like(rhs, 0.25)
    sh, sth = ctx.poisson_solve(A.HIP_POISSON_REDBLACK, x, rhs, g.dx, g.dy, g.dz, prm)
    ctx.close()
    assert sh == A.CFD_SUCCESS and sth.iterations == 0 and sth.status == A.POISSON_CONVERGED
    assert np.all(x == 0.25)


def test_deterministic(hip_lib):
    """Fixed-order reductions: two runs are bitwise identical."""
    g, f, p = cases.tg3(33)
    outs = []
    for _ in range(2):
        fh = _clone(g, f)
        ctx = api.HipProjection(33, 33, 33)
        for _ in range(3):
            cases.tg3_bc(fh)
            assert ctx.step(fh, g, p) == A.CFD_SUCCESS
        outs.append(_fields(fh))
        ctx.close()
    for k in outs[0]:
        np.testing.assert_array_equal(outs[0][k], outs[1][k], err_msg=k)


def test_unsupported_source_callback(hip_lib):
    g, f, p = cases.kat_2d()
    cb = A.SourceFunc(lambda *a: None)
    p.source_func = C.cast(cb, C.c_void_p)
    ctx = api.HipProjection(16, 16, 1)
    before = _fields(f)
    assert ctx.step(f, g, p) == A.CFD_ERROR_UNSUPPORTED
    for k, v in before.items():
        np.testing.assert_array_equal(getattr(f, k), v)
    ctx.close()


def test_max_iter_failure_leaves_field(hip_lib):
    """A pressure solve that cannot converge returns CFD_ERROR_MAX_ITER and leaves
    the caller's field untouched (solver_projection.c:220-224)."""
    g, f, p = cases.tg3(17)
    ctx = api.HipProjection(17, 17, 17, poisson_max_iter=2)
    before = _fields(f)
    assert ctx.step(f, g, p) == A.CFD_ERROR_MAX_ITER
    for k, v in before.items():
        np.testing.assert_array_equal(getattr(f, k), v)
    ctx.close()


@pytest.mark.parametrize("where", [(0, 0, 0), (3, 4, 5)])
def test_nonfinite_input_status_matches_oracle(hip_lib, where):
    """A NaN on the boundary survives the step -> CFD_ERROR_DIVERGED
    (solver_projection.c:281-289); an interior NaN is absorbed by the +-100
    velocity clamp (fmin(100, NaN) = 100, :180-182) exactly as in the reference."""
    g, f, p = cases.tg3(17)
    f.u[where] = float("nan")
    fo = _clone(g, f)
    ctx = api.HipProjection(17, 17, 17)
    s = ctx.step(f, g, p)
    so, _, _ = oracle.projection_step(fo, g, p)
    assert s == so
    assert s == (A.CFD_ERROR_DIVERGED if where == (0, 0, 0) else A.CFD_SUCCESS)
    if s == A.CFD_SUCCESS:
        for k in ("u", "v", "w", "p"):
            assert _rel_maxdiff(getattr(f, k), getattr(fo, k)) <= CG_FIELD_RTOL, k
    ctx.close()


def test_device_resident_matches_host_path(hip_lib):
    """upload / step_device x N / download equals N host-buffer steps."""
    g, f, p = cases.cavity(33, 33, 33, Re=100.0, dt=5e-4)
    api.cavity_bc(f, 1.0)
    fa = _clone(g, f)
    fb = _clone(g, f)
    ca = api.HipProjection(33, 33, 33)
    cb = api.HipProjection(33, 33, 33)
    for _ in range(3):
        assert ca.step(fa, g, p) == A.CFD_SUCCESS
    cb.upload(fb)
    for _ in range(3):
        assert cb.step_device(g, p) == A.CFD_SUCCESS
    cb.download(fb)
    for k in ("u", "v", "w", "p"):
        np.testing.assert_array_equal(getattr(fa, k), getattr(fb, k), err_msg=k)
    ca.close()
    cb.close()


def test_tg3d_16_l2_matches_reference(hip_lib):
    """Taylor-Green 3-D 16^3, 100 steps through projection_hip: relative L2 error
    of the reference build, 5.336557e-02."""
    g, f, p = cases.tg3(16)
    reg = api.Registry()
    s = reg.create("projection_hip")
    assert s.init(g, p) == A.CFD_SUCCESS
    for _ in range(100):
        cases.tg3_bc(f)
        assert s.step(f, g, p) == A.CFD_SUCCESS
    eu, ev = cases.tg3_l2_errors(g, f, 100 * 1e-3)
    assert eu == pytest.approx(5.336557e-02, rel=2e-6)
    assert ev == pytest.approx(5.336557e-02, rel=2e-6)
    s.close()


def test_ghia_33_re100_device_resident(hip_lib):
    """33x33 cavity, Re=100, 5000 steps of dt=5e-4: Ghia RMS_u = 0.0382 as the
    reference (docs/validation/cavity-backends-validation.md:115) and within the
    reference's 0.001 backend-consistency tolerance of the oracle
    (test_cavity_backends.c:43)."""
    from tests import ghia
    g, f, p = cases.cavity(33, 33, 1, Re=100.0, dt=5e-4)
    api.cavity_bc(f, 1.0)
    ctx = api.HipProjection(33, 33, 1)
    ctx.upload(f)
    for _ in range(5000):
        assert ctx.step_device(g, p) == A.CFD_SUCCESS
    ctx.download(f)
    rms_u, rms_v = ghia.rms_errors(f, g, 100)
    assert round(rms_u, 4) == 0.0382
    assert abs(rms_v - 0.0440) < 0.001
    ctx.close()


def test_tg3d_32_device_resident_l2_vs_oracle(hip_lib):
    """BASELINE configs[1] at test size: Taylor-Green 32^3, 100 steps, fields
    resident in HBM with the periodic BCs applied on the device before every
    step. The relative L2 errors against the analytic decay match the oracle's
    to 1e-9 (CG dot order only) and pass the reference's TG3_L2_ERROR_TOL =
    0.25 (taylor_green_3d_reference.h:58)."""
    g, f, p = cases.tg3(32)
    ctx = api.HipProjection(32, 32, 32)
    ctx.upload(f)
    for _ in range(100):
        for fid in (A.HIP_FIELD_U, A.HIP_FIELD_V, A.HIP_FIELD_W, A.HIP_FIELD_P):
            ctx.apply_scalar_bc(fid, A.BC_TYPE_PERIODIC)
        assert ctx.step_device(g, p) == A.CFD_SUCCESS, api._native.last_error()
    ctx.download(f)
    ctx.close()
    eu, ev = cases.tg3_l2_errors(g, f, 100 * 1e-3)
    go, fo, po = cases.tg3(32)
    for _ in range(100):
        cases.tg3_bc(fo)
        assert oracle.projection_step(fo, go, po)[0] == A.CFD_SUCCESS
    eo_u, eo_v = cases.tg3_l2_errors(go, fo, 100 * 1e-3)
    assert eu == pytest.approx(eo_u, rel=1e-9) and ev == pytest.approx(eo_v, rel=1e-9)
    assert eu < 0.25 and ev < 0.25
