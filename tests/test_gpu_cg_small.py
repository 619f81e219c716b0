"""The persistent small-grid CG (k_cg_small: the whole solve in one
cooperative launch) against the sweep kernels and the oracle. Same per-cell
arithmetic as the sweeps; only the dot-product summation order differs, so
the bar is the CG one: iteration counts within 1, solutions within 1e-10
relative (linear_solver_cg.c:290-461 is the reference loop)."""
import numpy as np
import pytest

from cfd_amd import _abi as A
from cfd_amd import api
from oracle import oracle
from tests import cases

pytestmark = pytest.mark.gpu


def _solve(shape, rhs, d, small, monkeypatch, prm=None):
    monkeypatch.setenv("CFD_HIP_CG_SMALL", "1" if small else "0")
    nx, ny, nz = shape
    ctx = api.HipProjection(nx, ny, nz)
    ctx.reset_timing()
    ctx.enable_timing(True)
    x = np.zeros((nz, ny, nx))
    s, st = ctx.poisson_solve(A.HIP_POISSON_CG, x, rhs, d[0], d[1], d[2], prm)
    kt = ctx.timing()
    ctx.close()
    return s, st, x, kt


@pytest.mark.parametrize("shape", [(65, 65, 1), (128, 128, 1), (17, 17, 17), (40, 30, 20)])
def test_cg_small_matches_sweeps_and_oracle(hip_lib, shape, monkeypatch):
    nx, ny, nz = shape
    rng = np.random.default_rng(nx * ny + nz)
    rhs = np.zeros((nz, ny, nx))
    if nz > 1:
        rhs[1:-1, 1:-1, 1:-1] = rng.standard_normal((nz - 2, ny - 2, nx - 2))
    else:
        rhs[0, 1:-1, 1:-1] = rng.standard_normal((ny - 2, nx - 2))
    d = (1.0 / (nx - 1), 1.0 / (ny - 1), (1.0 / (nz - 1)) if nz > 1 else 0.0)
    s0, st0, x0, kt0 = _solve(shape, rhs, d, False, monkeypatch)
    s1, st1, x1, kt1 = _solve(shape, rhs, d, True, monkeypatch)
    assert kt1["cg_small"][1] == 1 and kt0["cg_small"][1] == 0
    assert kt1["cg_sweep_a"][1] == 0
    assert s1 == s0 == A.CFD_SUCCESS
    assert abs(st1.iterations - st0.iterations) <= 1
    assert st1.initial_residual == st0.initial_residual
    scale = np.max(np.abs(x0))
    assert np.max(np.abs(x1 - x0)) / scale < 1e-10
    xo = np.zeros_like(rhs)
    so, sto = oracle.cg_solve(xo, rhs, *d)
    assert abs(st1.iterations - sto.iterations) <= 1
    assert np.max(np.abs(x1 - xo)) / np.max(np.abs(xo)) < 1e-9


def test_cg_small_max_iter_and_stats(hip_lib, monkeypatch):
    """A capped solve: the same status, iteration count and residuals as the
    sweep path (linear_solver_cg.c:437-459)."""
    g, rhs = cases.cos_rhs(33, nz=1)
    prm = oracle.poisson_params(max_iterations=7)
    d = (g.dx, g.dy, 0.0)
    s0, st0, x0, _ = _solve((33, 33, 1), rhs, d, False, monkeypatch, prm)
    s1, st1, x1, _ = _solve((33, 33, 1), rhs, d, True, monkeypatch, prm)
    assert s0 == s1 == A.CFD_ERROR_MAX_ITER
    assert st0.iterations == st1.iterations == 7
    assert st1.status == st0.status
    assert st1.final_residual == pytest.approx(st0.final_residual, rel=1e-10)
    np.testing.assert_allclose(x1, x0, rtol=0, atol=1e-12 * np.max(np.abs(x0)))


def test_cg_small_cavity_steps_vs_oracle(hip_lib, monkeypatch):
    """configs[0]'s path (2-D cavity steps through the plugin's host-buffer
    step, small CG by default) against the oracle: fields within 1e-10, CG
    iterations within 1 per step, and the small solve actually taken."""
    from tests.test_gpu_parity import _clone
    monkeypatch.delenv("CFD_HIP_CG_SMALL", raising=False)
    g, f, p = cases.cavity(64, 64, 1, Re=1000.0, dt=5e-4)
    fo = _clone(g, f)
    fh = _clone(g, f)
    ctx = api.HipProjection(g.nx, g.ny, g.nz)
    ctx.reset_timing()
    ctx.enable_timing(True)
    for _ in range(5):
        api.cavity_bc(fo, 1.0)
        api.cavity_bc(fh, 1.0)
        so, sto, io = oracle.projection_step(fo, g, p, A.ORACLE_POISSON_CG)
        sth = A.SolverStats()
        assert so == A.CFD_SUCCESS
        assert ctx.step(fh, g, p, sth) == A.CFD_SUCCESS
        assert abs(ctx.poisson_stats().iterations - io) <= 1
    assert ctx.timing()["cg_small"][1] == 5
    ctx.close()
    for k in ("u", "v", "p"):
        ref = getattr(fo, k)
        scale = max(1.0, float(np.max(np.abs(ref))))
        assert float(np.max(np.abs(getattr(fh, k) - ref))) / scale <= 1e-10, k


def _fold_problem():
    nx, ny, nz = 40, 30, 20
    rng = np.random.default_rng(4)
    rhs = np.zeros((nz, ny, nx))
    rhs[1:-1, 1:-1, 1:-1] = rng.standard_normal((nz - 2, ny - 2, nx - 2))
    return (nx, ny, nz), rhs, (1.0 / (nx - 1), 1.0 / (ny - 1), 1.0 / (nz - 1))


def _match_oracle_x(x, prm, rhs, d):
    xo = np.zeros_like(rhs)
    so, sto = oracle.cg_solve(xo, rhs, *d, prm)
    assert np.max(np.abs(x - xo)) / np.max(np.abs(xo)) < 1e-10
    return so, sto


@pytest.mark.parametrize("max_iter", [1, 3, 4, 5, 7, 8, 9, 12])
def test_sweep_cg_fold_boundaries_capped(hip_lib, monkeypatch, max_iter):
    """The sweep path folds x += alpha p every fourth iteration (in sweep A of
    it = 4m) and k_cg_finalize applies what is pending when the loop stops:
    1..4 updates depending on max_iter mod 4. A capped solve at every
    residue class against the oracle's sequential updates
    (linear_solver_cg.c:379-380,437-459): same status and count, x 1e-10."""
    shape, rhs, d = _fold_problem()
    prm = oracle.poisson_params(max_iterations=max_iter)
    s, st, x, kt = _solve(shape, rhs, d, False, monkeypatch, prm)
    assert kt["cg_small"][1] == 0
    so, sto = _match_oracle_x(x, prm, rhs, d)
    assert s == so == A.CFD_ERROR_MAX_ITER
    assert st.iterations == sto.iterations == max_iter
    assert st.final_residual == pytest.approx(sto.final_residual, rel=1e-9)


@pytest.mark.parametrize("residue", [0, 1, 2, 3])
def test_sweep_cg_fold_boundaries_converged(hip_lib, monkeypatch, residue):
    """Convergence (not a cap) after a chosen iteration count in each residue
    class mod 4: the relative tolerance is placed between the oracle's
    residual after m iterations, a new minimum, and the smallest one before
    it, so both solvers stop at m."""
    shape, rhs, d = _fold_problem()
    res = {}
    for m in range(1, 40):
        xo = np.zeros_like(rhs)
        _, sto = oracle.cg_solve(xo, rhs, *d, oracle.poisson_params(max_iterations=m))
        res[m] = sto.final_residual
        res0 = sto.initial_residual
    pick = None
    for m in range(8, 40):
        prev = min(res[q] for q in range(1, m))
        if m % 4 == residue and res[m] < prev / 1.05:
            pick = (m, float(np.sqrt(res[m] * prev)) / res0)
            break
    assert pick is not None, res
    m, rel = pick
    prm = oracle.poisson_params(tolerance=rel, absolute_tolerance=0.0, max_iterations=1000)
    s, st, x, _ = _solve(shape, rhs, d, False, monkeypatch, prm)
    so, sto = _match_oracle_x(x, prm, rhs, d)
    assert s == so == A.CFD_SUCCESS
    assert st.iterations == sto.iterations == m
