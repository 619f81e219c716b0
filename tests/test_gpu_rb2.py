"""Two RB-SOR iterations per sweep (k_rb2, cfd_amd/csrc/hip/rb2.hpp) against
the oracle, bit for bit: iterate, iteration count, status, initial and final
L-inf residual (linear_solver_redblack.c:80-147 driven by
linear_solver.c:397-485).

Every host path of relax_solve_rb2 is forced in turn:
  CFD_HIP_RB2 = 2            the reference's arithmetic in the sweep
  CFD_HIP_RB2 = 1            certified fast arithmetic (the product)
  + CFD_HIP_RB2_TEST = 1     every approximate decision ambiguous: the host
                             resolves each iterate's residual exactly
  + CFD_HIP_RB2_TEST = 2     every sweep uncertified: the host reruns with
                             one iteration per sweep (k_rb1)
  + CFD_HIP_RB2_TEST = 3     every SOR update takes the in-kernel exact
                             recompute (the path of tiny neighbour sums)
and the loop stops on both the input and the middle iterate of a sweep
(odd and even iteration counts, converged and capped)."""
import numpy as np
import pytest

from cfd_amd import api
from cfd_amd import _abi as A
from oracle import oracle

pytestmark = pytest.mark.gpu

SHAPES = [
    ((17, 17, 17), dict(tolerance=1e-2)),
    ((130, 20, 9), dict(max_iterations=40)),
    ((130, 20, 9), dict(max_iterations=41)),
    ((250, 30, 40), dict(max_iterations=25)),
    ((131, 27, 70), dict(max_iterations=12)),
    ((63, 70, 12), dict(max_iterations=9)),
    ((57, 25, 7), dict(tolerance=1e-3)),
    ((58, 26, 8), dict(tolerance=3e-3)),
    ((120, 49, 33), dict(max_iterations=2)),
    ((120, 49, 33), dict(max_iterations=1)),
]
MODES = [("2", "0"), ("1", "0"), ("1", "1"), ("1", "2"), ("1", "3")]


def _solve(shape, kw):
    nx, ny, nz = shape
    rng = np.random.default_rng(nx * 7 + nz * 3 + ny)
    rhs = rng.standard_normal((nz, ny, nx))
    x0 = 0.1 * rng.standard_normal((nz, ny, nx))
    d = 1.0 / (nx - 1)
    dz = 1.0 / (nz - 1)
    base = dict(max_iterations=2000)
    base.update(kw)
    prm = oracle.poisson_params(**base)
    xo = x0.copy()
    so, sto = oracle.redblack_solve(xo, rhs, d, d, dz, prm)
    ctx = api.HipProjection(nx, ny, nz)
    xh = x0.copy()
    sh, sth = ctx.poisson_solve(A.HIP_POISSON_REDBLACK, xh, rhs, d, d, dz, prm)
    ctx.close()
    return (so, sto, xo), (sh, sth, xh)


@pytest.mark.parametrize("shape,kw", SHAPES)
@pytest.mark.parametrize("mode,knob", MODES)
def test_rb2_bitwise(hip_lib, monkeypatch, shape, kw, mode, knob):
    monkeypatch.setenv("CFD_HIP_RB2", mode)
    monkeypatch.setenv("CFD_HIP_RB2_TEST", knob)
    (so, sto, xo), (sh, sth, xh) = _solve(shape, kw)
    assert sh == so
    assert (sth.iterations, sth.status) == (sto.iterations, sto.status)
    assert sth.initial_residual == sto.initial_residual
    assert sth.final_residual == sto.final_residual
    np.testing.assert_array_equal(xh, xo)


def test_rb2_stops_on_both_iterates(hip_lib, monkeypatch):
    """Converged solves whose iteration count is odd and even both occur
    in SHAPES' converging cases (the loop decides on a sweep's input or on
    its middle iterate); checked here so a shape change cannot lose one."""
    monkeypatch.setenv("CFD_HIP_RB2", "1")
    seen = set()
    for shape, kw in SHAPES:
        if "tolerance" not in kw:
            continue
        (_, sto, _), _ = _solve(shape, kw)
        if sto.status == 0:
            seen.add(sto.iterations % 2)
    assert seen == {0, 1}, seen


@pytest.mark.parametrize("mode", ["1", "2"])
@pytest.mark.parametrize("iters", [30, 31])
def test_rb2_tiny_front_bitwise(hip_lib, monkeypatch, mode, iters):
    """A solve from x0 = 0 with a right-hand side of 1e-262 in one corner and
    zero tolerances: the iterate's front decays to values far below 2^-899
    (about 22 000 cells at 30 iterations), whose neighbour sums the fast
    division must not take -- those waves recompute their update exactly
    (rb2.hpp rb2_sorc); bitwise against the oracle, capped at an even and an
    odd iteration."""
    monkeypatch.setenv("CFD_HIP_RB2", mode)
    nx, ny, nz = 96, 80, 70
    rhs = np.zeros((nz, ny, nx))
    rhs[2:6, 2:6, 2:6] = 1e-262
    x0 = np.zeros_like(rhs)
    d = 1.0 / (nx - 1)
    prm = oracle.poisson_params(max_iterations=iters, tolerance=0.0, absolute_tolerance=0.0)
    xo = x0.copy()
    so, sto = oracle.redblack_solve(xo, rhs, d, d, d, prm)
    nzv = np.abs(xo[xo != 0])
    assert int((nzv < 2.0 ** -899).sum()) > 1000  # the front really is that small
    ctx = api.HipProjection(nx, ny, nz)
    xh = x0.copy()
    sh, sth = ctx.poisson_solve(A.HIP_POISSON_REDBLACK, xh, rhs, d, d, d, prm)
    ctx.close()
    assert sh == so
    assert (sth.iterations, sth.status) == (sto.iterations, sto.status)
    assert sth.initial_residual == sto.initial_residual
    assert sth.final_residual == sto.final_residual
    np.testing.assert_array_equal(xh, xo)


@pytest.mark.parametrize("iters", [5, 6])
def test_rb2_uncertified_input_bitwise(hip_lib, monkeypatch, capfd, iters):
    """An initial guess with one interior value above the certified range
    (|v| > 2^800): the first two-iteration sweep certifies its input X by the
    k_rb2_xmax pre-pass (r06; the march no longer certifies X itself), fails,
    and the host reruns with one iteration per sweep (k_rb1); bitwise against
    the oracle, and the launch log shows the uncertified stop."""
    monkeypatch.setenv("CFD_HIP_RB2", "1")
    monkeypatch.setenv("CFD_HIP_RB2_LOG", "1")
    nx, ny, nz = 70, 66, 40
    rng = np.random.default_rng(11)
    rhs = rng.standard_normal((nz, ny, nx))
    x0 = 0.1 * rng.standard_normal((nz, ny, nx))
    x0[20, 30, 35] = 1e245  # 2^800 ~ 6.7e240
    d = 1.0 / (nx - 1)
    prm = oracle.poisson_params(max_iterations=iters, tolerance=0.0, absolute_tolerance=0.0)
    xo = x0.copy()
    so, sto = oracle.redblack_solve(xo, rhs, d, d, d, prm)
    assert np.isfinite(xo).all()
    ctx = api.HipProjection(nx, ny, nz)
    xh = x0.copy()
    sh, sth = ctx.poisson_solve(A.HIP_POISSON_REDBLACK, xh, rhs, d, d, d, prm)
    ctx.close()
    assert sh == so
    assert (sth.iterations, sth.status) == (sto.iterations, sto.status)
    assert sth.initial_residual == sto.initial_residual
    assert sth.final_residual == sto.final_residual
    np.testing.assert_array_equal(xh, xo)
    err = capfd.readouterr().err
    assert "1 uncertified" in err, err[-2000:]
