"""The one-pass Red-Black SOR kernel (k_rb1) against the oracle on shapes
that exercise its tiling -- partial x and y tiles, z chunks, odd extents,
early stops, the three tile widths -- bit for bit: iterate, iteration count, status, initial and
final L-inf residual (linear_solver_redblack.c:80-147,
linear_solver.c:397-485)."""
import numpy as np
import pytest

from cfd_amd import _abi as A
from cfd_amd import api
from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape,kw", [
    ((17, 17, 17), dict(tolerance=1e-2)),
    ((130, 20, 9), dict(max_iterations=40, check_interval=3)),
    ((250, 30, 40), dict(max_iterations=25)),
    ((131, 27, 70), dict(max_iterations=12)),
    ((126, 14, 5), dict(max_iterations=30, check_interval=2)),
    ((255, 50, 140), dict(max_iterations=6)),
    ((63, 70, 12), dict(max_iterations=9)),
    # nx = 124 T + 1: no remainder strip (the full tiles store every pair)
    ((249, 21, 10), dict(max_iterations=11)),
    ((250, 21, 10), dict(max_iterations=11)),
])
@pytest.mark.parametrize("tc", ["64", "32", "16"])
def test_rb_one_pass_bitwise(hip_lib, shape, kw, tc, monkeypatch):
    """Every tile width (TC x pairs by 1024 / TC rows), forced through
    CFD_HIP_RB1_TC, on every shape."""
    monkeypatch.setenv("CFD_HIP_RB1_TC", tc)
    nx, ny, nz = shape
    rng = np.random.default_rng(nx * 7 + nz)
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
    assert sh == so
    assert (sth.iterations, sth.status) == (sto.iterations, sto.status)
    assert sth.initial_residual == sto.initial_residual
    assert sth.final_residual == sto.final_residual
    np.testing.assert_array_equal(xh, xo)
