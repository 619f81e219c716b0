"""BASELINE.json's largest single-device configuration, 1024x1024x512
(config 5's grid: 4.3 GB per field, byte offsets beyond 2^32), checked through
size-independent properties the oracle cannot reach at this size:

  - scale equivariance: with x0 = 0, a zero absolute tolerance and a
    power-of-two factor c, every operation of CG / RB-SOR / Jacobi scales
    exactly, so solve(c * rhs) == c * solve(rhs) bit for bit with the same
    iteration count (a wrong index or a race at large offsets breaks it);
  - agreement with a restatement on the host of one Jacobi sweep in numpy
    (same expression order), on a few planes at the far end of the grid.
"""
import numpy as np
import pytest

from cfd_amd import _abi as A
from cfd_amd import api
from oracle import oracle

pytestmark = pytest.mark.gpu

NX, NY, NZ = 1024, 1024, 512


def _rhs():
    d = 1.0 / (NX - 1)
    x = np.arange(NX) * d
    z = np.arange(NZ) * (1.0 / (NZ - 1))
    rhs = np.empty((NZ, NY, NX))
    rhs[...] = np.cos(np.pi * x)[None, None, :]
    rhs *= np.cos(np.pi * x[:NY])[None, :, None]
    rhs *= (np.cos(np.pi * z) + 0.25)[:, None, None]
    return rhs, d, 1.0 / (NZ - 1)


@pytest.fixture(scope="module")
def big():
    ctx = api.HipProjection(NX, NY, NZ)
    rhs, d, dz = _rhs()
    yield ctx, rhs, d, dz
    ctx.close()


@pytest.mark.parametrize("method,iters", [(A.HIP_POISSON_CG, 9), (A.HIP_POISSON_REDBLACK, 3),
                                          (A.HIP_POISSON_JACOBI, 2)])
def test_max_size_scale_equivariance(hip_lib, big, method, iters):
    ctx, rhs, d, dz = big
    prm = oracle.poisson_params(tolerance=0.0, absolute_tolerance=0.0, max_iterations=iters)
    x1 = np.zeros((NZ, NY, NX))
    s1, st1 = ctx.poisson_solve(method, x1, rhs, d, d, dz, prm)
    x2 = np.zeros((NZ, NY, NX))
    s2, st2 = ctx.poisson_solve(method, x2, 4.0 * rhs, d, d, dz, prm)
    assert s1 == s2 == A.CFD_ERROR_MAX_ITER
    assert st1.iterations == st2.iterations
    assert st2.final_residual == 4.0 * st1.final_residual
    assert np.isfinite(x1).all() and np.abs(x1).max() > 0
    np.testing.assert_array_equal(x2, 4.0 * x1)


def test_max_size_jacobi_sweep_far_planes(hip_lib, big):
    """One Jacobi iteration from x0 = 0 is x = -rhs * inv_factor on the interior
    (linear_solver_jacobi.c:92-109 with zero neighbours), then the Neumann BC:
    checked on the last interior planes, where offsets exceed 2^32 bytes."""
    ctx, rhs, d, dz = big
    prm = oracle.poisson_params(tolerance=0.0, absolute_tolerance=0.0, max_iterations=1)
    x = np.zeros((NZ, NY, NX))
    ctx.poisson_solve(A.HIP_POISSON_JACOBI, x, rhs, d, d, dz, prm)
    dx2 = d * d
    inv_dz2 = 1.0 / (dz * dz)
    inv_factor = 1.0 / (2.0 * (1.0 / dx2 + 1.0 / dx2 + inv_dz2))
    zero = 0.0
    ks = slice(NZ - 4, NZ - 1)
    exp = -(rhs[ks, 1:-1, 1:-1] - (zero + zero) / dx2 - (zero + zero) / dx2 -
            (zero + zero) * inv_dz2) * inv_factor
    np.testing.assert_array_equal(x[NZ - 4:NZ - 1, 1:-1, 1:-1][:3], exp)
    np.testing.assert_array_equal(x[NZ - 1], x[NZ - 2])          # z face: Neumann
    np.testing.assert_array_equal(x[NZ - 2, :, NX - 1], x[NZ - 2, :, NX - 2])
