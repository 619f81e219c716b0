"""The oracle with a caller apply_bc override (oracle_set_poisson_bc_hook)
against the gates of tests/math/test_poisson_3d.c (:329-371 L2 < 1e-2 at
17^3, :600-627 O(h^2) for CG, :633-675 cross-solver 1e-4), so the checker
tests/test_gpu_poisson_3d.py compares the GPU backend with is itself pinned
by the reference test's own bars. CPU only."""
import math

import pytest

from cfd_amd import _abi as A
from tests.test_gpu_poisson_3d import (L2_ERROR_TOL, METHODS, N3D, SOLVER_COMPARE_TOL, Problem,
                                       oracle_solve)


def test_oracle_3d_sinusoidal_gates():
    pb = Problem(N3D, N3D)
    errs = []
    for m in METHODS:
        s, st, x = oracle_solve(m, pb, pb.dirichlet)
        assert s == A.CFD_SUCCESS and st.status == A.POISSON_CONVERGED, (m, s)
        errs.append(pb.l2(x))
    assert all(e < L2_ERROR_TOL for e in errs), errs
    assert all(abs(e - errs[0]) < SOLVER_COMPARE_TOL for e in errs[1:]), errs


def test_oracle_grid_convergence_cg():
    errs, hs = [], []
    for n in (9, 17, 33):
        pb = Problem(n, n)
        s, _, x = oracle_solve(A.POISSON_METHOD_CG, pb, pb.dirichlet)
        assert s == A.CFD_SUCCESS
        errs.append(pb.l2(x))
        hs.append(pb.dx)
    for a in (1, 2):
        assert math.log(errs[a - 1] / errs[a]) / math.log(hs[a - 1] / hs[a]) > 1.7, errs


@pytest.mark.parametrize("method", [A.POISSON_METHOD_CG, A.POISSON_METHOD_JACOBI])
def test_oracle_nz1_2d(method):
    pb = Problem(33, 1)
    s, _, x = oracle_solve(method, pb, pb.dirichlet)
    assert s == A.CFD_SUCCESS and pb.l2(x) < L2_ERROR_TOL


def test_oracle_hook_cleared():
    """After a hooked solve the default Neumann BC is back: a plain solve
    ends with equal first and second planes (cg.c:447 Neumann)."""
    import numpy as np
    from oracle import oracle
    pb = Problem(9, 9)
    oracle_solve(A.POISSON_METHOD_CG, pb, pb.dirichlet)
    x = np.zeros(pb.shape)
    rhs = np.ascontiguousarray(pb.rhs - pb.rhs[1:-1, 1:-1, 1:-1].mean())
    oracle.cg_solve(x, rhs, pb.dx, pb.dy, pb.dz, oracle.poisson_params(max_iterations=5))
    np.testing.assert_array_equal(x[0], x[1])
    np.testing.assert_array_equal(x[:, :, 0], x[:, :, 1])
