"""Host-side mirror (libcfd_host.so) against the oracle's restatement of the
reference boundary conditions and grid (CPU only)."""
import math

import numpy as np
import pytest

from cfd_amd import _abi as A
from cfd_amd import api
from oracle import oracle


@pytest.mark.parametrize("shape", [(16, 16, 1), (17, 13, 11)])
@pytest.mark.parametrize("bc", [A.BC_TYPE_NEUMANN, A.BC_TYPE_PERIODIC])
def test_scalar_bc_matches_oracle(shape, bc):
    nx, ny, nz = shape
    a = np.random.default_rng(3).standard_normal((nz, ny, nx))
    b = a.copy()
    api.bc_apply_scalar_3d(a, bc)
    (oracle.bc_neumann if bc == A.BC_TYPE_NEUMANN else oracle.bc_periodic)(b)
    np.testing.assert_array_equal(a, b)


def test_bc_as_gather_map():
    """The composition of the reference's x->y->z face copies equals a per-axis
    index map (the form the device kernel uses): Neumann clamps, periodic wraps."""
    nx, ny, nz = 7, 6, 5
    a = np.random.default_rng(4).standard_normal((nz, ny, nx))
    for kind, fn in (("neumann", oracle.bc_neumann), ("periodic", oracle.bc_periodic)):
        b = a.copy()
        fn(b)

        def m(c, n):
            if kind == "neumann":
                return 1 if c == 0 else (n - 2 if c == n - 1 else c)
            return n - 2 if c == 0 else (1 if c == n - 1 else c)

        want = np.empty_like(a)
        for k in range(nz):
            for j in range(ny):
                for i in range(nx):
                    want[k, j, i] = a[m(k, nz), m(j, ny), m(i, nx)]
        np.testing.assert_array_equal(b, want)


def test_dirichlet_face_precedence():
    a = np.zeros((5, 6, 7))
    b = a.copy()
    v = api.dirichlet(1, 2, 3, 4, 5, 6)
    api._native.host().bc_apply_dirichlet_scalar_3d(a.ctypes.data_as(A.c_double_p), 7, 6, 5, 42,
                                                     v)
    oracle.bc_dirichlet(b, v)
    np.testing.assert_array_equal(a, b)
    assert a[0, 0, 0] == 6.0 and a[4, 5, 6] == 5.0 and a[2, 0, 0] == 4.0 and a[2, 3, 0] == 1.0


def test_grid_uniform_matches_reference_formula():
    g = api.Grid(9, 5, 4, 0.0, 2.0, -1.0, 1.0, 0.0, 0.5)
    dx = (2.0 - 0.0) / 8
    assert g.dx == dx and g.x[8] == 0.0 + 8 * dx
    assert g.stride_z == 45 and g.c.k_start == 1 and g.c.k_end == 3
    assert g.c.inv_dz2 == 1.0 / (g.dz * g.dz)


def test_params_default():
    p = api.params_default()
    assert (p.dt, p.mu, p.max_iter, p.source_amplitude_u) == (0.001, 0.01, 100, 0.1)
    assert p.alpha == 0.0 and not p.source_func


def test_error_strings():
    assert api.status_name(A.CFD_ERROR_MAX_ITER) == "Max iterations reached"
    assert api.status_name(A.CFD_ERROR_DIVERGED) == "NSSolver diverged"
