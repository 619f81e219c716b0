"""State carried between calls on one hip_proj context: mixing integrators,
density updates and restart files."""
import os
import tempfile

import numpy as np
import pytest

from cfd_amd import _abi as A
from cfd_amd import api
from oracle import oracle
from tests import cases

pytestmark = pytest.mark.gpu

C = api.C


def _rk4_device(ctx, g, p):
    return ctx._lib().hip_rk4_step_device(ctx.ctx, g.ptr, C.byref(p), C.byref(A.SolverStats()))


def test_projection_after_rk4_on_one_context(hip_lib):
    """RK4 borrows the CG work arrays as stage buffers (rk4_hip.hip) and leaves
    wall values in them; a projection step on the same context afterwards must
    equal the step of a fresh context on the same state (bitwise: same kernels,
    same reduction order)."""
    n = 17
    g, f, p = cases.tg3(n)
    ids = {"u": A.HIP_FIELD_U, "v": A.HIP_FIELD_V, "w": A.HIP_FIELD_W, "p": A.HIP_FIELD_P,
           "rho": A.HIP_FIELD_RHO}
    a = api.HipProjection(n, n, n)
    for k, i in ids.items():
        a.set_field(i, getattr(f, k))
    for _ in range(2):
        assert _rk4_device(a, g, p) == A.CFD_SUCCESS, api._native.last_error()
    state = {k: a.get_field(i) for k, i in ids.items()}
    for fid in (A.HIP_FIELD_U, A.HIP_FIELD_V, A.HIP_FIELD_W, A.HIP_FIELD_P):
        a.apply_scalar_bc(fid, A.BC_TYPE_PERIODIC)
    assert a.step_device(g, p) == A.CFD_SUCCESS, api._native.last_error()
    it_a = a.poisson_stats().iterations
    got = {k: a.get_field(ids[k]) for k in ("u", "v", "w", "p")}
    a.close()

    b = api.HipProjection(n, n, n)
    for k in ("u", "v", "w", "p"):
        b.set_field(ids[k], state[k])
    b.set_density(1.0)
    for fid in (A.HIP_FIELD_U, A.HIP_FIELD_V, A.HIP_FIELD_W, A.HIP_FIELD_P):
        b.apply_scalar_bc(fid, A.BC_TYPE_PERIODIC)
    assert b.step_device(g, p) == A.CFD_SUCCESS
    assert b.poisson_stats().iterations == it_a
    want = {k: b.get_field(ids[k]) for k in ("u", "v", "w", "p")}
    b.close()
    for k in want:
        np.testing.assert_array_equal(got[k], want[k], err_msg=k)


def test_set_density_refreshes_per_cell_density(hip_lib):
    """Once a per-cell density exists (RK4 created it), set_density and upload
    keep it equal to the new value; RK4 then matches the oracle on that rho."""
    n = (13, 11, 9)
    g = api.Grid(*n, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0)
    f = api.FlowField(*n)
    rng = np.random.default_rng(3)
    for k in ("u", "v", "w"):
        getattr(f, k)[...] = 0.05 * rng.standard_normal(f.u.shape)
    f.p[...] = 1.0
    f.rho[...] = 1.0
    f.T[...] = 300.0
    p = api.params_default()
    p.dt = 1e-4
    ctx = api.HipProjection(*n)
    ctx.upload(f)
    assert _rk4_device(ctx, g, p) == A.CFD_SUCCESS  # creates rho = rho0 = 1
    ctx.set_density(1.7)
    np.testing.assert_array_equal(ctx.get_field(A.HIP_FIELD_RHO), np.full(f.u.shape, 1.7))
    f.rho[...] = 2.5
    ctx.upload(f)
    np.testing.assert_array_equal(ctx.get_field(A.HIP_FIELD_RHO), np.full(f.u.shape, 2.5))
    fo = api.FlowField(*n)
    fo.copy_from(f)
    assert _rk4_device(ctx, g, p) == A.CFD_SUCCESS
    assert oracle.rk4_step(fo, g, p)[0] == A.CFD_SUCCESS
    np.testing.assert_array_equal(ctx.get_field(A.HIP_FIELD_U), fo.u)
    ctx.close()


def test_checkpoint_read_keeps_nonuniform_density(hip_lib):
    """A restart file with a non-uniform density restores it per cell even
    when the context had no density array (RK4 then reads rho[idx])."""
    n = (12, 10, 8)
    g = api.Grid(*n, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0)
    f = api.FlowField(*n)
    rng = np.random.default_rng(11)
    for k in ("u", "v", "w", "p"):
        getattr(f, k)[...] = 0.05 * rng.standard_normal(f.u.shape)
    f.rho[...] = 1.0 + 0.2 * rng.random(f.u.shape)
    f.T[...] = 300.0
    p = api.params_default()
    p.dt = 1e-4
    with tempfile.TemporaryDirectory() as d:
        path = os.path.join(d, "r.cfdchk")
        assert api.checkpoint_write(path, g, f, p, 0.5, "rk4") == A.CFD_SUCCESS
        ctx = api.HipProjection(*n)
        st = ctx.checkpoint_read(path)[0]
        assert st == A.CFD_SUCCESS, api._native.last_error()
    np.testing.assert_array_equal(ctx.get_field(A.HIP_FIELD_RHO), f.rho)
    fo = api.FlowField(*n)
    fo.copy_from(f)
    assert _rk4_device(ctx, g, p) == A.CFD_SUCCESS
    assert oracle.rk4_step(fo, g, p)[0] == A.CFD_SUCCESS
    for k, fid in (("u", A.HIP_FIELD_U), ("p", A.HIP_FIELD_P)):
        np.testing.assert_array_equal(ctx.get_field(fid), getattr(fo, k), err_msg=k)
    ctx.close()
