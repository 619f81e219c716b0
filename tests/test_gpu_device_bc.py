"""The reference's device-pointer BC layer (boundary_conditions_gpu.cuh) on
caller-owned device arrays (torch tensors on the GPU, packed layout, the
caller's stream), bitwise against the host reference BCs of libcfd_host.so
(boundary_conditions_core_impl.h:41-186 order) applied to the same data."""
import ctypes as C

import numpy as np
import pytest
import torch

from cfd_amd import _abi as A
from cfd_amd import _native, api

pytestmark = pytest.mark.gpu


def _dev(a):
    return torch.from_numpy(a.copy()).to("cuda")


def _stream():
    return C.c_void_p(torch.cuda.current_stream().cuda_stream)


@pytest.mark.parametrize("shape", [(5, 7, 9), (9, 20, 130), (1, 6, 11), (1, 33, 17)])
@pytest.mark.parametrize("bc", [A.BC_TYPE_NEUMANN, A.BC_TYPE_PERIODIC])
def test_scalar_and_velocity_bcs_bitwise(hip_lib, shape, bc):
    nz, ny, nx = shape
    rng = np.random.default_rng(nx * ny + nz)
    a = rng.standard_normal(shape)
    ref = a.copy()
    api.bc_apply_scalar_3d(ref, bc)
    d = _dev(a)
    hip_lib.bc_apply_scalar_3d_gpu(C.c_void_p(d.data_ptr()), nx, ny, nz, bc, _stream())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d.cpu().numpy(), ref)
    # velocity form: u, v, w each get the scalar BC
    us = [rng.standard_normal(shape) for _ in range(3)]
    ds = [_dev(u) for u in us]
    ptr = [C.c_void_p(x.data_ptr()) for x in ds]
    hip_lib.bc_apply_velocity_3d_gpu(ptr[0], ptr[1], ptr[2], nx, ny, nz, bc, _stream())
    torch.cuda.synchronize()
    for u, x in zip(us, ds):
        r = u.copy()
        if nz > 1 or x is not ds[2]:
            api.bc_apply_scalar_3d(r, bc)
        np.testing.assert_array_equal(x.cpu().numpy(), r)


def test_dirichlet_2d_bitwise(hip_lib):
    host = _native.host()
    ny, nx = 12, 10
    rng = np.random.default_rng(1)
    a = rng.standard_normal((1, ny, nx))
    vals = api.dirichlet(left=1.5, right=-2.0, top=3.25, bottom=0.5)
    ref = a.copy()
    host.bc_apply_dirichlet_scalar_3d(ref.ctypes.data_as(A.c_double_p), nx, ny, 1, 0,
                                      C.byref(vals))
    d = _dev(a)
    hip_lib.bc_apply_dirichlet_scalar_gpu(C.c_void_p(d.data_ptr()), nx, ny, C.byref(vals),
                                          _stream())
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d.cpu().numpy(), ref)
    u, v = _dev(a), _dev(-a)
    vv = api.dirichlet(top=7.0)
    hip_lib.bc_apply_dirichlet_velocity_gpu(C.c_void_p(u.data_ptr()), C.c_void_p(v.data_ptr()),
                                            nx, ny, C.byref(vals), C.byref(vv), _stream())
    torch.cuda.synchronize()
    rv = -a
    host.bc_apply_dirichlet_scalar_3d(rv.ctypes.data_as(A.c_double_p), nx, ny, 1, 0, C.byref(vv))
    np.testing.assert_array_equal(u.cpu().numpy(), ref)
    np.testing.assert_array_equal(v.cpu().numpy(), rv)


def test_degenerate_sizes_are_no_ops(hip_lib):
    """nx, ny < 3 or nz == 2 return without touching memory (boundary_conditions_gpu.cu:477-485)."""
    a = np.arange(2 * 5 * 5, dtype=np.float64).reshape(2, 5, 5)
    d = _dev(a)
    hip_lib.bc_apply_scalar_3d_gpu(C.c_void_p(d.data_ptr()), 5, 5, 2, A.BC_TYPE_NEUMANN, None)
    hip_lib.bc_apply_scalar_gpu(C.c_void_p(d.data_ptr()), 2, 25, A.BC_TYPE_NEUMANN, None)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(d.cpu().numpy(), a)
