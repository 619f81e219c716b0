"""Scenario builders restating the reference's own test harnesses.

Every builder cites the reference file it restates; the same host objects
are then handed to the HIP product path and to the CPU oracle.
"""
from __future__ import annotations

import math

import numpy as np

from cfd_amd import _abi as A
from cfd_amd import api

# tests/solvers/navier_stokes/cpu/test_ns_solver_3d.c:345-348 (projection, nz = 1)
KAT_PROJECTION_L2 = (6.84647639323831686e-02, 3.42315494726977212e-02, 1.00000039251590289e+00)
# test_ns_solver_3d.c:363-366 (RK4, nz = 1; one step: the step wrapper forces max_iter = 1)
KAT_RK4_L2 = (6.88584742267390471e-02, 3.49775875752817156e-02, 1.00000000000000000e+00)


def kat_2d():
    """16x16 nz=1 backward-compat KAT (test_ns_solver_3d.c:267-348)."""
    nx = ny = 16
    g = api.Grid(nx, ny, 1, 0.0, 1.0, 0.0, 1.0, 0.0, 0.0)
    f = api.FlowField(nx, ny, 1)
    for j in range(ny):
        for i in range(nx):
            f.u[0, j, i] = 0.1 * math.sin(math.pi * g.y[j])
            f.v[0, j, i] = 0.05 * math.sin(2.0 * math.pi * g.x[i])
    f.w[...] = 0.0
    f.p[...] = 1.0
    f.rho[...] = 1.0
    f.T[...] = 300.0
    p = api.params_default()
    p.dt = 1e-4
    p.source_amplitude_u = 0.0
    p.source_amplitude_v = 0.0
    return g, f, p


def l2_rms(a: np.ndarray) -> float:
    """compute_l2_norm of test_ns_solver_3d.c:253-259 (sequential sum)."""
    s = 0.0
    for v in a.ravel():
        s += v * v
    return math.sqrt(s / a.size)


def tg3(n: int, nu: float = 0.01):
    """Taylor-Green 3-D IC on [0, 2pi]^3 (taylor_green_3d_reference.h:177-230)."""
    L = 2.0 * math.pi
    g = api.Grid(n, n, n, 0.0, L, 0.0, L, 0.0, L)
    f = api.FlowField(n, n, n)
    f.u[...] = tg3_analytic(g, "u", 0.0, nu)
    f.v[...] = tg3_analytic(g, "v", 0.0, nu)
    f.w[...] = 0.0
    f.p[...] = 0.0
    f.rho[...] = 1.0
    f.T[...] = 300.0
    tg3_bc(f)
    return g, f, api.validation_params(1e-3, nu)


def _libm(fn, a):
    return np.array([fn(float(v)) for v in a])


def tg3_analytic(g: api.Grid, comp: str, t: float, nu: float) -> np.ndarray:
    """tg3_analytical_u/v (taylor_green_3d_reference.h:64-74), libm-evaluated in
    the reference's left-to-right product order."""
    cx, sx = _libm(math.cos, g.x), _libm(math.sin, g.x)
    cy, sy = _libm(math.cos, g.y), _libm(math.sin, g.y)
    cz = _libm(math.cos, g.z)
    e = math.exp(-3.0 * nu * t)
    X = lambda a: a[None, None, :]
    Y = lambda a: a[None, :, None]
    Z = lambda a: a[:, None, None]
    if comp == "u":
        return X(cx) * Y(sy) * Z(cz) * e
    return -X(sx) * Y(cy) * Z(cz) * e


def tg3_bc(f: api.FlowField):
    for a in (f.u, f.v, f.w, f.p):
        api.bc_apply_scalar_3d(a, A.BC_TYPE_PERIODIC)


def tg3_l2_errors(g: api.Grid, f: api.FlowField, t: float, nu: float = 0.01):
    """Relative interior L2 errors of u, v (taylor_green_3d_reference.h:349-372)."""
    n = g.nx
    ue = tg3_analytic(g, "u", t, nu)[1:n - 1, 1:n - 1, 1:n - 1]
    ve = tg3_analytic(g, "v", t, nu)[1:n - 1, 1:n - 1, 1:n - 1]
    ui = f.u[1:n - 1, 1:n - 1, 1:n - 1]
    vi = f.v[1:n - 1, 1:n - 1, 1:n - 1]
    eu = math.sqrt(float(np.sum((ui - ue) ** 2)) / float(np.sum(ue ** 2)))
    ev = math.sqrt(float(np.sum((vi - ve) ** 2)) / float(np.sum(ve ** 2)))
    return eu, ev


def cavity(nx: int, ny: int, nz: int = 1, Re: float = 100.0, dt: float = 5e-4):
    """Lid-driven cavity at rest (lid_driven_cavity_common.h:98-140, 238-270);
    3-D variant of SURVEY.md §8d config 3 with the z faces as walls."""
    zmax = 1.0 if nz > 1 else 0.0
    g = api.Grid(nx, ny, nz, 0.0, 1.0, 0.0, 1.0, 0.0, zmax)
    f = api.FlowField(nx, ny, nz)
    f.u[...] = 0.0
    f.v[...] = 0.0
    f.w[...] = 0.0
    f.p[...] = 0.0
    f.rho[...] = 1.0
    f.T[...] = 300.0
    nu = 1.0 * 1.0 / Re
    return g, f, api.validation_params(dt, nu)


def cos_rhs(n: int, nz: int | None = None):
    """rhs = cos(pi x) cos(pi y) cos(pi z) on [0,1]^3, interior only
    (SURVEY.md §8d / App. B CG iteration counts)."""
    nz = n if nz is None else nz
    g = api.Grid(n, n, nz, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0 if nz > 1 else 0.0)
    rhs = np.zeros((nz, n, n))
    zc = np.cos(math.pi * g.z)[:, None, None] if nz > 1 else np.ones((1, 1, 1))
    val = zc * np.cos(math.pi * g.y)[None, :, None] * np.cos(math.pi * g.x)[None, None, :]
    if nz > 1:
        rhs[1:-1, 1:-1, 1:-1] = val[1:-1, 1:-1, 1:-1]
    else:
        rhs[:, 1:-1, 1:-1] = val[:, 1:-1, 1:-1]
    return g, rhs
