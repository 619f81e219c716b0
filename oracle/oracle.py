"""TEST INFRASTRUCTURE ONLY -- Python handle on the CPU oracle (liboracle.so).

The oracle is a plain-C restatement of the reference's scalar/OpenMP
projection path (see oracle.h for the pinning statement). Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, and only
as the checker or the timed CPU baseline -- never as the product path.
"""
from __future__ import annotations

import ctypes as C
import subprocess
from pathlib import Path

import numpy as np

from cfd_amd import _abi as A

ORACLE_DIR = Path(__file__).resolve().parent
# void (*)(double* x, size_t nx, size_t ny, size_t nz, void* ctx)
BC_HOOK = C.CFUNCTYPE(None, C.POINTER(C.c_double), C.c_size_t, C.c_size_t, C.c_size_t,
                      C.c_void_p)
LIB = ORACLE_DIR / "build" / "liboracle.so"
_lib = None


def build(force: bool = False) -> Path:
    if force and LIB.exists():
        LIB.unlink()
    subprocess.run(["make", "-C", str(ORACLE_DIR)], check=True, stdout=subprocess.DEVNULL)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not LIB.exists():
            build()
        L = C.CDLL(str(LIB))
        P = C.POINTER
        d = A.c_double_p
        sz = C.c_size_t

        def sig(name, res, *args):
            f = getattr(L, name)
            f.restype = res
            f.argtypes = list(args)

        sig("oracle_set_threads", None, C.c_int)
        sig("oracle_get_threads", C.c_int)
        sig("oracle_set_poisson_cap", None, C.c_int)
        sig("oracle_set_projection_poisson_params", None, P(A.PoissonParams))
        sig("oracle_set_gpu_rhs", None, C.c_int)
        sig("oracle_set_poisson_bc_hook", None, BC_HOOK, C.c_void_p)
        sig("oracle_projection_step", C.c_int, P(A.FlowField), P(A.Grid), P(A.SolverParams),
            P(A.SolverStats), C.c_int, P(C.c_int))
        sig("oracle_last_phase_ms", None, d)
        sig("oracle_last_poisson_stats", None, P(A.PoissonStats))
        sig("oracle_cg_solve", C.c_int, d, d, sz, sz, sz, C.c_double, C.c_double, C.c_double,
            P(A.PoissonParams), P(A.PoissonStats))
        sig("oracle_redblack_solve", C.c_int, d, d, sz, sz, sz, C.c_double, C.c_double,
            C.c_double, P(A.PoissonParams), P(A.PoissonStats))
        sig("oracle_jacobi_solve", C.c_int, d, d, d, sz, sz, sz, C.c_double, C.c_double,
            C.c_double, P(A.PoissonParams), P(A.PoissonStats))
        sig("oracle_poisson_params_default", A.PoissonParams)
        sig("oracle_cg_fixed_iters", C.c_double, d, d, sz, sz, sz, C.c_double, C.c_double,
            C.c_double, C.c_int)
        sig("oracle_bc_neumann_3d", None, d, sz, sz, sz)
        sig("oracle_bc_periodic_3d", None, d, sz, sz, sz)
        sig("oracle_bc_dirichlet_3d", None, d, sz, sz, sz, P(A.DirichletValues))
        sig("oracle_poisson_apply_bc", None, d, sz, sz, sz)
        sig("oracle_grid_create_uniform", P(A.Grid), sz, sz, sz, C.c_double, C.c_double,
            C.c_double, C.c_double, C.c_double, C.c_double)
        sig("oracle_grid_destroy", None, P(A.Grid))
        sig("oracle_field_create", P(A.FlowField), sz, sz, sz)
        sig("oracle_field_destroy", None, P(A.FlowField))
        sig("oracle_params_default", A.SolverParams)
        sig("oracle_max_velocity_pressure", None, P(A.FlowField), d, d)
        sig("oracle_apply_thermal_bcs", C.c_int, P(A.FlowField), P(A.SolverParams))
        sig("oracle_rk4_step", C.c_int, P(A.FlowField), P(A.Grid), P(A.SolverParams),
            P(A.SolverStats))
        sig("oracle_energy_step", C.c_int, P(A.FlowField), P(A.Grid), P(A.SolverParams),
            C.c_double, C.c_double)
        sig("oracle_gpu_explicit_step", C.c_int, P(A.FlowField), P(A.Grid), P(A.SolverParams))
        _lib = L
    return _lib


def _dp(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(A.c_double_p)


def set_threads(n: int) -> None:
    lib().oracle_set_threads(n)


def projection_step(field, grid, params, poisson=A.ORACLE_POISSON_CG):
    """One reference `projection` step on a cfd_amd.api.FlowField / Grid.
    Returns (status, stats, poisson_iterations)."""
    st = A.SolverStats()
    it = C.c_int(0)
    s = lib().oracle_projection_step(field.ptr, grid.ptr, C.byref(params), C.byref(st),
                                     poisson, C.byref(it))
    return s, st, it.value


def last_poisson_stats() -> A.PoissonStats:
    """Poisson stats of the last projection_step (iterations, residuals, status)."""
    st = A.PoissonStats()
    lib().oracle_last_poisson_stats(C.byref(st))
    return st


def set_projection_poisson_params(params=None):
    lib().oracle_set_projection_poisson_params(C.byref(params) if params is not None else None)


def last_phase_ms():
    out = (C.c_double * 4)()
    lib().oracle_last_phase_ms(out)
    return list(out)


def poisson_params(**kw) -> A.PoissonParams:
    p = lib().oracle_poisson_params_default()
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def cg_solve(x: np.ndarray, rhs: np.ndarray, dx, dy, dz, params=None):
    nz, ny, nx = x.shape
    st = A.PoissonStats()
    s = lib().oracle_cg_solve(_dp(x), _dp(rhs), nx, ny, nz, dx, dy, dz,
                              C.byref(params) if params is not None else None, C.byref(st))
    return s, st


def redblack_solve(x, rhs, dx, dy, dz, params=None):
    nz, ny, nx = x.shape
    st = A.PoissonStats()
    s = lib().oracle_redblack_solve(_dp(x), _dp(rhs), nx, ny, nz, dx, dy, dz,
                                    C.byref(params) if params is not None else None, C.byref(st))
    return s, st


def jacobi_solve(x, rhs, dx, dy, dz, params=None):
    nz, ny, nx = x.shape
    st = A.PoissonStats()
    xt = x.copy()
    s = lib().oracle_jacobi_solve(_dp(x), _dp(xt), _dp(rhs), nx, ny, nz, dx, dy, dz,
                                  C.byref(params) if params is not None else None, C.byref(st))
    return s, st


def cg_fixed_iters(x, rhs, dx, dy, dz, iters) -> float:
    nz, ny, nx = x.shape
    return lib().oracle_cg_fixed_iters(_dp(x), _dp(rhs), nx, ny, nz, dx, dy, dz, iters)


def rk4_step(field, grid, params):
    """rk4_step -> rk4_impl (solver_rk4.c:69-259), one step; returns (status, stats)."""
    st = A.SolverStats()
    s = lib().oracle_rk4_step(field.ptr, grid.ptr, C.byref(params), C.byref(st))
    return s, st


def gpu_explicit_step(field, grid, params) -> int:
    """gpu_solver_step's explicit pressure-relaxation step (solver_projection_gpu.cu:523-570)."""
    return lib().oracle_gpu_explicit_step(field.ptr, grid.ptr, C.byref(params))


def apply_thermal_bcs(field, params) -> int:
    """energy_apply_thermal_bcs (energy_solver.c:204-334) on field.T."""
    return lib().oracle_apply_thermal_bcs(field.ptr, C.byref(params))


def bc_neumann(a: np.ndarray):
    nz, ny, nx = a.shape
    lib().oracle_bc_neumann_3d(_dp(a), nx, ny, nz)


def bc_periodic(a: np.ndarray):
    nz, ny, nx = a.shape
    lib().oracle_bc_periodic_3d(_dp(a), nx, ny, nz)


def bc_dirichlet(a: np.ndarray, values: A.DirichletValues):
    nz, ny, nx = a.shape
    lib().oracle_bc_dirichlet_3d(_dp(a), nx, ny, nz, C.byref(values))


def poisson_apply_bc(a: np.ndarray):
    nz, ny, nx = a.shape
    lib().oracle_poisson_apply_bc(_dp(a), nx, ny, nz)
