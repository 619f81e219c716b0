"""Loading of the in-tree native libraries (cfd_amd/lib/*.so) with typed signatures.

The HIP library is the product: there is no Python or CPU fallback for any
of its entry points. If it cannot be built or loaded, `hip()` raises.

torch is imported before libcfd_hip.so is loaded when it is installed: torch
bundles its own libamdhip64.so with the same SONAME (libamdhip64.so.7), so
loading torch first makes our library bind to that single HIP runtime instead
of bringing a second copy into the process.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import sys
import threading
from pathlib import Path

from . import _abi as A
from . import _sha

PKG_DIR = Path(__file__).resolve().parent
LIB_DIR = PKG_DIR / "lib"
CSRC_DIR = PKG_DIR / "csrc"
# CFD_AMD_HIP_LIB: another build of the library (A/B experiments on one box)
HIP_LIB = Path(os.environ["CFD_AMD_HIP_LIB"]) if os.environ.get("CFD_AMD_HIP_LIB") else (
    LIB_DIR / "libcfd_hip.so")
HOST_LIB = LIB_DIR / "libcfd_host.so"

_lock = threading.Lock()
_host = None
_hip = None


def build(force: bool = False, jobs: int = 4) -> None:
    """Compile libcfd_hip.so (hipcc, gfx950) and libcfd_host.so (gcc) in-tree."""
    args = ["make", "-C", str(CSRC_DIR), f"-j{jobs}"]
    if force:
        subprocess.run(["make", "-C", str(CSRC_DIR), "clean"], check=True,
                       stdout=subprocess.DEVNULL)
    subprocess.run(args, check=True)


def kernel_source_sha() -> str:
    """sha256 over the HIP sources (csrc/hip/*.hip, *.hpp) the built library
    came from: PMC profiles record it, bench.py uses a profile's byte counts
    only for the same kernels (the loader guarantees the library was built
    from these sources, see _check_build_id)."""
    return _sha.kernel_source_sha()


def _ensure_built() -> None:
    if HIP_LIB.exists() and HOST_LIB.exists():
        return
    build()


def _check_build_id(lib) -> None:
    """Refuse a libcfd_hip.so built from other sources than the ones beside it
    (a stale build would run old kernels under the new sources' name, and
    bench.py would charge it the new kernels' PMC bytes). CFD_AMD_HIP_LIB (an
    explicitly chosen other build, A/B experiments) skips the check."""
    if os.environ.get("CFD_AMD_HIP_LIB"):
        return
    got = lib.hip_proj_build_id().decode()
    want = _sha.library_source_sha()
    if got != want:
        raise RuntimeError(f"{HIP_LIB} was built from other sources (build id {got}, sources "
                           f"{want}): rebuild it with `make -C {CSRC_DIR}`")


def _sig(lib, name, restype, *argtypes):
    fn = getattr(lib, name)
    fn.restype = restype
    fn.argtypes = list(argtypes)
    return fn


def _bind_host(lib) -> None:
    P = C.POINTER
    _sig(lib, "cfd_get_last_error", C.c_char_p)
    _sig(lib, "cfd_get_last_status", C.c_int)
    _sig(lib, "cfd_clear_error", None)
    _sig(lib, "cfd_get_error_string", C.c_char_p, C.c_int)
    _sig(lib, "grid_create", P(A.Grid), C.c_size_t, C.c_size_t, C.c_size_t, C.c_double,
         C.c_double, C.c_double, C.c_double, C.c_double, C.c_double)
    _sig(lib, "grid_destroy", None, P(A.Grid))
    _sig(lib, "grid_initialize_uniform", None, P(A.Grid))
    _sig(lib, "flow_field_create", P(A.FlowField), C.c_size_t, C.c_size_t, C.c_size_t)
    _sig(lib, "flow_field_destroy", None, P(A.FlowField))
    _sig(lib, "initialize_flow_field", None, P(A.FlowField), P(A.Grid))
    _sig(lib, "ns_solver_params_default", A.SolverParams)
    _sig(lib, "ns_solver_stats_default", A.SolverStats)
    _sig(lib, "bc_apply_scalar_3d", C.c_int, A.c_double_p, C.c_size_t, C.c_size_t, C.c_size_t,
         C.c_size_t, C.c_int)
    _sig(lib, "bc_apply_dirichlet_scalar_3d", C.c_int, A.c_double_p, C.c_size_t, C.c_size_t,
         C.c_size_t, C.c_size_t, P(A.DirichletValues))
    _sig(lib, "bc_apply_dirichlet_velocity_3d", C.c_int, A.c_double_p, A.c_double_p,
         A.c_double_p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_size_t, P(A.DirichletValues),
         P(A.DirichletValues), P(A.DirichletValues))
    _sig(lib, "cfd_registry_create", C.c_void_p)
    _sig(lib, "cfd_registry_destroy", None, C.c_void_p)
    _sig(lib, "cfd_registry_register_defaults", None, C.c_void_p)
    _sig(lib, "cfd_registry_has", C.c_int, C.c_void_p, C.c_char_p)
    _sig(lib, "cfd_registry_list", C.c_int, C.c_void_p, P(C.c_char_p), C.c_int)
    _sig(lib, "cfd_registry_get_description", C.c_char_p, C.c_void_p, C.c_char_p)
    _sig(lib, "cfd_solver_create", P(A.NSSolver), C.c_void_p, C.c_char_p)
    _sig(lib, "solver_destroy", None, P(A.NSSolver))
    _sig(lib, "solver_init", C.c_int, P(A.NSSolver), P(A.Grid), P(A.SolverParams))
    _sig(lib, "solver_step", C.c_int, P(A.NSSolver), P(A.FlowField), P(A.Grid),
         P(A.SolverParams), P(A.SolverStats))
    _sig(lib, "solver_solve", C.c_int, P(A.NSSolver), P(A.FlowField), P(A.Grid),
         P(A.SolverParams), P(A.SolverStats))
    _sig(lib, "cfd_backend_is_available", C.c_int, C.c_int)
    _sig(lib, "cfd_backend_get_name", C.c_char_p, C.c_int)
    _sig(lib, "cfd_registry_list_by_backend", C.c_int, C.c_void_p, C.c_int, P(C.c_char_p),
         C.c_int)
    _sig(lib, "cfd_solver_create_checked", P(A.NSSolver), C.c_void_p, C.c_char_p)
    _sig(lib, "cfd_host_set_hip_patch", None, C.c_int)
    _sig(lib, "simulation_list_solvers", C.c_int, P(C.c_char_p), C.c_int)
    _sig(lib, "init_simulation_with_solver", P(A.SimulationData), C.c_size_t, C.c_size_t,
         C.c_size_t, C.c_double, C.c_double, C.c_double, C.c_double, C.c_double, C.c_double,
         C.c_char_p)
    _sig(lib, "free_simulation", None, P(A.SimulationData))
    _sig(lib, "run_simulation_step", C.c_int, P(A.SimulationData))
    _sig(lib, "run_simulation_solve", C.c_int, P(A.SimulationData))
    _sig(lib, "cfd_checkpoint_write", C.c_int, C.c_char_p, P(A.Grid), P(A.FlowField),
         P(A.SolverParams), C.c_double, C.c_char_p, C.c_char_p, C.c_char_p)
    _sig(lib, "cfd_checkpoint_read", C.c_int, C.c_char_p, P(P(A.Grid)), P(P(A.FlowField)),
         P(A.SolverParams), P(C.c_double), C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t,
         C.c_char_p, C.c_size_t)
    _sig(lib, "save_simulation_checkpoint", C.c_int, P(A.SimulationData), C.c_char_p)
    _sig(lib, "load_simulation_from_checkpoint", P(A.SimulationData), C.c_char_p)
    _sig(lib, "restore_simulation_checkpoint", C.c_int, P(A.SimulationData), C.c_char_p)
    _sig(lib, "write_vtk_output", None, C.c_char_p, C.c_char_p, A.c_double_p, C.c_size_t,
         C.c_size_t, C.c_size_t, C.c_double, C.c_double, C.c_double, C.c_double, C.c_double,
         C.c_double)
    _sig(lib, "write_vtk_vector_output", None, C.c_char_p, C.c_char_p, A.c_double_p,
         A.c_double_p, A.c_double_p, C.c_size_t, C.c_size_t, C.c_size_t, C.c_double, C.c_double,
         C.c_double, C.c_double, C.c_double, C.c_double)
    _sig(lib, "write_vtk_flow_field", None, C.c_char_p, P(A.FlowField), C.c_size_t, C.c_size_t,
         C.c_size_t, C.c_double, C.c_double, C.c_double, C.c_double, C.c_double, C.c_double)
    _sig(lib, "poisson_solver_params_default", A.PoissonParams)
    _sig(lib, "poisson_solver_stats_default", A.PoissonStats)
    _sig(lib, "poisson_solver_backend_available", C.c_bool, C.c_int)
    _sig(lib, "poisson_solver_create", P(A.PoissonSolver), C.c_int, C.c_int)
    _sig(lib, "poisson_solver_init", C.c_int, P(A.PoissonSolver), C.c_size_t, C.c_size_t,
         C.c_size_t, C.c_double, C.c_double, C.c_double, P(A.PoissonParams))
    _sig(lib, "poisson_solver_destroy", None, P(A.PoissonSolver))
    _sig(lib, "poisson_solver_solve", C.c_int, P(A.PoissonSolver), A.c_double_p, A.c_double_p,
         A.c_double_p, P(A.PoissonStats))
    _sig(lib, "poisson_solver_iterate", C.c_int, P(A.PoissonSolver), A.c_double_p, A.c_double_p,
         A.c_double_p, A.c_double_p)


def _bind_hip(lib) -> None:
    P = C.POINTER
    V = C.c_void_p
    _sig(lib, "hip_proj_config_default", A.HipProjConfig)
    _sig(lib, "cfd_hip_stream_bench", C.c_int, C.c_int, C.c_size_t, C.c_int,
         P(C.c_double), P(C.c_double))
    _sig(lib, "cfd_hip_stream_bench_nm", C.c_int, C.c_int, C.c_size_t, C.c_int, C.c_int, C.c_int,
         P(C.c_double))
    _sig(lib, "hip_projection_available", C.c_int)
    _sig(lib, "hip_proj_create", V, C.c_size_t, C.c_size_t, C.c_size_t, P(A.HipProjConfig))
    _sig(lib, "hip_proj_destroy", None, V)
    _sig(lib, "hip_proj_step", C.c_int, V, P(A.FlowField), P(A.Grid), P(A.SolverParams),
         P(A.SolverStats))
    _sig(lib, "hip_proj_upload", C.c_int, V, P(A.FlowField))
    _sig(lib, "hip_proj_download", C.c_int, V, P(A.FlowField))
    _sig(lib, "hip_proj_step_device", C.c_int, V, P(A.Grid), P(A.SolverParams),
         P(A.SolverStats))
    _sig(lib, "hip_proj_get_field", C.c_int, V, C.c_int, A.c_double_p)
    _sig(lib, "hip_proj_set_field", C.c_int, V, C.c_int, A.c_double_p)
    _sig(lib, "hip_proj_fill_field", C.c_int, V, C.c_int, C.c_double)
    _sig(lib, "hip_proj_set_density", C.c_int, V, C.c_double)
    _sig(lib, "hip_proj_apply_scalar_bc", C.c_int, V, C.c_int, C.c_int)
    _sig(lib, "hip_proj_apply_dirichlet", C.c_int, V, C.c_int, P(A.DirichletValues))
    _sig(lib, "hip_proj_get_poisson_stats", C.c_int, V, P(A.PoissonStats))
    _sig(lib, "hip_proj_field_crc32", C.c_int, V, C.c_int, P(C.c_uint32))
    _sig(lib, "hip_proj_checkpoint_write", C.c_int, V, C.c_char_p, P(A.Grid), P(A.SolverParams),
         C.c_double, C.c_char_p, C.c_char_p, C.c_char_p)
    _sig(lib, "hip_proj_checkpoint_read", C.c_int, V, C.c_char_p, P(P(A.Grid)),
         P(A.SolverParams), P(C.c_double), C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t,
         C.c_char_p, C.c_size_t)
    _sig(lib, "hip_proj_apply_thermal_bcs", C.c_int, V, P(A.SolverParams))
    _sig(lib, "hip_proj_enable_timing", None, V, C.c_int)
    _sig(lib, "hip_proj_reset_timing", None, V)
    _sig(lib, "hip_proj_get_timing", None, V, A.c_double_p, P(C.c_longlong))
    _sig(lib, "hip_proj_get_timing_n", C.c_int, V, A.c_double_p, P(C.c_longlong), C.c_int)
    _sig(lib, "hip_proj_get_clock_sample", C.c_int, V, P(C.c_double), P(C.c_longlong))
    _sig(lib, "hip_proj_get_placement", C.c_int, V, P(C.c_double), C.c_int, P(C.c_int))
    _sig(lib, "hip_proj_abi_version", C.c_int)
    _sig(lib, "hip_proj_build_id", C.c_char_p)
    _sig(lib, "hip_proj_synchronize", C.c_int, V)
    _sig(lib, "hip_proj_sync_host", C.c_int, V, P(A.FlowField))
    _sig(lib, "hip_proj_mark_host_dirty", C.c_int, V)
    _sig(lib, "hip_proj_device_bytes", C.c_size_t, V)
    _sig(lib, "hip_proj_row_pitch", C.c_size_t, V)
    _sig(lib, "hip_proj_cg_fixed_iters", C.c_double, V, A.c_double_p, C.c_double, C.c_double,
         C.c_double, C.c_int)
    _sig(lib, "hip_proj_cg_fixed_iters_ex", C.c_double, V, A.c_double_p, C.c_double,
         C.c_double, C.c_double, C.c_int, C.c_double)
    _sig(lib, "hip_proj_poisson_solve", C.c_int, V, C.c_int, A.c_double_p, A.c_double_p,
         C.c_double, C.c_double, C.c_double, P(A.PoissonParams), P(A.PoissonStats))
    _sig(lib, "hip_proj_poisson_solve_ex", C.c_int, V, C.c_int, A.c_double_p, A.c_double_p,
         C.c_double, C.c_double, C.c_double, P(A.PoissonParams), P(A.PoissonStats), C.c_int,
         A.c_double_p)
    _sig(lib, "hip_proj_slab_layout", C.c_int, C.c_size_t, C.c_int, C.c_int, P(C.c_size_t),
         P(C.c_size_t))
    _sig(lib, "hip_proj_comm_unique_id", C.c_int, C.c_char_p)
    _sig(lib, "hip_proj_comm_create_rccl", V, C.c_char_p, C.c_int, C.c_int, C.c_int)
    _sig(lib, "hip_proj_group_create", V, C.c_int)
    _sig(lib, "hip_proj_group_destroy", None, V)
    _sig(lib, "hip_proj_comm_create_local", V, V, C.c_int, C.c_int)
    _sig(lib, "hip_proj_comm_destroy", None, V)
    _sig(lib, "hip_proj_comm_rank", C.c_int, V)
    _sig(lib, "hip_proj_comm_size", C.c_int, V)
    _sig(lib, "hip_proj_comm_device_allreduce", C.c_int, V)
    _sig(lib, "hip_proj_comm_mailbox_bench", C.c_int, V, C.c_int, C.c_int, P(C.c_double))
    _sig(lib, "hip_proj_create_slab", V, C.c_size_t, C.c_size_t, C.c_size_t, V,
         P(A.HipProjConfig))
    _sig(lib, "hip_proj_slab_info", C.c_int, V, P(C.c_size_t), P(C.c_size_t), P(C.c_int),
         P(C.c_int))
    _sig(lib, "hip_rk4_step_device", C.c_int, V, P(A.Grid), P(A.SolverParams), P(A.SolverStats))
    _sig(lib, "hip_rk4_step", C.c_int, V, P(A.FlowField), P(A.Grid), P(A.SolverParams),
         P(A.SolverStats))
    _sig(lib, "create_projection_hip_solver", P(A.NSSolver))
    _sig(lib, "create_rk4_hip_solver", P(A.NSSolver))
    _sig(lib, "cfd_hip_register_solvers", None, V)
    _sig(lib, "hip_proj_write_vtk", C.c_int, V, C.c_char_p, P(A.Grid), C.c_double)
    # boundary_conditions_gpu.h (device pointers, packed layout, opaque stream)
    _sig(lib, "bc_apply_neumann_gpu", None, V, C.c_size_t, C.c_size_t, V)
    _sig(lib, "bc_apply_scalar_gpu", None, V, C.c_size_t, C.c_size_t, C.c_int, V)
    _sig(lib, "bc_apply_velocity_gpu", None, V, V, C.c_size_t, C.c_size_t, C.c_int, V)
    _sig(lib, "bc_apply_dirichlet_scalar_gpu", None, V, C.c_size_t, C.c_size_t,
         P(A.DirichletValues), V)
    _sig(lib, "bc_apply_dirichlet_velocity_gpu", None, V, V, C.c_size_t, C.c_size_t,
         P(A.DirichletValues), P(A.DirichletValues), V)
    _sig(lib, "bc_apply_scalar_3d_gpu", None, V, C.c_size_t, C.c_size_t, C.c_size_t, C.c_int, V)
    _sig(lib, "bc_apply_velocity_3d_gpu", None, V, V, V, C.c_size_t, C.c_size_t, C.c_size_t,
         C.c_int, V)
    _sig(lib, "create_cg_gpu_solver", P(A.PoissonSolver))
    _sig(lib, "create_redblack_gpu_solver", P(A.PoissonSolver))
    _sig(lib, "create_jacobi_gpu_solver", P(A.PoissonSolver))
    # gpu_device.h API
    _sig(lib, "gpu_config_default", A.GpuConfig)
    _sig(lib, "gpu_is_available", C.c_int)
    _sig(lib, "gpu_get_device_info", C.c_int, P(A.GpuDeviceInfo), C.c_int)
    _sig(lib, "gpu_select_device", C.c_int, C.c_int)
    _sig(lib, "gpu_should_use", C.c_int, P(A.GpuConfig), C.c_size_t, C.c_size_t, C.c_size_t,
         C.c_int)
    _sig(lib, "gpu_solver_create", V, C.c_size_t, C.c_size_t, C.c_size_t, P(A.GpuConfig))
    _sig(lib, "gpu_solver_destroy", None, V)
    _sig(lib, "gpu_solver_upload", C.c_int, V, P(A.FlowField))
    _sig(lib, "gpu_solver_download", C.c_int, V, P(A.FlowField))
    _sig(lib, "gpu_solver_step", C.c_int, V, P(A.Grid), P(A.SolverParams), P(A.GpuSolverStats))
    _sig(lib, "gpu_solver_get_stats", A.GpuSolverStats, V)
    _sig(lib, "gpu_solver_reset_stats", None, V)
    _sig(lib, "solve_navier_stokes_gpu", C.c_int, P(A.FlowField), P(A.Grid), P(A.SolverParams),
         P(A.GpuConfig))
    _sig(lib, "solve_projection_method_gpu", C.c_int, P(A.FlowField), P(A.Grid),
         P(A.SolverParams), P(A.GpuConfig))
    _sig(lib, "solve_rk4_method_gpu", C.c_int, P(A.FlowField), P(A.Grid), P(A.SolverParams),
         P(A.GpuConfig))


def _import_torch_first() -> None:
    if "torch" in sys.modules or os.environ.get("CFD_AMD_NO_TORCH"):
        return
    try:
        import torch  # noqa: F401  (shares its HIP runtime with libcfd_hip.so)
    except Exception:
        pass


def host():
    """libcfd_host.so (loaded RTLD_GLOBAL so the HIP plugin resolves cfd_set_error)."""
    global _host
    with _lock:
        if _host is None:
            _ensure_built()
            lib = C.CDLL(str(HOST_LIB), mode=C.RTLD_GLOBAL)
            _bind_host(lib)
            _host = lib
        return _host


def hip():
    """libcfd_hip.so, the HIP product library. Raises if it cannot be loaded."""
    global _hip
    host()
    with _lock:
        if _hip is None:
            _ensure_built()
            _import_torch_first()
            lib = C.CDLL(str(HIP_LIB), mode=C.RTLD_GLOBAL)
            _bind_hip(lib)
            _check_build_id(lib)
            if lib.hip_proj_abi_version() != A.HIP_PROJ_ABI_VERSION:
                raise RuntimeError(f"{HIP_LIB}: ABI version {lib.hip_proj_abi_version()}, "
                                   f"the bindings expect {A.HIP_PROJ_ABI_VERSION}")
            _hip = lib
        return _hip


def last_error() -> str:
    msg = host().cfd_get_last_error()
    return msg.decode() if msg else ""
