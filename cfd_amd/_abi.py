"""ctypes mirrors of include/cfd_hip/cfd_abi.h and projection_hip.h.

These describe the same memory layout as the reference's C structs
(lib/include/cfd/solvers/navier_stokes_solver.h:54-277,
lib/include/cfd/core/grid.h:17-40, lib/include/cfd/solvers/poisson_solver.h:100-233),
so Python can build a grid / flow_field / params once and hand the same
objects to the product library and to the CPU oracle.
"""
from __future__ import annotations

import ctypes as C

c_double_p = C.POINTER(C.c_double)

# cfd_status_t (cfd_status.h:13-24)
CFD_SUCCESS = 0
CFD_ERROR = -1
CFD_ERROR_NOMEM = -2
CFD_ERROR_INVALID = -3
CFD_ERROR_IO = -4
CFD_ERROR_UNSUPPORTED = -5
CFD_ERROR_DIVERGED = -6
CFD_ERROR_MAX_ITER = -7
CFD_ERROR_LIMIT_EXCEEDED = -8
CFD_ERROR_NOT_FOUND = -9

# bc_type_t (boundary_conditions.h:19-27)
BC_TYPE_PERIODIC = 0
BC_TYPE_NEUMANN = 1
BC_TYPE_DIRICHLET = 2

# poisson_solver_status_t
POISSON_CONVERGED = 0
POISSON_MAX_ITER = 1
POISSON_STAGNATED = 3

# hip_poisson_method_t / hip_field_id_t / hip_kernel_timer_t
HIP_POISSON_CG = 0
HIP_POISSON_REDBLACK = 1
HIP_POISSON_JACOBI = 2
HIP_FIELD_U, HIP_FIELD_V, HIP_FIELD_W, HIP_FIELD_P, HIP_FIELD_T, HIP_FIELD_RHO = range(6)
KERNEL_TIMERS = ["predictor", "cg_setup", "cg_sweep_a", "cg_sweep_b", "corrector",
                 "relax", "residual", "energy", "rk_stage", "cg_sweep_bx", "cc_update",
                 "cc_spmv", "halo", "allreduce", "cg_small", "relax2", "cc_fused", "cc_fold"]
HIP_KT_COUNT = len(KERNEL_TIMERS)
HIP_PROJ_ABI_VERSION = 3  # projection_hip.h

# oracle_poisson_kind_t
ORACLE_POISSON_CG = 0
ORACLE_POISSON_REDBLACK = 1
ORACLE_POISSON_JACOBI = 2


class Grid(C.Structure):
    _fields_ = [
        ("x", c_double_p), ("y", c_double_p), ("dx", c_double_p), ("dy", c_double_p),
        ("nx", C.c_size_t), ("ny", C.c_size_t),
        ("xmin", C.c_double), ("xmax", C.c_double), ("ymin", C.c_double), ("ymax", C.c_double),
        ("z", c_double_p), ("dz", c_double_p), ("nz", C.c_size_t),
        ("zmin", C.c_double), ("zmax", C.c_double), ("stride_z", C.c_size_t),
        ("inv_dz2", C.c_double), ("k_start", C.c_size_t), ("k_end", C.c_size_t),
    ]


class FlowField(C.Structure):
    _fields_ = [
        ("u", c_double_p), ("v", c_double_p), ("w", c_double_p), ("p", c_double_p),
        ("rho", c_double_p), ("T", c_double_p),
        ("nx", C.c_size_t), ("ny", C.c_size_t), ("nz", C.c_size_t),
    ]


class DirichletValues(C.Structure):
    _fields_ = [("left", C.c_double), ("right", C.c_double), ("top", C.c_double),
                ("bottom", C.c_double), ("front", C.c_double), ("back", C.c_double)]


class ThermalBC(C.Structure):
    _fields_ = [("left", C.c_int), ("right", C.c_int), ("bottom", C.c_int), ("top", C.c_int),
                ("front", C.c_int), ("back", C.c_int), ("dirichlet_values", DirichletValues)]


SourceFunc = C.CFUNCTYPE(None, C.c_double, C.c_double, C.c_double, C.c_double, C.c_void_p,
                         c_double_p, c_double_p, c_double_p)
HeatSourceFunc = C.CFUNCTYPE(C.c_double, C.c_double, C.c_double, C.c_double, C.c_double,
                             C.c_void_p)


class SolverParams(C.Structure):
    _fields_ = [
        ("dt", C.c_double), ("cfl", C.c_double), ("gamma", C.c_double), ("mu", C.c_double),
        ("k", C.c_double), ("max_iter", C.c_int), ("tolerance", C.c_double),
        ("source_amplitude_u", C.c_double), ("source_amplitude_v", C.c_double),
        ("source_decay_rate", C.c_double), ("pressure_coupling", C.c_double),
        ("source_func", C.c_void_p), ("source_context", C.c_void_p),
        ("alpha", C.c_double), ("beta", C.c_double), ("T_ref", C.c_double),
        ("gravity", C.c_double * 3),
        ("heat_source_func", C.c_void_p), ("heat_source_context", C.c_void_p),
        ("thermal_bc", ThermalBC),
    ]


class SolverStats(C.Structure):
    _fields_ = [
        ("iterations", C.c_int), ("residual", C.c_double), ("max_velocity", C.c_double),
        ("max_pressure", C.c_double), ("max_temperature", C.c_double),
        ("cfl_number", C.c_double), ("elapsed_time_ms", C.c_double), ("status", C.c_int),
    ]


class NSSolver(C.Structure):
    _fields_ = [
        ("name", C.c_char_p), ("description", C.c_char_p), ("version", C.c_char_p),
        ("capabilities", C.c_int), ("backend", C.c_int), ("context", C.c_void_p),
        ("init", C.c_void_p), ("destroy", C.c_void_p), ("step", C.c_void_p),
        ("solve", C.c_void_p), ("apply_boundary", C.c_void_p), ("compute_dt", C.c_void_p),
        ("get_name", C.c_void_p), ("get_description", C.c_void_p),
        ("get_capabilities", C.c_void_p),
    ]


class PoissonParams(C.Structure):
    _fields_ = [("tolerance", C.c_double), ("absolute_tolerance", C.c_double),
                ("max_iterations", C.c_int), ("omega", C.c_double),
                ("check_interval", C.c_int), ("verbose", C.c_bool),
                ("preconditioner", C.c_int)]


class PoissonStats(C.Structure):
    _fields_ = [("status", C.c_int), ("iterations", C.c_int),
                ("initial_residual", C.c_double), ("final_residual", C.c_double),
                ("elapsed_time_ms", C.c_double)]


class HipProjConfig(C.Structure):
    _fields_ = [
        ("device", C.c_int), ("poisson_method", C.c_int),
        ("poisson_tolerance", C.c_double), ("poisson_abs_tolerance", C.c_double),
        ("poisson_max_iter", C.c_int), ("poisson_check_interval", C.c_int),
        ("sor_omega", C.c_double), ("poll_interval", C.c_int), ("kchunk", C.c_int),
        ("verbose", C.c_int), ("sweep_rows", C.c_int), ("sweep_variant", C.c_int),
        ("rhs_density", C.c_int), ("poisson_fail_fatal", C.c_int), ("relax_two_pass", C.c_int),
        ("sweep_variant_fold", C.c_int),
        ("dirty_faces", C.c_int),
        ("dirty_sync_interval", C.c_int),
        ("cg_variant", C.c_int),
        ("dirty_verify_interval", C.c_int),
    ]


class SimulationData(C.Structure):
    _fields_ = [
        ("grid", C.POINTER(Grid)), ("field", C.POINTER(FlowField)), ("params", SolverParams),
        ("solver", C.POINTER(NSSolver)), ("registry", C.c_void_p),
        ("last_stats", SolverStats), ("outputs", C.c_void_p), ("run_prefix", C.c_char_p),
        ("current_time", C.c_double), ("output_base_dir", C.c_char * 512),
    ]


# gpu_device.h:32-82 (include/cfd_hip/gpu_device.h)
class GpuConfig(C.Structure):
    _fields_ = [
        ("enable_gpu", C.c_int), ("min_grid_size", C.c_size_t), ("min_steps", C.c_int),
        ("block_size_x", C.c_int), ("block_size_y", C.c_int), ("poisson_max_iter", C.c_int),
        ("poisson_tolerance", C.c_double), ("persistent_memory", C.c_int),
        ("async_transfers", C.c_int), ("sync_after_kernel", C.c_int), ("verbose", C.c_int),
    ]


class GpuDeviceInfo(C.Structure):
    _fields_ = [
        ("device_id", C.c_int), ("name", C.c_char * 256), ("total_memory", C.c_size_t),
        ("free_memory", C.c_size_t), ("compute_capability_major", C.c_int),
        ("compute_capability_minor", C.c_int), ("multiprocessor_count", C.c_int),
        ("max_threads_per_block", C.c_int), ("warp_size", C.c_int), ("is_available", C.c_int),
    ]


class GpuSolverStats(C.Structure):
    _fields_ = [
        ("kernel_time_ms", C.c_double), ("transfer_time_ms", C.c_double),
        ("poisson_time_ms", C.c_double), ("poisson_iterations", C.c_int),
        ("poisson_residual", C.c_double), ("memory_allocated", C.c_size_t),
        ("kernels_launched", C.c_int),
    ]


# poisson_solver_method_t / poisson_solver_backend_t (poisson_solver.h)
POISSON_METHOD_JACOBI = 0
POISSON_METHOD_GAUSS_SEIDEL = 1
POISSON_METHOD_SOR = 2
POISSON_METHOD_REDBLACK_SOR = 3
POISSON_METHOD_CG = 4
POISSON_METHOD_BICGSTAB = 5
POISSON_METHOD_MULTIGRID = 6
NS_SOLVER_BACKEND_SCALAR = 0  # ns_solver_backend_t (navier_stokes_solver.h:172-177)
NS_SOLVER_BACKEND_SIMD = 1
NS_SOLVER_BACKEND_OMP = 2
NS_SOLVER_BACKEND_CUDA = 3
# hip_poisson_bc_t (include/cfd_hip/projection_hip.h)
HIP_POISSON_BC_NEUMANN = 0
HIP_POISSON_BC_NONE = 1
HIP_POISSON_BC_FIXED = 2

POISSON_BACKEND_AUTO = 0
POISSON_BACKEND_SCALAR = 1
POISSON_BACKEND_OMP = 2
POISSON_BACKEND_SIMD = 3
POISSON_BACKEND_GPU = 4
POISSON_ERROR = -1


class PoissonSolver(C.Structure):
    _fields_ = [
        ("name", C.c_char_p), ("description", C.c_char_p), ("method", C.c_int),
        ("backend", C.c_int), ("nx", C.c_size_t), ("ny", C.c_size_t), ("nz", C.c_size_t),
        ("dx", C.c_double), ("dy", C.c_double), ("dz", C.c_double),
        ("params", PoissonParams), ("context", C.c_void_p), ("init", C.c_void_p),
        ("destroy", C.c_void_p), ("solve", C.c_void_p), ("iterate", C.c_void_p),
        ("apply_bc", C.c_void_p),
    ]
