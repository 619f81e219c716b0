/*
 * oracle.h -- TEST INFRASTRUCTURE ONLY. Not part of the product.
 *
 * A plain-C restatement of the shaia/CFD reference's scalar (and OpenMP)
 * Chorin projection path, used as the parity checker for the HIP path and as
 * the timed CPU baseline in bench.py. Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load it. The product library
 * (cfd_amd/lib/libcfd_hip.so) never links or calls anything here.
 *
 * Parity pinning: the reference cannot be compiled here under the build rules
 * (its headers include the CMake-generated cfd/cfd_export.h), so this
 * restatement is pinned by the reference's own golden vectors
 * (tests/solvers/navier_stokes/cpu/test_ns_solver_3d.c:345-348, reproduced
 * bit-exactly) and by reference outputs recorded in SURVEY.md App. B
 * (CG iteration counts, Taylor-Green L2 errors, Ghia RMS). See DESIGN.md.
 *
 * Every function cites the reference file:line it restates.
 */
#ifndef CFD_ORACLE_H
#define CFD_ORACLE_H

#include "cfd_hip/cfd_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Thread count for the OpenMP twin (solver_projection_omp.c / *_omp.c).
 * 1 (default) = the scalar reference path with sequential summation order. */
void oracle_set_threads(int nthreads);
/* Timing-only sampling for the CPU baseline: n > 0 caps the projection's
 * pressure solve at n iterations and accepts the result (0 = off). */
void oracle_set_poisson_cap(int n);
int oracle_get_threads(void);
/* Override the pressure-solver parameters used inside oracle_projection_step
 * (the reference always passes NULL = defaults, linear_solver.c:684); NULL
 * restores the defaults. Used to pair with a HIP context configured alike. */
void oracle_set_projection_poisson_params(const poisson_solver_params_t* p);
/* 1: the projection step's RHS is div(u*) / dt without rho, as the reference
 * GPU computes it (solver_projection_gpu.cu:706-707); 0 (default): (rho / dt)
 * div(u*), solver_projection.c:195-211. */
void oracle_set_gpu_rhs(int on);
/* A caller apply_bc override for the Poisson solvers (solver->apply_bc,
 * linear_solver.c:356-359; test_poisson_3d.c:274): called wherever the
 * reference calls poisson_solver_apply_bc. NULL restores the Neumann default. */
typedef void (*oracle_bc_hook)(double* x, size_t nx, size_t ny, size_t nz, void* ctx);
void oracle_set_poisson_bc_hook(oracle_bc_hook fn, void* ctx);

/* grid.c:9-127 (grid_create + grid_initialize_uniform) */
grid* oracle_grid_create_uniform(size_t nx, size_t ny, size_t nz, double xmin, double xmax,
                                 double ymin, double ymax, double zmin, double zmax);
void oracle_grid_destroy(grid* g);
/* solver_explicit_euler.c:79-122 */
flow_field* oracle_field_create(size_t nx, size_t ny, size_t nz);
void oracle_field_destroy(flow_field* f);
/* solver_explicit_euler.c:58-78 */
ns_solver_params_t oracle_params_default(void);

/* boundary_conditions_core_impl.h:41-186 (x faces, then y faces, then z faces) */
void oracle_bc_neumann_3d(double* f, size_t nx, size_t ny, size_t nz);
void oracle_bc_periodic_3d(double* f, size_t nx, size_t ny, size_t nz);
void oracle_bc_dirichlet_3d(double* f, size_t nx, size_t ny, size_t nz,
                            const bc_dirichlet_values_t* values);
/* linear_solver.c:348-392: z planes by copy, then per-plane x/y Neumann */
void oracle_poisson_apply_bc(double* x, size_t nx, size_t ny, size_t nz);

/* linear_solver.c:37-47 */
poisson_solver_params_t oracle_poisson_params_default(void);

/* linear_solver_cg.c:290-461 (CG and Jacobi-PCG). Returns CFD_SUCCESS when
 * converged, CFD_ERROR_MAX_ITER otherwise (incl. breakdown). */
cfd_status_t oracle_cg_solve(double* x, const double* rhs, size_t nx, size_t ny, size_t nz,
                             double dx, double dy, double dz,
                             const poisson_solver_params_t* params,
                             poisson_solver_stats_t* stats);
/* linear_solver_redblack.c:80-147 driven by linear_solver.c:397-485 */
cfd_status_t oracle_redblack_solve(double* x, const double* rhs, size_t nx, size_t ny, size_t nz,
                                   double dx, double dy, double dz,
                                   const poisson_solver_params_t* params,
                                   poisson_solver_stats_t* stats);
/* linear_solver_jacobi.c:76-129 driven by linear_solver.c:397-485 */
cfd_status_t oracle_jacobi_solve(double* x, double* x_temp, const double* rhs, size_t nx,
                                 size_t ny, size_t nz, double dx, double dy, double dz,
                                 const poisson_solver_params_t* params,
                                 poisson_solver_stats_t* stats);
/* linear_solver.c:304-346 (L-infinity residual of lap(x) - rhs) */
double oracle_poisson_residual_linf(const double* x, const double* rhs, size_t nx, size_t ny,
                                    size_t nz, double dx, double dy, double dz);

/* Pressure solver used inside the projection step. The reference hard-codes
 * CG (solver_projection.c:217-218); the RB-SOR and Jacobi variants exist for
 * the north star's Red-Black-SOR projection configuration. */
typedef enum {
    ORACLE_POISSON_CG = 0,
    ORACLE_POISSON_REDBLACK = 1,
    ORACLE_POISSON_JACOBI = 2
} oracle_poisson_kind_t;

/* One projection step exactly as projection_step (solver_registry.c:921-947)
 * -> solve_projection_method (solver_projection.c:46-297) with max_iter = 1.
 * Fills stats like the wrapper (iterations = 1, max velocity/pressure/T).
 * poisson_iters (optional) receives the pressure-solver iteration count. */
cfd_status_t oracle_projection_step(flow_field* field, const grid* g,
                                    const ns_solver_params_t* params, ns_solver_stats_t* stats,
                                    oracle_poisson_kind_t poisson, int* poisson_iters);

/* Phase timings (ms) of the most recent oracle_projection_step, for the CPU
 * baseline: [0] predictor, [1] divergence, [2] poisson, [3] corrector+rest. */
void oracle_last_phase_ms(double out[4]);
/* Poisson stats (iterations, initial / final residual, status) of the last
 * oracle_projection_step. */
void oracle_last_poisson_stats(poisson_solver_stats_t* out);

/* CG with a fixed iteration count and no early exit (baseline microbench,
 * SURVEY.md §8d). Returns wall ms. */
double oracle_cg_fixed_iters(double* x, const double* rhs, size_t nx, size_t ny, size_t nz,
                             double dx, double dy, double dz, int iters);

/* energy_solver.c:21-176 / :185-196 / :204-334 */
cfd_status_t oracle_energy_step(flow_field* field, const grid* g, const ns_solver_params_t* params,
                                double dt, double time);
cfd_status_t oracle_apply_thermal_bcs(flow_field* field, const ns_solver_params_t* params);

/* One RK4 step as rk4_step (solver_registry.c:748-772) -> rk4_impl
 * (solver_rk4.c:69-259) with max_iter = 1. */
cfd_status_t oracle_rk4_step(flow_field* field, const grid* g, const ns_solver_params_t* params,
                             ns_solver_stats_t* stats);

/* gpu_solver_step (solver_projection_gpu.cu:523-570): the reference device
 * API's explicit pressure-relaxation step (not the projection). */
cfd_status_t oracle_gpu_explicit_step(flow_field* field, const grid* g,
                                      const ns_solver_params_t* params);

/* solver_registry.c:31-62 */
void oracle_max_velocity_pressure(const flow_field* f, double* max_vel, double* max_p);
double oracle_max_temperature(const flow_field* f);

#ifdef __cplusplus
}
#endif

#endif /* CFD_ORACLE_H */
