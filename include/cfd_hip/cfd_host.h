/*
 * cfd_host.h -- standalone host-side mirror of the reference's public API
 * around the projection hot path (libcfd_host.so).
 *
 * When the HIP projection is dropped into a reference build, the reference
 * provides all of these symbols itself and only libcfd_hip.so is linked. For
 * standalone use (our tests, bench.py, examples) libcfd_host.so provides the
 * same functions with the same signatures and semantics:
 *   errors       lib/include/cfd/core/cfd_status.h:29-46, lib/src/core/logging.c:13-90
 *   grid         lib/include/cfd/core/grid.h:56-88, lib/src/core/grid.c:9-127
 *   flow field   lib/include/cfd/solvers/navier_stokes_solver.h:410-432
 *   BCs (3-D)    lib/include/cfd/boundary/boundary_conditions.h:1222-1255
 *   registry     lib/include/cfd/solvers/navier_stokes_solver.h:291-371,
 *                lib/src/api/solver_registry.c:202-494
 *   simulation   lib/include/cfd/api/simulation_api.h (init_simulation_with_solver,
 *                run_simulation_step, run_simulation_solve, free_simulation,
 *                save/load/restore_simulation_checkpoint)
 *   restart      lib/include/cfd/io/checkpoint.h (cfd_checkpoint_write/read)
 * cfd_registry_register_defaults registers the HIP projection solvers when
 * libcfd_hip.so is loaded in the process (it looks up cfd_hip_register_solvers).
 */
#ifndef CFD_HIP_CFD_HOST_H
#define CFD_HIP_CFD_HOST_H

#include "cfd_hip/cfd_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* errors */
CFD_HIP_EXPORT void cfd_set_error(cfd_status_t status, const char* message);
CFD_HIP_EXPORT const char* cfd_get_last_error(void);
CFD_HIP_EXPORT cfd_status_t cfd_get_last_status(void);
CFD_HIP_EXPORT const char* cfd_get_error_string(cfd_status_t status);
CFD_HIP_EXPORT void cfd_clear_error(void);

/* grid */
CFD_HIP_EXPORT grid* grid_create(size_t nx, size_t ny, size_t nz, double xmin, double xmax,
                                 double ymin, double ymax, double zmin, double zmax);
CFD_HIP_EXPORT void grid_destroy(grid* grid);
CFD_HIP_EXPORT void grid_initialize_uniform(grid* grid);

/* flow field */
CFD_HIP_EXPORT flow_field* flow_field_create(size_t nx, size_t ny, size_t nz);
CFD_HIP_EXPORT void flow_field_destroy(flow_field* field);
CFD_HIP_EXPORT void initialize_flow_field(flow_field* field, const grid* grid);
CFD_HIP_EXPORT ns_solver_params_t ns_solver_params_default(void);
CFD_HIP_EXPORT ns_solver_stats_t ns_solver_stats_default(void);

/* boundary conditions on host arrays */
CFD_HIP_EXPORT cfd_status_t bc_apply_scalar_3d(double* field, size_t nx, size_t ny, size_t nz,
                                               size_t stride_z, bc_type_t type);
CFD_HIP_EXPORT cfd_status_t bc_apply_velocity_3d(double* u, double* v, double* w, size_t nx,
                                                 size_t ny, size_t nz, size_t stride_z,
                                                 bc_type_t type);
CFD_HIP_EXPORT cfd_status_t bc_apply_dirichlet_scalar_3d(double* field, size_t nx, size_t ny,
                                                         size_t nz, size_t stride_z,
                                                         const bc_dirichlet_values_t* values);
CFD_HIP_EXPORT cfd_status_t bc_apply_dirichlet_velocity_3d(
    double* u, double* v, double* w, size_t nx, size_t ny, size_t nz, size_t stride_z,
    const bc_dirichlet_values_t* u_values, const bc_dirichlet_values_t* v_values,
    const bc_dirichlet_values_t* w_values);

/* registry and solver lifecycle */
CFD_HIP_EXPORT ns_solver_registry_t* cfd_registry_create(void);
CFD_HIP_EXPORT void cfd_registry_destroy(ns_solver_registry_t* registry);
CFD_HIP_EXPORT void cfd_registry_register_defaults(ns_solver_registry_t* registry);
CFD_HIP_EXPORT int cfd_registry_register(ns_solver_registry_t* registry, const char* type_name,
                                         ns_solver_factory_func factory);
CFD_HIP_EXPORT int cfd_registry_unregister(ns_solver_registry_t* registry, const char* type_name);
CFD_HIP_EXPORT int cfd_registry_list(ns_solver_registry_t* registry, const char** names,
                                     int max_count);
CFD_HIP_EXPORT int cfd_registry_has(ns_solver_registry_t* registry, const char* type_name);
CFD_HIP_EXPORT const char* cfd_registry_get_description(ns_solver_registry_t* registry,
                                                        const char* type_name);
CFD_HIP_EXPORT ns_solver_t* cfd_solver_create(ns_solver_registry_t* registry,
                                              const char* type_name);
CFD_HIP_EXPORT void solver_destroy(ns_solver_t* solver);
CFD_HIP_EXPORT cfd_status_t solver_init(ns_solver_t* solver, const grid* grid,
                                        const ns_solver_params_t* params);
CFD_HIP_EXPORT cfd_status_t solver_step(ns_solver_t* solver, flow_field* field, const grid* grid,
                                        const ns_solver_params_t* params,
                                        ns_solver_stats_t* stats);
CFD_HIP_EXPORT cfd_status_t solver_solve(ns_solver_t* solver, flow_field* field,
                                         const grid* grid, const ns_solver_params_t* params,
                                         ns_solver_stats_t* stats);
CFD_HIP_EXPORT int cfd_backend_is_available(ns_solver_backend_t backend);
CFD_HIP_EXPORT const char* cfd_backend_get_name(ns_solver_backend_t backend);
/* solver_registry.c:1638-1694: filter by the backend inferred from the name at
 * registration; create only when that backend is available */
CFD_HIP_EXPORT int cfd_registry_list_by_backend(ns_solver_registry_t* registry,
                                                ns_solver_backend_t backend, const char** names,
                                                int max_count);
CFD_HIP_EXPORT ns_solver_t* cfd_solver_create_checked(ns_solver_registry_t* registry,
                                                      const char* type_name);
/* Mirror-only switch (no reference counterpart). 0 (default): the registry
 * behaves like the UNPATCHED reference, whose infer_backend_from_type
 * (solver_registry.c:257-279) knows only `_gpu`, so `projection_hip` is a
 * SCALAR entry, and whose simulation_list_solvers table
 * (simulation_api.c:454-465) lacks the HIP names. 1: the reference with the
 * INTEGRATION.md §1 edits applied (`_hip` -> GPU backend, HIP names listed). */
CFD_HIP_EXPORT void cfd_host_set_hip_patch(int enable);

/* simulation API subset (simulation_api.h) */
typedef struct {
    grid* grid;
    flow_field* field;
    ns_solver_params_t params;
    ns_solver_t* solver;
    ns_solver_registry_t* registry;
    ns_solver_stats_t last_stats;
    void* outputs;          /* output registry: not provided by this mirror (NULL) */
    char* run_prefix;
    double current_time;
    char output_base_dir[512];
} simulation_data;

CFD_HIP_EXPORT simulation_data* init_simulation_with_solver(size_t nx, size_t ny, size_t nz,
                                                            double xmin, double xmax,
                                                            double ymin, double ymax,
                                                            double zmin, double zmax,
                                                            const char* solver_type);
CFD_HIP_EXPORT void free_simulation(simulation_data* sim);
CFD_HIP_EXPORT cfd_status_t run_simulation_step(simulation_data* sim);
CFD_HIP_EXPORT cfd_status_t run_simulation_solve(simulation_data* sim);
CFD_HIP_EXPORT const ns_solver_stats_t* simulation_get_stats(const simulation_data* sim);
/* simulation_api.c:452-478: the static name table (see cfd_host_set_hip_patch) */
CFD_HIP_EXPORT int simulation_list_solvers(const char** names, int max_count);

/* restart files (lib/include/cfd/io/checkpoint.h:49-115, simulation_api.h:93-111):
 * the reference's `.cfdchk` format, status codes and ownership rules */
CFD_HIP_EXPORT cfd_status_t cfd_checkpoint_write(const char* path, const grid* g,
                                                 const flow_field* field,
                                                 const ns_solver_params_t* params,
                                                 double current_time, const char* solver_name,
                                                 const char* run_prefix,
                                                 const char* output_base_dir);
CFD_HIP_EXPORT cfd_status_t cfd_checkpoint_read(const char* path, grid** out_grid,
                                                flow_field** out_field,
                                                ns_solver_params_t* out_params,
                                                double* out_current_time, char* out_solver_name,
                                                size_t solver_name_cap, char* out_run_prefix,
                                                size_t run_prefix_cap, char* out_output_base_dir,
                                                size_t output_base_dir_cap);
CFD_HIP_EXPORT cfd_status_t save_simulation_checkpoint(const simulation_data* sim,
                                                       const char* path);
CFD_HIP_EXPORT simulation_data* load_simulation_from_checkpoint(const char* path);
CFD_HIP_EXPORT cfd_status_t restore_simulation_checkpoint(simulation_data* sim,
                                                          const char* path);

/* ---- legacy VTK output (vtk_output.c:110-275): ASCII STRUCTURED_POINTS,
 * same text as the reference writers. */
CFD_HIP_EXPORT void write_vtk_output(const char* filename, const char* field_name,
                                     const double* data, size_t nx, size_t ny, size_t nz,
                                     double xmin, double xmax, double ymin, double ymax,
                                     double zmin, double zmax);
CFD_HIP_EXPORT void write_vtk_vector_output(const char* filename, const char* field_name,
                                            const double* u_data, const double* v_data,
                                            const double* w_data, size_t nx, size_t ny, size_t nz,
                                            double xmin, double xmax, double ymin, double ymax,
                                            double zmin, double zmax);
CFD_HIP_EXPORT void write_vtk_flow_field(const char* filename, const flow_field* field,
                                         size_t nx, size_t ny, size_t nz, double xmin,
                                         double xmax, double ymin, double ymax, double zmin,
                                         double zmax);

/* ---- Poisson solver interface (poisson_solver.h:132-375, linear_solver.c:25-535)
 * Only POISSON_BACKEND_GPU solvers exist here (the CPU backends are the
 * reference's own); AUTO selects GPU when a HIP device is visible. The
 * factories live in libcfd_hip.so (create_*_gpu_solver) and are found at run
 * time, like the projection plugins. */
CFD_HIP_EXPORT poisson_solver_params_t poisson_solver_params_default(void);
CFD_HIP_EXPORT poisson_solver_stats_t poisson_solver_stats_default(void);
CFD_HIP_EXPORT bool poisson_solver_backend_available(poisson_solver_backend_t backend);
CFD_HIP_EXPORT poisson_solver_t* poisson_solver_create(poisson_solver_method_t method,
                                                       poisson_solver_backend_t backend);
CFD_HIP_EXPORT cfd_status_t poisson_solver_init(poisson_solver_t* solver, size_t nx, size_t ny,
                                                size_t nz, double dx, double dy, double dz,
                                                const poisson_solver_params_t* params);
CFD_HIP_EXPORT void poisson_solver_destroy(poisson_solver_t* solver);
CFD_HIP_EXPORT cfd_status_t poisson_solver_solve(poisson_solver_t* solver, double* x,
                                                 double* x_temp, const double* rhs,
                                                 poisson_solver_stats_t* stats);
CFD_HIP_EXPORT cfd_status_t poisson_solver_iterate(poisson_solver_t* solver, double* x,
                                                   double* x_temp, const double* rhs,
                                                   double* residual);

#ifdef __cplusplus
}
#endif

#endif /* CFD_HIP_CFD_HOST_H */
