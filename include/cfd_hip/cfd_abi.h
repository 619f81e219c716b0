/*
 * cfd_abi.h -- ABI-compatible plain-C types of the shaia/CFD solver-plugin surface.
 *
 * These are the types that cross the drop-in boundary of the Chorin projection
 * hot path. Every struct below has the same member order, member types and
 * therefore the same layout as the reference definitions it cites, so a
 * reference build can hand its own objects to this library (and vice versa)
 * without conversion. Nothing here depends on HIP or on torch.
 *
 * Reference definitions (paths relative to the reference repository):
 *   cfd_status_t             lib/include/cfd/core/cfd_status.h:13-24
 *   grid                     lib/include/cfd/core/grid.h:17-40
 *   bc_type_t                lib/include/cfd/boundary/boundary_conditions.h:19-27
 *   bc_dirichlet_values_t    lib/include/cfd/boundary/boundary_conditions.h:50-57
 *   flow_field               lib/include/cfd/solvers/navier_stokes_solver.h:54-64
 *   ns_source_func_t         lib/include/cfd/solvers/navier_stokes_solver.h:78-81
 *   ns_heat_source_func_t    lib/include/cfd/solvers/navier_stokes_solver.h:92-93
 *   ns_thermal_bc_config_t   lib/include/cfd/solvers/navier_stokes_solver.h:108-116
 *   ns_solver_params_t       lib/include/cfd/solvers/navier_stokes_solver.h:121-158
 *   ns_solver_backend_t      lib/include/cfd/solvers/navier_stokes_solver.h:172-177
 *   ns_solver_capabilities_t lib/include/cfd/solvers/navier_stokes_solver.h:183-192
 *   ns_solver_stats_t        lib/include/cfd/solvers/navier_stokes_solver.h:198-207
 *   struct NSSolver          lib/include/cfd/solvers/navier_stokes_solver.h:254-277
 *   poisson_solver_*         lib/include/cfd/solvers/poisson_solver.h:60-233
 */
#ifndef CFD_HIP_CFD_ABI_H
#define CFD_HIP_CFD_ABI_H

#include <stdbool.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifndef CFD_HIP_EXPORT
#define CFD_HIP_EXPORT __attribute__((visibility("default")))
#endif

#ifdef CFD_HIP_REFERENCE_TYPES
/* Inside a reference build: the reference's own
 * headers define these types, with the layouts restated below. */
#include "cfd/core/cfd_status.h"
#include "cfd/core/grid.h"
#include "cfd/boundary/boundary_conditions.h"
#include "cfd/solvers/navier_stokes_solver.h"
#include "cfd/solvers/poisson_solver.h"
#else

/* ---- status codes (values are part of the ABI) ------------------------- */
typedef enum {
    CFD_SUCCESS = 0,
    CFD_ERROR = -1,
    CFD_ERROR_NOMEM = -2,
    CFD_ERROR_INVALID = -3,
    CFD_ERROR_IO = -4,
    CFD_ERROR_UNSUPPORTED = -5,
    CFD_ERROR_DIVERGED = -6,
    CFD_ERROR_MAX_ITER = -7,
    CFD_ERROR_LIMIT_EXCEEDED = -8,
    CFD_ERROR_NOT_FOUND = -9
} cfd_status_t;

/* ---- structured grid (uniform or stretched coordinates) ----------------- */
typedef struct {
    double* x;
    double* y;
    double* dx;
    double* dy;
    size_t nx;
    size_t ny;
    double xmin;
    double xmax;
    double ymin;
    double ymax;
    double* z;        /* NULL when nz == 1 */
    double* dz;       /* NULL when nz == 1 */
    size_t nz;
    double zmin;
    double zmax;
    size_t stride_z;  /* nx*ny when nz > 1, else 0 */
    double inv_dz2;
    size_t k_start;
    size_t k_end;
} grid;

/* ---- boundary-condition vocabulary -------------------------------------- */
typedef enum {
    BC_TYPE_PERIODIC,
    BC_TYPE_NEUMANN,
    BC_TYPE_DIRICHLET,
    BC_TYPE_NOSLIP,
    BC_TYPE_INLET,
    BC_TYPE_OUTLET,
    BC_TYPE_SYMMETRY
} bc_type_t;

typedef struct {
    double left;    /* i = 0      */
    double right;   /* i = nx-1   */
    double top;     /* j = ny-1   */
    double bottom;  /* j = 0      */
    double front;   /* k = nz-1   */
    double back;    /* k = 0      */
} bc_dirichlet_values_t;

/* ---- flow state: SoA host arrays, x fastest, idx = k*nx*ny + j*nx + i --- */
typedef struct {
    double* u;
    double* v;
    double* w;
    double* p;
    double* rho;
    double* T;
    size_t nx;
    size_t ny;
    size_t nz;
} flow_field;

typedef void (*ns_source_func_t)(double x, double y, double z, double t, void* context,
                                 double* source_u, double* source_v, double* source_w);
typedef double (*ns_heat_source_func_t)(double x, double y, double z, double t, void* context);

typedef struct {
    bc_type_t left;
    bc_type_t right;
    bc_type_t bottom;
    bc_type_t top;
    bc_type_t front;
    bc_type_t back;
    bc_dirichlet_values_t dirichlet_values;
} ns_thermal_bc_config_t;

typedef struct {
    double dt;
    double cfl;
    double gamma;
    double mu;          /* used as kinematic viscosity by the projection step */
    double k;
    int max_iter;
    double tolerance;
    double source_amplitude_u;
    double source_amplitude_v;
    double source_decay_rate;
    double pressure_coupling;
    ns_source_func_t source_func;
    void* source_context;
    double alpha;       /* thermal diffusivity, 0 disables the energy equation */
    double beta;        /* Boussinesq expansion coefficient */
    double T_ref;
    double gravity[3];
    ns_heat_source_func_t heat_source_func;
    void* heat_source_context;
    ns_thermal_bc_config_t thermal_bc;
} ns_solver_params_t;

/* Defaults of ns_solver_params_default() (navier_stokes_solver.h:36-49). */
#define DEFAULT_TIME_STEP            0.001
#define DEFAULT_CFL_NUMBER           0.2
#define DEFAULT_GAMMA                1.4
#define DEFAULT_VISCOSITY            0.01
#define DEFAULT_THERMAL_CONDUCTIVITY 0.0242
#define DEFAULT_MAX_ITERATIONS       100
#define DEFAULT_TOLERANCE            1e-6
#define DEFAULT_SOURCE_AMPLITUDE_U   0.1
#define DEFAULT_SOURCE_AMPLITUDE_V   0.05
#define DEFAULT_SOURCE_DECAY_RATE    0.1
#define DEFAULT_PRESSURE_COUPLING    0.1

/* ---- NS solver plugin vtable -------------------------------------------- */
typedef struct NSSolver ns_solver_t;

typedef enum {
    NS_SOLVER_BACKEND_SCALAR = 0,
    NS_SOLVER_BACKEND_SIMD = 1,
    NS_SOLVER_BACKEND_OMP = 2,
    NS_SOLVER_BACKEND_CUDA = 3  /* the reference's only GPU backend id; HIP solvers report it too */
} ns_solver_backend_t;

typedef enum {
    NS_SOLVER_CAP_NONE = 0,
    NS_SOLVER_CAP_INCOMPRESSIBLE = (1 << 0),
    NS_SOLVER_CAP_COMPRESSIBLE = (1 << 1),
    NS_SOLVER_CAP_STEADY_STATE = (1 << 2),
    NS_SOLVER_CAP_TRANSIENT = (1 << 3),
    NS_SOLVER_CAP_SIMD = (1 << 4),
    NS_SOLVER_CAP_PARALLEL = (1 << 5),
    NS_SOLVER_CAP_GPU = (1 << 6)
} ns_solver_capabilities_t;

typedef struct {
    int iterations;
    double residual;
    double max_velocity;
    double max_pressure;
    double max_temperature;
    double cfl_number;
    double elapsed_time_ms;
    cfd_status_t status;
} ns_solver_stats_t;

typedef void* ns_solver_context_t;

typedef cfd_status_t (*ns_solver_init_func)(ns_solver_t* solver, const grid* grid,
                                            const ns_solver_params_t* params);
typedef void (*ns_solver_destroy_func)(ns_solver_t* solver);
typedef cfd_status_t (*ns_solver_step_func)(ns_solver_t* solver, flow_field* field,
                                            const grid* grid, const ns_solver_params_t* params,
                                            ns_solver_stats_t* stats);
typedef cfd_status_t (*ns_solver_solve_func)(ns_solver_t* solver, flow_field* field,
                                             const grid* grid, const ns_solver_params_t* params,
                                             ns_solver_stats_t* stats);
typedef void (*ns_solver_boundary_func)(ns_solver_t* solver, flow_field* field, const grid* grid);
typedef double (*ns_solver_compute_dt_func)(ns_solver_t* solver, const flow_field* field,
                                            const grid* grid, const ns_solver_params_t* params);
typedef const char* (*ns_solver_get_name_func)(const ns_solver_t* solver);
typedef const char* (*ns_solver_get_description_func)(const ns_solver_t* solver);
typedef ns_solver_capabilities_t (*ns_solver_get_capabilities_func)(const ns_solver_t* solver);

struct NSSolver {
    const char* name;
    const char* description;
    const char* version;
    ns_solver_capabilities_t capabilities;
    ns_solver_backend_t backend;
    ns_solver_context_t context;
    ns_solver_init_func init;
    ns_solver_destroy_func destroy;
    ns_solver_step_func step;
    ns_solver_solve_func solve;
    ns_solver_boundary_func apply_boundary;
    ns_solver_compute_dt_func compute_dt;
    ns_solver_get_name_func get_name;
    ns_solver_get_description_func get_description;
    ns_solver_get_capabilities_func get_capabilities;
};

typedef struct NSSolverRegistry ns_solver_registry_t;
typedef ns_solver_t* (*ns_solver_factory_func)(void);

/* ---- Poisson plugin vtable (secondary boundary) ------------------------- */
typedef enum {
    POISSON_METHOD_JACOBI,
    POISSON_METHOD_GAUSS_SEIDEL,
    POISSON_METHOD_SOR,
    POISSON_METHOD_REDBLACK_SOR,
    POISSON_METHOD_CG,
    POISSON_METHOD_BICGSTAB,
    POISSON_METHOD_MULTIGRID
} poisson_solver_method_t;

typedef enum {
    POISSON_BACKEND_AUTO,
    POISSON_BACKEND_SCALAR,
    POISSON_BACKEND_OMP,
    POISSON_BACKEND_SIMD,
    POISSON_BACKEND_GPU
} poisson_solver_backend_t;

typedef enum {
    POISSON_CONVERGED = 0,
    POISSON_MAX_ITER = 1,
    POISSON_DIVERGED = 2,
    POISSON_STAGNATED = 3,
    POISSON_ERROR = -1
} poisson_solver_status_t;

typedef enum {
    POISSON_PRECOND_NONE = 0,
    POISSON_PRECOND_JACOBI = 1
} poisson_precond_type_t;

typedef struct {
    double tolerance;
    double absolute_tolerance;
    int max_iterations;
    double omega;
    int check_interval;
    bool verbose;
    poisson_precond_type_t preconditioner;
} poisson_solver_params_t;

typedef struct {
    poisson_solver_status_t status;
    int iterations;
    double initial_residual;
    double final_residual;
    double elapsed_time_ms;
} poisson_solver_stats_t;

typedef struct poisson_solver poisson_solver_t;
typedef void* poisson_solver_context_t;

typedef cfd_status_t (*poisson_solver_init_func)(poisson_solver_t* solver, size_t nx, size_t ny,
                                                 size_t nz, double dx, double dy, double dz,
                                                 const poisson_solver_params_t* params);
typedef void (*poisson_solver_destroy_func)(poisson_solver_t* solver);
typedef cfd_status_t (*poisson_solver_solve_func)(poisson_solver_t* solver, double* x,
                                                  double* x_temp, const double* rhs,
                                                  poisson_solver_stats_t* stats);
typedef cfd_status_t (*poisson_solver_iterate_func)(poisson_solver_t* solver, double* x,
                                                    double* x_temp, const double* rhs,
                                                    double* residual);
typedef void (*poisson_solver_apply_bc_func)(poisson_solver_t* solver, double* x);

struct poisson_solver {
    const char* name;
    const char* description;
    poisson_solver_method_t method;
    poisson_solver_backend_t backend;
    size_t nx;
    size_t ny;
    size_t nz;
    double dx;
    double dy;
    double dz;
    poisson_solver_params_t params;
    poisson_solver_context_t context;
    poisson_solver_init_func init;
    poisson_solver_destroy_func destroy;
    poisson_solver_solve_func solve;
    poisson_solver_iterate_func iterate;
    poisson_solver_apply_bc_func apply_bc;
};

#endif /* CFD_HIP_REFERENCE_TYPES */

#ifdef __cplusplus
}
#endif

#endif /* CFD_HIP_CFD_ABI_H */
