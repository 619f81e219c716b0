/*
 * poisson_hip_plugin.c -- the poisson_solver_t GPU backend (POISSON_BACKEND_GPU).
 *
 * The reference's factories create_cg_gpu_solver / create_redblack_gpu_solver /
 * create_jacobi_gpu_solver (declared in lib/src/solvers/linear/linear_solver_internal.h:54-57,
 * reached through poisson_solver_create, linear_solver.c:150-235) under the same
 * names, so the reference's linear_solver.c links them unchanged. Like the
 * reference's backends (poisson_solver_cg_gpu.cu:55-203) they keep host-buffer
 * semantics: solve uploads x and rhs, runs the whole iteration in HBM, and
 * downloads x; iterate and apply_bc stay NULL.
 *
 * Numerics follow the CPU reference the HIP kernels are pinned to (lagged-BC CG,
 * linear_solver_cg.c:290-461; RB-SOR with the odd colour first and the L-inf
 * check, linear_solver_redblack.c:80-147 + linear_solver.c:397-485; Jacobi,
 * linear_solver_jacobi.c:76-129), with the caller's poisson_solver_params_t.
 * BiCGSTAB (create_bicgstab_gpu_solver) is outside the projection path and
 * is not provided.
 */
#include "cfd_hip/projection_hip.h"

#include <stdlib.h>

extern void cfd_set_error(cfd_status_t status, const char* message) __attribute__((weak));

typedef struct {
    hip_proj_ctx_t* ctx;
    int method; /* hip_poisson_method_t */
} poisson_hip_ctx;

static void perr(cfd_status_t s, const char* m) {
    if (cfd_set_error) cfd_set_error(s, m);
}

static cfd_status_t phip_init(poisson_solver_t* solver, size_t nx, size_t ny, size_t nz,
                              double dx, double dy, double dz,
                              const poisson_solver_params_t* params) {
    (void)dx; (void)dy; (void)dz; (void)params;
    if (!hip_projection_available()) {
        perr(CFD_ERROR_UNSUPPORTED, "HIP GPU not available at runtime");
        return CFD_ERROR_UNSUPPORTED;
    }
    poisson_hip_ctx* pc = (poisson_hip_ctx*)solver->context;
    if (!pc) return CFD_ERROR_INVALID;
    if (pc->ctx) {
        hip_proj_destroy(pc->ctx);
        pc->ctx = NULL;
    }
    hip_proj_config_t cfg = hip_proj_config_default();
    cfg.poisson_method = pc->method;
    pc->ctx = hip_proj_create(nx, ny, nz < 1 ? 1 : nz, &cfg);
    if (!pc->ctx) {
        perr(CFD_ERROR_NOMEM, "GPU Poisson: device context creation failed");
        return CFD_ERROR_NOMEM;
    }
    return CFD_SUCCESS;
}

static void phip_destroy(poisson_solver_t* solver) {
    if (!solver || !solver->context) return;
    poisson_hip_ctx* pc = (poisson_hip_ctx*)solver->context;
    if (pc->ctx) hip_proj_destroy(pc->ctx);
    free(pc);
    solver->context = NULL;
}

static cfd_status_t phip_solve(poisson_solver_t* solver, double* x, double* x_temp,
                               const double* rhs, poisson_solver_stats_t* stats) {
    (void)x_temp; /* every working vector lives in HBM */
    if (!solver || !x || !rhs) return CFD_ERROR_INVALID;
    poisson_hip_ctx* pc = (poisson_hip_ctx*)solver->context;
    if (!pc || !pc->ctx) return CFD_ERROR_INVALID;
    double dz = (solver->nz > 1) ? solver->dz : 0.0;
    return hip_proj_poisson_solve(pc->ctx, pc->method, x, rhs, solver->dx, solver->dy, dz,
                                  &solver->params, stats);
}

static poisson_solver_t* make(const char* name, const char* desc,
                              poisson_solver_method_t method, int hip_method) {
    poisson_solver_t* s = (poisson_solver_t*)calloc(1, sizeof(poisson_solver_t));
    poisson_hip_ctx* pc = (poisson_hip_ctx*)calloc(1, sizeof(poisson_hip_ctx));
    if (!s || !pc) {
        free(s);
        free(pc);
        perr(CFD_ERROR_NOMEM, "Failed to allocate GPU Poisson solver");
        return NULL;
    }
    pc->method = hip_method;
    s->name = name;
    s->description = desc;
    s->method = method;
    s->backend = POISSON_BACKEND_GPU;
    /* poisson_solver_params_default (linear_solver.c:37-47) */
    s->params.tolerance = 1e-6;
    s->params.absolute_tolerance = 1e-10;
    s->params.max_iterations = 5000;
    s->params.omega = 0.0;
    s->params.check_interval = 1;
    s->params.verbose = false;
    s->params.preconditioner = POISSON_PRECOND_NONE;
    s->context = pc;
    s->init = phip_init;
    s->destroy = phip_destroy;
    s->solve = phip_solve;
    s->iterate = NULL;
    s->apply_bc = NULL;
    return s;
}

poisson_solver_t* create_cg_gpu_solver(void) {
    return make("cg_gpu", "Conjugate Gradient (HIP, MI355X)", POISSON_METHOD_CG, HIP_POISSON_CG);
}

poisson_solver_t* create_redblack_gpu_solver(void) {
    return make("redblack_gpu", "Red-Black SOR (HIP, MI355X)", POISSON_METHOD_REDBLACK_SOR,
                HIP_POISSON_REDBLACK);
}

poisson_solver_t* create_jacobi_gpu_solver(void) {
    return make("jacobi_gpu", "Jacobi (HIP, MI355X)", POISSON_METHOD_JACOBI, HIP_POISSON_JACOBI);
}
