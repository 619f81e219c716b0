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
 * A caller may override solver->apply_bc (test_poisson_3d.c:274); the
 * reference's CUDA backends ignore it, these honour it:
 *  - CG applies the BC only at solve start and end (linear_solver_cg.c:320,
 *    447), so the override runs on the host around the device solve, which
 *    then never writes boundary cells (HIP_POISSON_BC_NONE): any override;
 *  - RB-SOR / Jacobi apply it after every iteration. An override that
 *    leaves the interior alone and writes x-independent boundary values
 *    (Dirichlet; "keep the caller's boundary"; any mix per cell) is found by
 *    calling it on two different probe arrays (probe_bc); the boundary it
 *    leaves is then imposed on the device after every iteration
 *    (HIP_POISSON_BC_FIXED). Other overrides are CFD_ERROR_UNSUPPORTED.
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
#include <string.h>

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

static int interior_cell(const poisson_solver_t* s, size_t e) {
    const size_t nx = s->nx, ny = s->ny, nz = s->nz < 1 ? 1 : s->nz;
    const size_t i = e % nx, j = (e / nx) % ny, k = e / (nx * ny);
    const int kin = (nz > 1) ? (k >= 1 && k <= nz - 2) : 1;
    return i >= 1 && i <= nx - 2 && j >= 1 && j <= ny - 2 && kin;
}

/* The boundary an apply_bc override leaves after every relaxation iteration,
 * found by running it on two unrelated probe arrays. It must leave interior
 * cells alone; each boundary cell is either written with the same value in
 * both probes (that value is kept) or left untouched in both (the cell then
 * keeps keep[e]: x's own value for RB-SOR, whose sweeps never write boundary
 * cells, or x_temp's for Jacobi, whose memcpy(x, x_temp) brings it in,
 * linear_solver_jacobi.c:118). Returns the full-size array of boundary values
 * (interior entries unused), or NULL for an override outside this class. */
static double probe_a(size_t e) { return 0.5 + (double)(e % 97) * 0.015625; }
static double probe_b(size_t e) { return -3.0 - (double)(e % 89) * 0.0078125; }

static double* probe_bc(poisson_solver_t* s, const double* keep) {
    const size_t n = s->nx * s->ny * (s->nz < 1 ? 1 : s->nz);
    double* a = (double*)malloc(n * sizeof(double));
    double* b = (double*)malloc(n * sizeof(double));
    if (!a || !b) {
        free(a);
        free(b);
        return NULL;
    }
    for (size_t e = 0; e < n; e++) {
        a[e] = probe_a(e);
        b[e] = probe_b(e);
    }
    s->apply_bc(s, a);
    s->apply_bc(s, b);
    int ok = 1;
    for (size_t e = 0; e < n && ok; e++) {
        const int untouched = a[e] == probe_a(e) && b[e] == probe_b(e);
        if (interior_cell(s, e)) ok = untouched;
        else if (untouched) a[e] = keep[e];
        else ok = memcmp(&a[e], &b[e], sizeof(double)) == 0;
    }
    free(b);
    if (!ok) {
        free(a);
        return NULL;
    }
    return a;
}

static cfd_status_t phip_solve(poisson_solver_t* solver, double* x, double* x_temp,
                               const double* rhs, poisson_solver_stats_t* stats) {
    /* every working vector lives in HBM; x_temp only supplies the boundary
     * a Jacobi apply_bc override leaves untouched */
    if (!solver || !x || !rhs) return CFD_ERROR_INVALID;
    poisson_hip_ctx* pc = (poisson_hip_ctx*)solver->context;
    if (!pc || !pc->ctx) return CFD_ERROR_INVALID;
    double dz = (solver->nz > 1) ? solver->dz : 0.0;
    if (pc->method == HIP_POISSON_JACOBI && !x_temp) {
        perr(CFD_ERROR_INVALID, "Jacobi requires a temp buffer"); /* linear_solver_jacobi.c:83-85 */
        return CFD_ERROR_INVALID;
    }
    if (!solver->apply_bc)
        return hip_proj_poisson_solve(pc->ctx, pc->method, x, rhs, solver->dx, solver->dy, dz,
                                      &solver->params, stats);
    if (pc->method == HIP_POISSON_CG) {
        poisson_solver_stats_t st;
        memset(&st, 0, sizeof(st));
        solver->apply_bc(solver, x); /* linear_solver_cg.c:320 */
        cfd_status_t r = hip_proj_poisson_solve_ex(pc->ctx, pc->method, x, rhs, solver->dx,
                                                   solver->dy, dz, &solver->params, &st,
                                                   HIP_POISSON_BC_NONE, NULL);
        /* :447, skipped by the breakdown exits and the converged-at-start return */
        const int early = st.status == POISSON_STAGNATED ||
                          (st.iterations == 0 && st.status == POISSON_CONVERGED);
        if ((r == CFD_SUCCESS || r == CFD_ERROR_MAX_ITER) && !early) solver->apply_bc(solver, x);
        if (stats) *stats = st;
        return r;
    }
    double* vals = probe_bc(solver, pc->method == HIP_POISSON_JACOBI ? x_temp : x);
    if (!vals) {
        perr(CFD_ERROR_UNSUPPORTED,
             "GPU Poisson: a relaxation apply_bc override must leave the interior alone and, "
             "per boundary cell, keep it or write an x-independent value; use CG otherwise");
        return CFD_ERROR_UNSUPPORTED;
    }
    cfd_status_t r = hip_proj_poisson_solve_ex(pc->ctx, pc->method, x, rhs, solver->dx,
                                               solver->dy, dz, &solver->params, stats,
                                               HIP_POISSON_BC_FIXED, vals);
    free(vals);
    return r;
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
