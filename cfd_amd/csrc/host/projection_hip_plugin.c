/*
 * projection_hip_plugin.c -- the ns_solver_t plugin for the HIP projection step.
 *
 * Mirrors the reference's registry wrappers for the projection solver
 * (lib/src/api/solver_registry.c:895-995 for `projection`, :1121-1181 for
 * `projection_gpu`): init allocates the solver context, step performs exactly
 * one time step (the wrapper's max_iter = 1, :928-929), solve performs
 * params->max_iter steps like solve_projection_method's loop, and the stats
 * are filled like the scalar wrapper (:936-945). The factory returns NULL with
 * CFD_ERROR_UNSUPPORTED when no HIP device is present (:1155-1160), which is
 * how reference test drivers decide to skip.
 */
#include "cfd_hip/projection_hip.h"

#include <stdlib.h>
#include <string.h>

/* Provided by the host library the plugin is loaded into (the reference's
 * libcfd_core or our libcfd_host); weak so the plugin has no hard link to either. */
extern void cfd_set_error(cfd_status_t status, const char* message) __attribute__((weak));
extern int cfd_registry_register(ns_solver_registry_t* registry, const char* type_name,
                                 ns_solver_factory_func factory) __attribute__((weak));

/* Library-internal entry points of projection_hip.hip (hidden visibility). */
#define CFD_HIP_INTERNAL __attribute__((visibility("hidden")))
CFD_HIP_INTERNAL cfd_status_t hip_proj_step_iter_internal(hip_proj_ctx_t* ctx, flow_field* field,
                                                          const grid* g,
                                                          const ns_solver_params_t* params,
                                                          ns_solver_stats_t* stats, int n_steps);
CFD_HIP_INTERNAL cfd_status_t hip_proj_step_host_internal(hip_proj_ctx_t* ctx, flow_field* field,
                                                          const grid* g,
                                                          const ns_solver_params_t* params,
                                                          ns_solver_stats_t* stats);
CFD_HIP_INTERNAL cfd_status_t hip_rk4_step_iter_internal(hip_proj_ctx_t* ctx, flow_field* field,
                                                         const grid* g,
                                                         const ns_solver_params_t* params,
                                                         ns_solver_stats_t* stats, int n_steps);
CFD_HIP_INTERNAL int hip_proj_matches_internal(const hip_proj_ctx_t* ctx, size_t nx, size_t ny,
                                               size_t nz);

typedef struct {
    hip_proj_ctx_t* ctx;
} plugin_ctx;

static void plugin_error(cfd_status_t s, const char* m) {
    if (cfd_set_error) cfd_set_error(s, m);
}

static int method_of(const ns_solver_t* solver) {
    if (solver->name && strcmp(solver->name, NS_SOLVER_TYPE_PROJECTION_HIP_RBSOR) == 0)
        return HIP_POISSON_REDBLACK;
    if (solver->name && strcmp(solver->name, NS_SOLVER_TYPE_PROJECTION_HIP_JACOBI) == 0)
        return HIP_POISSON_JACOBI;
    return HIP_POISSON_CG;
}

/* projection_hip_cg1: the single-reduction CG (cg_variant 1) */
static int cg_variant_of(const ns_solver_t* solver) {
    return (solver->name && strcmp(solver->name, NS_SOLVER_TYPE_PROJECTION_HIP_CG1) == 0) ? 1 : 0;
}

static cfd_status_t get_ctx(ns_solver_t* solver, const grid* g, hip_proj_ctx_t** out) {
    plugin_ctx* pc = (plugin_ctx*)solver->context;
    if (!pc) {
        pc = (plugin_ctx*)calloc(1, sizeof(plugin_ctx));
        if (!pc) return CFD_ERROR_NOMEM;
        solver->context = pc;
    }
    /* rebuild when the grid changes, like poisson_solve_3d's solver cache
     * (linear_solver.c:664-686) */
    if (pc->ctx && !hip_proj_matches_internal(pc->ctx, g->nx, g->ny, g->nz)) {
        hip_proj_destroy(pc->ctx);
        pc->ctx = NULL;
    }
    if (!pc->ctx) {
        hip_proj_config_t cfg = hip_proj_config_default();
        cfg.poisson_method = method_of(solver);
        cfg.cg_variant = cg_variant_of(solver);
        if (cfg.poisson_method == HIP_POISSON_JACOBI) cfg.poisson_max_iter = 2000; /* linear_solver.c:274-276 */
        /* CFD_HIP_DIRTY_FACES=N: the resident mode of `step` with a full
         * download every N steps (the driver's output interval), see
         * hip_proj_config_t.dirty_faces; the reference API has no other way in */
        const char* e = getenv("CFD_HIP_DIRTY_FACES");
        if (e && atoi(e) > 0) {
            cfg.dirty_faces = 1;
            cfg.dirty_sync_interval = atoi(e);
        }
        pc->ctx = hip_proj_create(g->nx, g->ny, g->nz, &cfg);
        if (!pc->ctx) return CFD_ERROR_UNSUPPORTED;
    }
    *out = pc->ctx;
    return CFD_SUCCESS;
}

static cfd_status_t plugin_init(ns_solver_t* solver, const grid* g,
                                const ns_solver_params_t* params) {
    (void)params;
    if (!g) return CFD_ERROR_INVALID;
    if (g->nx < 3 || g->ny < 3 || (g->nz > 1 && g->nz < 3)) return CFD_ERROR_INVALID;
    hip_proj_ctx_t* ctx = NULL;
    return get_ctx(solver, g, &ctx);
}

static void plugin_destroy(ns_solver_t* solver) {
    plugin_ctx* pc = (plugin_ctx*)solver->context;
    if (pc) {
        if (pc->ctx) hip_proj_destroy(pc->ctx);
        free(pc);
        solver->context = NULL;
    }
}

static int is_rk4(const ns_solver_t* solver) {
    return solver->name && strcmp(solver->name, NS_SOLVER_TYPE_RK4_HIP) == 0;
}

/* n steps of the solver's integrator on host buffers */
static cfd_status_t run_steps(ns_solver_t* solver, hip_proj_ctx_t* ctx, flow_field* field,
                              const grid* g, const ns_solver_params_t* params,
                              ns_solver_stats_t* stats, int n) {
    if (is_rk4(solver)) return hip_rk4_step_iter_internal(ctx, field, g, params, stats, n);
    return hip_proj_step_iter_internal(ctx, field, g, params, stats, n);
}

static cfd_status_t plugin_step(ns_solver_t* solver, flow_field* field, const grid* g,
                                const ns_solver_params_t* params, ns_solver_stats_t* stats) {
    if (!field || !g || !params) return CFD_ERROR_INVALID;
    if (field->nx < 3 || field->ny < 3) return CFD_ERROR_INVALID;
    hip_proj_ctx_t* ctx = NULL;
    cfd_status_t s = get_ctx(solver, g, &ctx);
    if (s != CFD_SUCCESS) return s;
    if (!is_rk4(solver)) return hip_proj_step_host_internal(ctx, field, g, params, stats);
    return run_steps(solver, ctx, field, g, params, stats, 1);
}

static cfd_status_t plugin_solve(ns_solver_t* solver, flow_field* field, const grid* g,
                                 const ns_solver_params_t* params, ns_solver_stats_t* stats) {
    if (!field || !g || !params) return CFD_ERROR_INVALID;
    if (field->nx < 3 || field->ny < 3) return CFD_ERROR_INVALID;
    hip_proj_ctx_t* ctx = NULL;
    cfd_status_t s = get_ctx(solver, g, &ctx);
    if (s != CFD_SUCCESS) return s;
    s = run_steps(solver, ctx, field, g, params, stats, params->max_iter);
    if (s == CFD_SUCCESS && stats) stats->iterations = params->max_iter;
    return s;
}

static ns_solver_t* make_solver(const char* name, const char* desc) {
    if (!hip_projection_available()) {
        plugin_error(CFD_ERROR_UNSUPPORTED, "HIP GPU not available at runtime");
        return NULL;
    }
    ns_solver_t* s = (ns_solver_t*)calloc(1, sizeof(*s));
    if (!s) return NULL;
    s->name = name;
    s->description = desc;
    s->version = "0.1.0";
    s->capabilities = NS_SOLVER_CAP_INCOMPRESSIBLE | NS_SOLVER_CAP_TRANSIENT | NS_SOLVER_CAP_GPU;
    s->backend = NS_SOLVER_BACKEND_CUDA;
    s->init = plugin_init;
    s->destroy = plugin_destroy;
    s->step = plugin_step;
    s->solve = plugin_solve;
    s->apply_boundary = NULL;
    s->compute_dt = NULL;
    return s;
}

ns_solver_t* create_projection_hip_solver(void) {
    return make_solver(NS_SOLVER_TYPE_PROJECTION_HIP,
                       "Projection method with CG pressure solve (HIP, MI355X)");
}

ns_solver_t* create_projection_hip_rbsor_solver(void) {
    return make_solver(NS_SOLVER_TYPE_PROJECTION_HIP_RBSOR,
                       "Projection method with Red-Black SOR pressure solve (HIP, MI355X)");
}

ns_solver_t* create_projection_hip_jacobi_solver(void) {
    return make_solver(NS_SOLVER_TYPE_PROJECTION_HIP_JACOBI,
                       "Projection method with Jacobi pressure solve (HIP, MI355X)");
}

ns_solver_t* create_projection_hip_cg1_solver(void) {
    return make_solver(NS_SOLVER_TYPE_PROJECTION_HIP_CG1,
                       "Projection method with single-reduction CG pressure solve "
                       "(Chronopoulos-Gear, one all-reduce per iteration; HIP, MI355X)");
}

/* rk4_hip: rk4_step / rk4_solve (solver_registry.c:748-800) on the device */
ns_solver_t* create_rk4_hip_solver(void) {
    return make_solver(NS_SOLVER_TYPE_RK4_HIP, "RK4 time integration (HIP, MI355X)");
}

void cfd_hip_register_solvers(ns_solver_registry_t* registry) {
    if (!registry || !cfd_registry_register) return;
    cfd_registry_register(registry, NS_SOLVER_TYPE_PROJECTION_HIP, create_projection_hip_solver);
    cfd_registry_register(registry, NS_SOLVER_TYPE_PROJECTION_HIP_RBSOR,
                          create_projection_hip_rbsor_solver);
    cfd_registry_register(registry, NS_SOLVER_TYPE_PROJECTION_HIP_JACOBI,
                          create_projection_hip_jacobi_solver);
    cfd_registry_register(registry, NS_SOLVER_TYPE_RK4_HIP, create_rk4_hip_solver);
    cfd_registry_register(registry, NS_SOLVER_TYPE_PROJECTION_HIP_CG1,
                          create_projection_hip_cg1_solver);
}
