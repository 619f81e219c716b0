/*
 * cfd_oracle.c -- TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * CPU restatement of the reference scalar projection path. Arithmetic is
 * written operation-for-operation in the same order as the reference so that
 * a -ffp-contract=off build reproduces the reference's golden vectors bit for
 * bit. With oracle_set_threads(n > 1) the same loops run under OpenMP (the
 * reference's projection_omp / cg_omp twins); only the summation order of
 * the dot products changes then.
 */
#include "oracle.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

#define MAX_VELOCITY 100.0           /* solver_projection.c:40 */
#define CG_BREAKDOWN_THRESHOLD 1e-30 /* linear_solver_internal.h:73 */

static int g_threads = 1;
static int g_poisson_cap = 0; /* >0: timing-only sample, CG capped and accepted */
static int g_have_pparams = 0;
static int g_gpu_rhs = 0;     /* 1: rhs = div / dt, the reference GPU's (solver_projection_gpu.cu:706-707) */
static poisson_solver_params_t g_pparams;
static double g_phase_ms[4];
static poisson_solver_stats_t g_last_pst; /* the last projection step's Poisson stats */

void oracle_set_threads(int n) { g_threads = n < 1 ? 1 : n; }
void oracle_set_poisson_cap(int n) { g_poisson_cap = n < 0 ? 0 : n; }
void oracle_set_projection_poisson_params(const poisson_solver_params_t* p) {
    g_have_pparams = p != NULL;
    if (p) g_pparams = *p;
}
void oracle_set_gpu_rhs(int on) { g_gpu_rhs = on ? 1 : 0; }
int oracle_get_threads(void) { return g_threads; }
void oracle_last_phase_ms(double out[4]) { memcpy(out, g_phase_ms, sizeof(g_phase_ms)); }
void oracle_last_poisson_stats(poisson_solver_stats_t* out) { if (out) *out = g_last_pst; }

static double now_ms(void) {
    struct timeval tv;
    gettimeofday(&tv, NULL);
    return tv.tv_sec * 1000.0 + tv.tv_usec / 1000.0;
}

#define DO_PRAGMA(x) _Pragma(#x)
#define PAR DO_PRAGMA(omp parallel for collapse(2) schedule(static) if(g_threads > 1) num_threads(g_threads))
#define PAR_SUM(v) DO_PRAGMA(omp parallel for collapse(2) schedule(static) reduction(+:v) if(g_threads > 1) num_threads(g_threads))
/* L-inf is a max, so a parallel reduction is bitwise the sequential one */
#define PAR_MAX(v) DO_PRAGMA(omp parallel for collapse(2) schedule(static) reduction(max:v) if(g_threads > 1) num_threads(g_threads))

/* ------------------------------------------------------------------------ */
/* grid / field / params (grid.c:9-127, solver_explicit_euler.c:58-122)     */
/* ------------------------------------------------------------------------ */
grid* oracle_grid_create_uniform(size_t nx, size_t ny, size_t nz, double xmin, double xmax,
                                 double ymin, double ymax, double zmin, double zmax) {
    grid* g = (grid*)calloc(1, sizeof(grid));
    if (!g) return NULL;
    g->nx = nx; g->ny = ny; g->nz = nz;
    g->xmin = xmin; g->xmax = xmax; g->ymin = ymin; g->ymax = ymax;
    g->x = (double*)calloc(nx, sizeof(double));
    g->y = (double*)calloc(ny, sizeof(double));
    g->dx = (double*)calloc(nx - 1, sizeof(double));
    g->dy = (double*)calloc(ny - 1, sizeof(double));
    double dx = (xmax - xmin) / (nx - 1);
    double dy = (ymax - ymin) / (ny - 1);
    for (size_t i = 0; i < nx; i++) g->x[i] = xmin + (i * dx);
    for (size_t j = 0; j < ny; j++) g->y[j] = ymin + (j * dy);
    for (size_t i = 0; i < nx - 1; i++) g->dx[i] = dx;
    for (size_t j = 0; j < ny - 1; j++) g->dy[j] = dy;
    if (nz > 1) {
        g->zmin = zmin; g->zmax = zmax;
        g->z = (double*)calloc(nz, sizeof(double));
        g->dz = (double*)calloc(nz - 1, sizeof(double));
        g->stride_z = nx * ny;
        g->k_start = 1; g->k_end = nz - 1;
        double dzv = (zmax - zmin) / (nz - 1);
        for (size_t k = 0; k < nz; k++) g->z[k] = zmin + (k * dzv);
        for (size_t k = 0; k < nz - 1; k++) g->dz[k] = dzv;
        g->inv_dz2 = 1.0 / (dzv * dzv);
    } else {
        g->k_start = 0; g->k_end = 1;
    }
    return g;
}

void oracle_grid_destroy(grid* g) {
    if (!g) return;
    free(g->x); free(g->y); free(g->dx); free(g->dy); free(g->z); free(g->dz);
    free(g);
}

flow_field* oracle_field_create(size_t nx, size_t ny, size_t nz) {
    flow_field* f = (flow_field*)calloc(1, sizeof(flow_field));
    if (!f) return NULL;
    size_t n = nx * ny * nz;
    f->nx = nx; f->ny = ny; f->nz = nz;
    f->u = (double*)calloc(n, sizeof(double));
    f->v = (double*)calloc(n, sizeof(double));
    f->w = (double*)calloc(n, sizeof(double));
    f->p = (double*)calloc(n, sizeof(double));
    f->rho = (double*)calloc(n, sizeof(double));
    f->T = (double*)calloc(n, sizeof(double));
    return f;
}

void oracle_field_destroy(flow_field* f) {
    if (!f) return;
    free(f->u); free(f->v); free(f->w); free(f->p); free(f->rho); free(f->T);
    free(f);
}

ns_solver_params_t oracle_params_default(void) {
    ns_solver_params_t p;
    memset(&p, 0, sizeof(p));
    p.dt = DEFAULT_TIME_STEP;
    p.cfl = DEFAULT_CFL_NUMBER;
    p.gamma = DEFAULT_GAMMA;
    p.mu = DEFAULT_VISCOSITY;
    p.k = DEFAULT_THERMAL_CONDUCTIVITY;
    p.max_iter = DEFAULT_MAX_ITERATIONS;
    p.tolerance = DEFAULT_TOLERANCE;
    p.source_amplitude_u = DEFAULT_SOURCE_AMPLITUDE_U;
    p.source_amplitude_v = DEFAULT_SOURCE_AMPLITUDE_V;
    p.source_decay_rate = DEFAULT_SOURCE_DECAY_RATE;
    p.pressure_coupling = DEFAULT_PRESSURE_COUPLING;
    return p;
}

/* ------------------------------------------------------------------------ */
/* boundary conditions (boundary_conditions_core_impl.h:41-186)              */
/* ------------------------------------------------------------------------ */
void oracle_bc_neumann_3d(double* f, size_t nx, size_t ny, size_t nz) {
    size_t sz = (nz > 1) ? nx * ny : 0;
    for (size_t k = 0; k < nz; k++) {
        size_t b = k * sz;
        for (size_t j = 0; j < ny; j++) {
            f[b + j * nx] = f[b + j * nx + 1];
            f[b + j * nx + nx - 1] = f[b + j * nx + nx - 2];
        }
    }
    for (size_t k = 0; k < nz; k++) {
        size_t b = k * sz;
        for (size_t i = 0; i < nx; i++) {
            f[b + i] = f[b + nx + i];
            f[b + (ny - 1) * nx + i] = f[b + (ny - 2) * nx + i];
        }
    }
    if (nz > 1) {
        size_t plane = nx * ny;
        for (size_t i = 0; i < plane; i++) {
            f[i] = f[sz + i];
            f[(nz - 1) * sz + i] = f[(nz - 2) * sz + i];
        }
    }
}

void oracle_bc_periodic_3d(double* f, size_t nx, size_t ny, size_t nz) {
    size_t sz = (nz > 1) ? nx * ny : 0;
    for (size_t k = 0; k < nz; k++) {
        size_t b = k * sz;
        for (size_t j = 0; j < ny; j++) {
            f[b + j * nx] = f[b + j * nx + nx - 2];
            f[b + j * nx + nx - 1] = f[b + j * nx + 1];
        }
    }
    for (size_t k = 0; k < nz; k++) {
        size_t b = k * sz;
        for (size_t i = 0; i < nx; i++) {
            f[b + i] = f[b + (ny - 2) * nx + i];
            f[b + (ny - 1) * nx + i] = f[b + nx + i];
        }
    }
    if (nz > 1) {
        size_t plane = nx * ny;
        for (size_t i = 0; i < plane; i++) {
            f[i] = f[(nz - 2) * sz + i];
            f[(nz - 1) * sz + i] = f[sz + i];
        }
    }
}

void oracle_bc_dirichlet_3d(double* f, size_t nx, size_t ny, size_t nz,
                            const bc_dirichlet_values_t* v) {
    size_t sz = (nz > 1) ? nx * ny : 0;
    for (size_t k = 0; k < nz; k++) {
        size_t b = k * sz;
        for (size_t j = 0; j < ny; j++) {
            f[b + j * nx] = v->left;
            f[b + j * nx + nx - 1] = v->right;
        }
    }
    for (size_t k = 0; k < nz; k++) {
        size_t b = k * sz;
        for (size_t i = 0; i < nx; i++) {
            f[b + i] = v->bottom;
            f[b + (ny - 1) * nx + i] = v->top;
        }
    }
    if (nz > 1) {
        size_t plane = nx * ny;
        for (size_t i = 0; i < plane; i++) {
            f[i] = v->back;
            f[(nz - 1) * sz + i] = v->front;
        }
    }
}

void oracle_poisson_apply_bc(double* x, size_t nx, size_t ny, size_t nz) {
    size_t plane = nx * ny;
    if (nz > 1) {
        memcpy(x, x + plane, plane * sizeof(double));
        memcpy(x + (nz - 1) * plane, x + (nz - 2) * plane, plane * sizeof(double));
    }
    for (size_t k = 0; k < nz; k++) oracle_bc_neumann_3d(x + k * plane, nx, ny, 1);
}

/* poisson_solver_apply_bc (linear_solver.c:348-359): the caller's apply_bc
 * override when one is installed, else the default Neumann BC above */
static oracle_bc_hook g_bc_hook = NULL;
static void* g_bc_hook_ctx = NULL;
void oracle_set_poisson_bc_hook(oracle_bc_hook fn, void* ctx) {
    g_bc_hook = fn;
    g_bc_hook_ctx = ctx;
}
static void solver_apply_bc(double* x, size_t nx, size_t ny, size_t nz) {
    if (g_bc_hook) g_bc_hook(x, nx, ny, nz, g_bc_hook_ctx);
    else oracle_poisson_apply_bc(x, nx, ny, nz);
}

/* ------------------------------------------------------------------------ */
/* Poisson solvers                                                           */
/* ------------------------------------------------------------------------ */
poisson_solver_params_t oracle_poisson_params_default(void) {
    poisson_solver_params_t p;
    memset(&p, 0, sizeof(p));
    p.tolerance = 1e-6;
    p.absolute_tolerance = 1e-10;
    p.max_iterations = 5000;
    p.omega = 0.0;
    p.check_interval = 1;
    p.verbose = false;
    p.preconditioner = POISSON_PRECOND_NONE;
    return p;
}

typedef struct {
    size_t nx, ny, nz, sz, k0, k1;
    double dx2_inv, dy2_inv, inv_dz2;
} lap_geom;

/* linear_solver_internal.h:157-171 and linear_solver_cg.c:202-210 */
static lap_geom make_geom(size_t nx, size_t ny, size_t nz, double dx, double dy, double dz) {
    lap_geom g;
    g.nx = nx; g.ny = ny; g.nz = nz;
    g.sz = (nz > 1) ? nx * ny : 0;
    g.k0 = (nz > 1) ? 1 : 0;
    g.k1 = (nz > 1) ? nz - 1 : 1;
    double dx2 = dx * dx, dy2 = dy * dy;
    g.dx2_inv = 1.0 / dx2;
    g.dy2_inv = 1.0 / dy2;
    g.inv_dz2 = (dz > 0.0) ? (1.0 / (dz * dz)) : 0.0;
    return g;
}

/* linear_solver_cg.c:67-80 */
static double dot(const lap_geom* g, const double* a, const double* b) {
    double sum = 0.0;
    size_t nx = g->nx, ny = g->ny, sz = g->sz;
    PAR_SUM(sum)
    for (size_t k = g->k0; k < g->k1; k++)
        for (size_t j = 1; j < ny - 1; j++)
            for (size_t i = 1; i < nx - 1; i++) {
                size_t idx = k * sz + j * nx + i;
                sum += a[idx] * b[idx];
            }
    return sum;
}

/* linear_solver_cg.c:85-96 */
static void axpy(const lap_geom* g, double alpha, const double* x, double* y) {
    size_t nx = g->nx, ny = g->ny, sz = g->sz;
    PAR
    for (size_t k = g->k0; k < g->k1; k++)
        for (size_t j = 1; j < ny - 1; j++)
            for (size_t i = 1; i < nx - 1; i++) {
                size_t idx = k * sz + j * nx + i;
                y[idx] += alpha * x[idx];
            }
}

/* linear_solver_cg.c:103-123: the Laplacian term exactly as the reference
 * groups it (x and y terms as (a - 2c) + b, z term as (a + b) - 2c). */
static inline double lap_at(const lap_geom* g, const double* p, size_t idx) {
    size_t nx = g->nx, sz = g->sz;
    return ((p[idx + 1] - (2.0 * p[idx]) + p[idx - 1]) * g->dx2_inv) +
           ((p[idx + nx] - (2.0 * p[idx]) + p[idx - nx]) * g->dy2_inv) +
           ((p[idx + sz] + p[idx - sz] - (2.0 * p[idx])) * g->inv_dz2);
}

static void apply_neg_laplacian(const lap_geom* g, const double* p, double* Ap) {
    size_t nx = g->nx, ny = g->ny, sz = g->sz;
    PAR
    for (size_t k = g->k0; k < g->k1; k++)
        for (size_t j = 1; j < ny - 1; j++)
            for (size_t i = 1; i < nx - 1; i++) {
                size_t idx = k * sz + j * nx + i;
                Ap[idx] = -lap_at(g, p, idx);
            }
}

cfd_status_t oracle_cg_solve(double* x, const double* rhs, size_t nx, size_t ny, size_t nz,
                             double dx, double dy, double dz,
                             const poisson_solver_params_t* params_in,
                             poisson_solver_stats_t* stats) {
    poisson_solver_params_t prm = params_in ? *params_in : oracle_poisson_params_default();
    lap_geom g = make_geom(nx, ny, nz, dx, dy, dz);
    size_t n = nx * ny * nz, sz = g.sz;
    int use_pc = (prm.preconditioner == POISSON_PRECOND_JACOBI);
    /* linear_solver_cg.c:212-213 */
    double diag_inv = 1.0 / (2.0 / (dx * dx) + 2.0 / (dy * dy) + 2.0 * g.inv_dz2);
    double* r = (double*)calloc(n, sizeof(double));
    double* p = (double*)calloc(n, sizeof(double));
    double* Ap = (double*)calloc(n, sizeof(double));
    double* z = use_pc ? (double*)calloc(n, sizeof(double)) : NULL;
    cfd_status_t ret = CFD_ERROR_MAX_ITER;
    int iter = 0;
    double res_norm = 0.0;
    int converged = 0;
    if (stats) {
        stats->status = POISSON_ERROR;
        stats->iterations = 0;
        stats->initial_residual = stats->final_residual = stats->elapsed_time_ms = 0.0;
    }
    double t0 = now_ms();

    solver_apply_bc(x, nx, ny, nz);                             /* cg.c:320 */
    PAR                                                          /* cg.c:134-158 */
    for (size_t k = g.k0; k < g.k1; k++)
        for (size_t j = 1; j < ny - 1; j++)
            for (size_t i = 1; i < nx - 1; i++) {
                size_t idx = k * sz + j * nx + i;
                double lap = lap_at(&g, x, idx);
                r[idx] = -rhs[idx] + lap;
            }
    double rho;
    if (use_pc) {
        PAR
        for (size_t k = g.k0; k < g.k1; k++)
            for (size_t j = 1; j < ny - 1; j++)
                for (size_t i = 1; i < nx - 1; i++) {
                    size_t idx = k * sz + j * nx + i;
                    z[idx] = diag_inv * r[idx];
                    p[idx] = z[idx];
                }
        rho = dot(&g, r, z);
    } else {
        PAR
        for (size_t k = g.k0; k < g.k1; k++)
            for (size_t j = 1; j < ny - 1; j++)
                for (size_t i = 1; i < nx - 1; i++) {
                    size_t idx = k * sz + j * nx + i;
                    p[idx] = r[idx];
                }
        rho = dot(&g, r, r);
    }
    double initial_res = sqrt(dot(&g, r, r));                   /* cg.c:345 */
    if (stats) stats->initial_residual = initial_res;
    double tolerance = prm.tolerance * initial_res;             /* cg.c:352-355 */
    if (tolerance < prm.absolute_tolerance) tolerance = prm.absolute_tolerance;
    if (initial_res < prm.absolute_tolerance) {                 /* cg.c:357-365 */
        if (stats) {
            stats->status = POISSON_CONVERGED;
            stats->iterations = 0;
            stats->final_residual = initial_res;
            stats->elapsed_time_ms = now_ms() - t0;
        }
        ret = CFD_SUCCESS;
        goto out;
    }
    res_norm = initial_res;
    for (iter = 0; iter < prm.max_iterations; iter++) {         /* cg.c:367-439 */
        apply_neg_laplacian(&g, p, Ap);
        double pAp = dot(&g, p, Ap);
        if (fabs(pAp) < CG_BREAKDOWN_THRESHOLD) goto breakdown;
        double alpha = rho / pAp;
        axpy(&g, alpha, p, x);
        axpy(&g, -alpha, Ap, r);
        double rho_new;
        if (use_pc) {
            PAR
            for (size_t k = g.k0; k < g.k1; k++)
                for (size_t j = 1; j < ny - 1; j++)
                    for (size_t i = 1; i < nx - 1; i++) {
                        size_t idx = k * sz + j * nx + i;
                        z[idx] = diag_inv * r[idx];
                    }
            rho_new = dot(&g, r, z);
        } else {
            rho_new = dot(&g, r, r);
        }
        res_norm = sqrt(dot(&g, r, r));
        if (iter % prm.check_interval == 0) {
            if (res_norm < tolerance || res_norm < prm.absolute_tolerance) {
                converged = 1;
                break;
            }
        }
        if (fabs(rho) < CG_BREAKDOWN_THRESHOLD) goto breakdown;
        double beta = rho_new / rho;
        const double* src = use_pc ? z : r;
        PAR
        for (size_t k = g.k0; k < g.k1; k++)
            for (size_t j = 1; j < ny - 1; j++)
                for (size_t i = 1; i < nx - 1; i++) {
                    size_t idx = k * sz + j * nx + i;
                    p[idx] = src[idx] + beta * p[idx];
                }
        rho = rho_new;
    }
    if (!converged && (res_norm < tolerance || res_norm < prm.absolute_tolerance)) converged = 1;
    solver_apply_bc(x, nx, ny, nz);                             /* cg.c:447 */
    if (stats) {
        stats->iterations = (iter < prm.max_iterations) ? (iter + 1) : iter;
        stats->final_residual = res_norm;
        stats->elapsed_time_ms = now_ms() - t0;
        stats->status = converged ? POISSON_CONVERGED : POISSON_MAX_ITER;
    }
    ret = converged ? CFD_SUCCESS : CFD_ERROR_MAX_ITER;
    goto out;
breakdown:                                                       /* linear_solver_internal.h:84-96 */
    if (stats) {
        stats->status = POISSON_STAGNATED;
        stats->iterations = iter + 1;
        stats->final_residual = res_norm;
        stats->elapsed_time_ms = now_ms() - t0;
    }
    ret = CFD_ERROR_MAX_ITER;
out:
    free(r); free(p); free(Ap); free(z);
    return ret;
}

double oracle_cg_fixed_iters(double* x, const double* rhs, size_t nx, size_t ny, size_t nz,
                             double dx, double dy, double dz, int iters) {
    lap_geom g = make_geom(nx, ny, nz, dx, dy, dz);
    size_t n = nx * ny * nz, sz = g.sz;
    double* r = (double*)calloc(n, sizeof(double));
    double* p = (double*)calloc(n, sizeof(double));
    double* Ap = (double*)calloc(n, sizeof(double));
    PAR
    for (size_t k = g.k0; k < g.k1; k++)
        for (size_t j = 1; j < ny - 1; j++)
            for (size_t i = 1; i < nx - 1; i++) {
                size_t idx = k * sz + j * nx + i;
                r[idx] = -rhs[idx] + lap_at(&g, x, idx);
                p[idx] = r[idx];
            }
    double rho = dot(&g, r, r);
    double t0 = now_ms();
    for (int it = 0; it < iters; it++) {
        apply_neg_laplacian(&g, p, Ap);
        double pAp = dot(&g, p, Ap);
        double alpha = rho / pAp;
        axpy(&g, alpha, p, x);
        axpy(&g, -alpha, Ap, r);
        double rho_new = dot(&g, r, r);
        double res = sqrt(dot(&g, r, r));
        (void)res;
        double beta = rho_new / rho;
        PAR
        for (size_t k = g.k0; k < g.k1; k++)
            for (size_t j = 1; j < ny - 1; j++)
                for (size_t i = 1; i < nx - 1; i++) {
                    size_t idx = k * sz + j * nx + i;
                    p[idx] = r[idx] + beta * p[idx];
                }
        rho = rho_new;
    }
    double t = now_ms() - t0;
    free(r); free(p); free(Ap);
    return t;
}

double oracle_poisson_residual_linf(const double* x, const double* rhs, size_t nx, size_t ny,
                                    size_t nz, double dx, double dy, double dz) {
    /* linear_solver.c:304-346: note this one divides by dx^2 instead of
     * multiplying by its inverse. */
    double dx2 = dx * dx, dy2 = dy * dy;
    double inv_dz2 = (dz > 0.0) ? (1.0 / (dz * dz)) : 0.0;
    size_t sz = (nz > 1) ? nx * ny : 0, k0 = (nz > 1) ? 1 : 0, k1 = (nz > 1) ? nz - 1 : 1;
    double mx = 0.0;
    PAR_MAX(mx)
    for (size_t k = k0; k < k1; k++)
        for (size_t j = 1; j < ny - 1; j++)
            for (size_t i = 1; i < nx - 1; i++) {
                size_t idx = k * sz + j * nx + i;
                double lap = (x[idx + 1] - 2.0 * x[idx] + x[idx - 1]) / dx2 +
                             (x[idx + nx] - 2.0 * x[idx] + x[idx - nx]) / dy2 +
                             (x[idx + sz] + x[idx - sz] - 2.0 * x[idx]) * inv_dz2;
                double res = fabs(lap - rhs[idx]);
                if (res > mx) mx = res;
            }
    return mx;
}

/* linear_solver_internal.h:184-220 */
static double optimal_omega(size_t nx, size_t ny, size_t nz, double dx, double dy, double dz) {
    double inv_dx2 = 1.0 / (dx * dx);
    double inv_dy2 = 1.0 / (dy * dy);
    double inv_dz2 = (dz > 0.0) ? (1.0 / (dz * dz)) : 0.0;
    double num = cos(M_PI / (double)(nx - 1)) * inv_dx2 + cos(M_PI / (double)(ny - 1)) * inv_dy2;
    double denom = inv_dx2 + inv_dy2;
    if (nz > 1 && inv_dz2 > 0.0) {
        num += cos(M_PI / (double)(nz - 1)) * inv_dz2;
        denom += inv_dz2;
    }
    double rho_j = num / denom;
    return 2.0 / (1.0 + sqrt(1.0 - (rho_j * rho_j)));
}

/* linear_solver.c:397-485 with the scalar iterate functions */
typedef void (*sweep_fn)(void* ctx, double* x, double* xt, const double* rhs);

static cfd_status_t solve_common(sweep_fn sweep, void* ctx, double* x, double* xt,
                                 const double* rhs, size_t nx, size_t ny, size_t nz, double dx,
                                 double dy, double dz, const poisson_solver_params_t* prm,
                                 poisson_solver_stats_t* stats) {
    double t0 = now_ms();
    double initial_res = oracle_poisson_residual_linf(x, rhs, nx, ny, nz, dx, dy, dz);
    double tolerance = prm->tolerance * initial_res;
    if (tolerance < prm->absolute_tolerance) tolerance = prm->absolute_tolerance;
    if (stats) stats->initial_residual = initial_res;
    if (initial_res < prm->absolute_tolerance) {
        if (stats) {
            stats->status = POISSON_CONVERGED;
            stats->iterations = 0;
            stats->final_residual = initial_res;
            stats->elapsed_time_ms = now_ms() - t0;
        }
        return CFD_SUCCESS;
    }
    int converged = 0, iter;
    double res = initial_res;
    for (iter = 0; iter < prm->max_iterations; iter++) {
        sweep(ctx, x, xt, rhs);
        if (iter % prm->check_interval == 0) {
            res = oracle_poisson_residual_linf(x, rhs, nx, ny, nz, dx, dy, dz);
            if (res < tolerance || res < prm->absolute_tolerance) {
                converged = 1;
                break;
            }
        }
    }
    if (stats) {
        stats->iterations = iter + 1;
        stats->final_residual = res;
        stats->elapsed_time_ms = now_ms() - t0;
        stats->status = converged ? POISSON_CONVERGED : POISSON_MAX_ITER;
    }
    return converged ? CFD_SUCCESS : CFD_ERROR_MAX_ITER;
}

typedef struct {
    size_t nx, ny, nz, sz, k0, k1;
    double dx2, dy2, inv_dz2, inv_factor, omega;
} relax_ctx;

static relax_ctx make_relax(size_t nx, size_t ny, size_t nz, double dx, double dy, double dz,
                            double omega) {
    relax_ctx c;
    c.nx = nx; c.ny = ny; c.nz = nz;
    c.sz = (nz > 1) ? nx * ny : 0;
    c.k0 = (nz > 1) ? 1 : 0;
    c.k1 = (nz > 1) ? nz - 1 : 1;
    c.dx2 = dx * dx;
    c.dy2 = dy * dy;
    c.inv_dz2 = (dz > 0.0) ? (1.0 / (dz * dz)) : 0.0;
    double factor = 2.0 * (1.0 / c.dx2 + 1.0 / c.dy2 + c.inv_dz2);
    c.inv_factor = 1.0 / factor;
    c.omega = omega;
    return c;
}

/* linear_solver_redblack.c:80-147: the pass it calls "red" updates cells
 * with (i+j+k) odd; the second pass updates (i+j+k) even. */
static void redblack_sweep(void* vctx, double* x, double* xt, const double* rhs) {
    (void)xt;
    relax_ctx* c = (relax_ctx*)vctx;
    size_t nx = c->nx, ny = c->ny, sz = c->sz;
    for (int pass = 0; pass < 2; pass++) {
        /* one colour's cells read only the other colour: any order within a
         * pass is bitwise the reference's loop */
        PAR
        for (size_t k = c->k0; k < c->k1; k++)
            for (size_t j = 1; j < ny - 1; j++) {
                size_t i0 = ((j + k) % 2 == 0) ? (pass == 0 ? 1 : 2) : (pass == 0 ? 2 : 1);
                for (size_t i = i0; i < nx - 1; i += 2) {
                    size_t idx = k * sz + j * nx + i;
                    double p_new = -(rhs[idx] - (x[idx + 1] + x[idx - 1]) / c->dx2 -
                                     (x[idx + nx] + x[idx - nx]) / c->dy2 -
                                     (x[idx + sz] + x[idx - sz]) * c->inv_dz2) *
                                   c->inv_factor;
                    x[idx] = x[idx] + c->omega * (p_new - x[idx]);
                }
            }
    }
    solver_apply_bc(x, c->nx, c->ny, c->nz);
}

cfd_status_t oracle_redblack_solve(double* x, const double* rhs, size_t nx, size_t ny, size_t nz,
                                   double dx, double dy, double dz,
                                   const poisson_solver_params_t* params,
                                   poisson_solver_stats_t* stats) {
    poisson_solver_params_t prm = params ? *params : oracle_poisson_params_default();
    double omega = (prm.omega <= 0.0) ? optimal_omega(nx, ny, nz, dx, dy, dz) : prm.omega;
    relax_ctx c = make_relax(nx, ny, nz, dx, dy, dz, omega);
    return solve_common(redblack_sweep, &c, x, NULL, rhs, nx, ny, nz, dx, dy, dz, &prm, stats);
}

/* linear_solver_jacobi.c:76-129 */
static void jacobi_sweep(void* vctx, double* x, double* xt, const double* rhs) {
    relax_ctx* c = (relax_ctx*)vctx;
    size_t nx = c->nx, ny = c->ny, sz = c->sz;
    PAR
    for (size_t k = c->k0; k < c->k1; k++)
        for (size_t j = 1; j < ny - 1; j++)
            for (size_t i = 1; i < nx - 1; i++) {
                size_t idx = k * sz + j * nx + i;
                xt[idx] = -(rhs[idx] - (x[idx + 1] + x[idx - 1]) / c->dx2 -
                            (x[idx + nx] + x[idx - nx]) / c->dy2 -
                            (x[idx + sz] + x[idx - sz]) * c->inv_dz2) *
                          c->inv_factor;
            }
    memcpy(x, xt, c->nx * c->ny * c->nz * sizeof(double));
    solver_apply_bc(x, c->nx, c->ny, c->nz);
}

cfd_status_t oracle_jacobi_solve(double* x, double* x_temp, const double* rhs, size_t nx,
                                 size_t ny, size_t nz, double dx, double dy, double dz,
                                 const poisson_solver_params_t* params,
                                 poisson_solver_stats_t* stats) {
    poisson_solver_params_t prm = params ? *params : oracle_poisson_params_default();
    if (!params) prm.max_iterations = 2000; /* linear_solver.c:274-276 */
    relax_ctx c = make_relax(nx, ny, nz, dx, dy, dz, 1.0);
    int own = 0;
    if (!x_temp) {
        x_temp = (double*)malloc(nx * ny * nz * sizeof(double));
        memcpy(x_temp, x, nx * ny * nz * sizeof(double));
        own = 1;
    }
    cfd_status_t s = solve_common(jacobi_sweep, &c, x, x_temp, rhs, nx, ny, nz, dx, dy, dz, &prm,
                                  stats);
    if (own) free(x_temp);
    return s;
}

/* ------------------------------------------------------------------------ */
/* energy equation (energy_solver.c)                                         */
/* ------------------------------------------------------------------------ */
cfd_status_t oracle_energy_step(flow_field* field, const grid* g, const ns_solver_params_t* params,
                                double dt, double time) {
    if (params->alpha <= 0.0) return CFD_SUCCESS;
    size_t nx = field->nx, ny = field->ny, nz = field->nz;
    size_t plane = nx * ny, total = plane * nz;
    double alpha = params->alpha;
    double dx0 = g->dx[0], dy0 = g->dy[0];
    double inv_2dx = 1.0 / (2.0 * dx0);
    double inv_2dy = 1.0 / (2.0 * dy0);
    double inv_dx2 = 1.0 / (dx0 * dx0);
    double inv_dy2 = 1.0 / (dy0 * dy0);
    size_t sz = (nz > 1) ? plane : 0, k0 = (nz > 1) ? 1 : 0, k1 = (nz > 1) ? nz - 1 : 1;
    double inv_2dz = (nz > 1 && g->dz) ? 1.0 / (2.0 * g->dz[0]) : 0.0;
    double inv_dz2 = (nz > 1 && g->dz) ? 1.0 / (g->dz[0] * g->dz[0]) : 0.0;
    double* Tn = (double*)malloc(total * sizeof(double));
    if (!Tn) return CFD_ERROR_NOMEM;
    memcpy(Tn, field->T, total * sizeof(double));
    const double* T = field->T;
    PAR
    for (size_t k = k0; k < k1; k++)
        for (size_t j = 1; j < ny - 1; j++)
            for (size_t i = 1; i < nx - 1; i++) {
                size_t idx = k * sz + j * nx + i;
                double Tc = T[idx];
                double dT_dx = (T[idx + 1] - T[idx - 1]) * inv_2dx;
                double dT_dy = (T[idx + nx] - T[idx - nx]) * inv_2dy;
                double dT_dz = (T[idx + sz] - T[idx - sz]) * inv_2dz;
                double adv = field->u[idx] * dT_dx + field->v[idx] * dT_dy + field->w[idx] * dT_dz;
                double d2x = (T[idx + 1] - 2.0 * Tc + T[idx - 1]) * inv_dx2;
                double d2y = (T[idx + nx] - 2.0 * Tc + T[idx - nx]) * inv_dy2;
                double d2z = (T[idx + sz] - 2.0 * Tc + T[idx - sz]) * inv_dz2;
                double diff = alpha * (d2x + d2y + d2z);
                double Q = 0.0;
                if (params->heat_source_func) {
                    double zc = (nz > 1 && g->z) ? g->z[k] : 0.0;
                    Q = params->heat_source_func(g->x[i], g->y[j], zc, time,
                                                 params->heat_source_context);
                }
                double dT = dt * (-adv + diff + Q);
                Tn[idx] = Tc + dT;
            }
    for (size_t n = 0; n < total; n++) {
        if (!isfinite(Tn[n])) {
            free(Tn);
            return CFD_ERROR_DIVERGED;
        }
    }
    memcpy(field->T, Tn, total * sizeof(double));
    free(Tn);
    return CFD_SUCCESS;
}

static int thermal_ok(bc_type_t t) {
    return t == BC_TYPE_PERIODIC || t == BC_TYPE_NEUMANN || t == BC_TYPE_DIRICHLET;
}

cfd_status_t oracle_apply_thermal_bcs(flow_field* field, const ns_solver_params_t* params) {
    if (params->alpha <= 0.0) return CFD_SUCCESS;
    const ns_thermal_bc_config_t* t = &params->thermal_bc;
    size_t nx = field->nx, ny = field->ny, nz = field->nz, plane = nx * ny;
    double* T = field->T;
    if (!thermal_ok(t->left) || !thermal_ok(t->right) || !thermal_ok(t->bottom) ||
        !thermal_ok(t->top) || (nz > 1 && (!thermal_ok(t->front) || !thermal_ok(t->back))))
        return CFD_ERROR_INVALID;
    for (size_t k = 0; k < nz; k++)
        for (size_t j = 0; j < ny; j++) {
            size_t b = k * plane, idx = b + j * nx;
            if (t->left == BC_TYPE_DIRICHLET) T[idx] = t->dirichlet_values.left;
            else if (t->left == BC_TYPE_NEUMANN) T[idx] = T[idx + 1];
            else T[idx] = T[b + j * nx + (nx - 2)];
        }
    for (size_t k = 0; k < nz; k++)
        for (size_t j = 0; j < ny; j++) {
            size_t b = k * plane, idx = b + j * nx + (nx - 1);
            if (t->right == BC_TYPE_DIRICHLET) T[idx] = t->dirichlet_values.right;
            else if (t->right == BC_TYPE_NEUMANN) T[idx] = T[idx - 1];
            else T[idx] = T[b + j * nx + 1];
        }
    for (size_t k = 0; k < nz; k++)
        for (size_t i = 0; i < nx; i++) {
            size_t b = k * plane, idx = b + i;
            if (t->bottom == BC_TYPE_DIRICHLET) T[idx] = t->dirichlet_values.bottom;
            else if (t->bottom == BC_TYPE_NEUMANN) T[idx] = T[idx + nx];
            else T[idx] = T[b + (ny - 2) * nx + i];
        }
    for (size_t k = 0; k < nz; k++)
        for (size_t i = 0; i < nx; i++) {
            size_t b = k * plane, idx = b + (ny - 1) * nx + i;
            if (t->top == BC_TYPE_DIRICHLET) T[idx] = t->dirichlet_values.top;
            else if (t->top == BC_TYPE_NEUMANN) T[idx] = T[idx - nx];
            else T[idx] = T[b + nx + i];
        }
    if (nz > 1) {
        for (size_t idx = 0; idx < plane; idx++) {
            if (t->back == BC_TYPE_DIRICHLET) T[idx] = t->dirichlet_values.back;
            else if (t->back == BC_TYPE_NEUMANN) T[idx] = T[plane + idx];
            else T[idx] = T[(nz - 2) * plane + idx];
        }
        size_t fb = (nz - 1) * plane;
        for (size_t off = 0; off < plane; off++) {
            if (t->front == BC_TYPE_DIRICHLET) T[fb + off] = t->dirichlet_values.front;
            else if (t->front == BC_TYPE_NEUMANN) T[fb + off] = T[(nz - 2) * plane + off];
            else T[fb + off] = T[plane + off];
        }
    }
    return CFD_SUCCESS;
}

/* ------------------------------------------------------------------------ */
/* stats (solver_registry.c:31-62)                                           */
/* ------------------------------------------------------------------------ */
void oracle_max_velocity_pressure(const flow_field* f, double* max_vel, double* max_p) {
    double mv = 0.0, mp = 0.0;
    size_t n = f->nx * f->ny * f->nz;
    for (size_t i = 0; i < n; i++) {
        double vel = sqrt((f->u[i] * f->u[i]) + (f->v[i] * f->v[i]) + (f->w[i] * f->w[i]));
        if (vel > mv) mv = vel;
        double ap = fabs(f->p[i]);
        if (ap > mp) mp = ap;
    }
    *max_vel = mv;
    *max_p = mp;
}

double oracle_max_temperature(const flow_field* f) {
    size_t n = f->nx * f->ny * f->nz;
    double m = f->T[0];
    for (size_t i = 1; i < n; i++)
        if (f->T[i] > m) m = f->T[i];
    return m;
}

/* ------------------------------------------------------------------------ */
/* projection step (solver_projection.c:46-297, max_iter = 1)                */
/* ------------------------------------------------------------------------ */

/* boundary_copy_utils.h:93-148 */
static void copy_boundary_velocities_3d(double* du, double* dv, double* dw, const double* su,
                                        const double* sv, const double* sw, size_t nx, size_t ny,
                                        size_t nz) {
    size_t plane = nx * ny;
    for (size_t k = 0; k < nz; k++) {
        size_t b = k * plane;
        for (size_t i = 0; i < nx; i++) {
            size_t bot = b + i, top = b + (ny - 1) * nx + i;
            du[bot] = su[bot]; dv[bot] = sv[bot];
            du[top] = su[top]; dv[top] = sv[top];
            if (nz > 1) { dw[bot] = sw[bot]; dw[top] = sw[top]; }
        }
        for (size_t j = 1; j < ny - 1; j++) {
            size_t l = b + j * nx, r = b + j * nx + nx - 1;
            du[l] = su[l]; dv[l] = sv[l];
            du[r] = su[r]; dv[r] = sv[r];
            if (nz > 1) { dw[l] = sw[l]; dw[r] = sw[r]; }
        }
    }
    if (nz > 1) {
        size_t back = (nz - 1) * plane;
        for (size_t j = 1; j < ny - 1; j++)
            for (size_t i = 1; i < nx - 1; i++) {
                size_t off = j * nx + i;
                du[off] = su[off]; dv[off] = sv[off]; dw[off] = sw[off];
                du[back + off] = su[back + off];
                dv[back + off] = sv[back + off];
                dw[back + off] = sw[back + off];
            }
    }
}

static inline double clampv(double x) { return fmax(-MAX_VELOCITY, fmin(MAX_VELOCITY, x)); }

cfd_status_t oracle_projection_step(flow_field* field, const grid* grid,
                                    const ns_solver_params_t* params, ns_solver_stats_t* stats,
                                    oracle_poisson_kind_t pkind, int* poisson_iters) {
    if (!field || !grid || !params) return CFD_ERROR_INVALID;
    if (field->nx < 3 || field->ny < 3 || (field->nz > 1 && field->nz < 3)) return CFD_ERROR_INVALID;
    size_t nx = field->nx, ny = field->ny, nz = field->nz;
    if (nz > 1 && grid->dz) {
        for (size_t k = 1; k < nz - 1; k++)
            if (fabs(grid->dz[k] - grid->dz[0]) > 1e-14) return CFD_ERROR_INVALID;
    }
    size_t plane = nx * ny, total = plane * nz, bytes = total * sizeof(double);
    double dx = grid->dx[0], dy = grid->dy[0];
    double dz = (nz > 1 && grid->dz) ? grid->dz[0] : 0.0;
    double dt = params->dt, nu = params->mu;
    size_t sz = (nz > 1) ? plane : 0, k0 = (nz > 1) ? 1 : 0, k1 = (nz > 1) ? (nz - 1) : 1;
    double inv_2dz = (nz > 1 && grid->dz) ? 1.0 / (2.0 * dz) : 0.0;
    double inv_dz2 = (nz > 1 && grid->dz) ? 1.0 / (dz * dz) : 0.0;
    double* us = (double*)malloc(bytes);
    double* vs = (double*)malloc(bytes);
    double* ws = (double*)malloc(bytes);
    double* pn = (double*)malloc(bytes);
    double* pt = (double*)calloc(total, sizeof(double));
    double* rhs = (double*)calloc(total, sizeof(double));
    cfd_status_t st = CFD_SUCCESS;
    if (!us || !vs || !ws || !pn || !pt || !rhs) { st = CFD_ERROR_NOMEM; goto done; }
    memcpy(us, field->u, bytes);
    memcpy(vs, field->v, bytes);
    memcpy(ws, field->w, bytes);
    memcpy(pn, field->p, bytes);

    double t0 = now_ms();
    const int iter = 0; /* projection_step forces max_iter = 1 (solver_registry.c:928-929) */
    const double* U = field->u;
    const double* V = field->v;
    const double* W = field->w;
    PAR
    for (size_t k = k0; k < k1; k++)
        for (size_t j = 1; j < ny - 1; j++)
            for (size_t i = 1; i < nx - 1; i++) {
                size_t idx = k * sz + j * nx + i;
                double u = U[idx], v = V[idx], w = W[idx];
                double du_dx = (U[idx + 1] - U[idx - 1]) / (2.0 * dx);
                double du_dy = (U[idx + nx] - U[idx - nx]) / (2.0 * dy);
                double du_dz = (U[idx + sz] - U[idx - sz]) * inv_2dz;
                double dv_dx = (V[idx + 1] - V[idx - 1]) / (2.0 * dx);
                double dv_dy = (V[idx + nx] - V[idx - nx]) / (2.0 * dy);
                double dv_dz = (V[idx + sz] - V[idx - sz]) * inv_2dz;
                double dw_dx = (W[idx + 1] - W[idx - 1]) / (2.0 * dx);
                double dw_dy = (W[idx + nx] - W[idx - nx]) / (2.0 * dy);
                double dw_dz = (W[idx + sz] - W[idx - sz]) * inv_2dz;
                double conv_u = u * du_dx + v * du_dy + w * du_dz;
                double conv_v = u * dv_dx + v * dv_dy + w * dv_dz;
                double conv_w = u * dw_dx + v * dw_dy + w * dw_dz;
                double d2u_dx2 = (U[idx + 1] - 2.0 * u + U[idx - 1]) / (dx * dx);
                double d2u_dy2 = (U[idx + nx] - 2.0 * u + U[idx - nx]) / (dy * dy);
                double d2u_dz2 = (U[idx + sz] - 2.0 * u + U[idx - sz]) * inv_dz2;
                double d2v_dx2 = (V[idx + 1] - 2.0 * v + V[idx - 1]) / (dx * dx);
                double d2v_dy2 = (V[idx + nx] - 2.0 * v + V[idx - nx]) / (dy * dy);
                double d2v_dz2 = (V[idx + sz] - 2.0 * v + V[idx - sz]) * inv_dz2;
                double d2w_dx2 = (W[idx + 1] - 2.0 * w + W[idx - 1]) / (dx * dx);
                double d2w_dy2 = (W[idx + nx] - 2.0 * w + W[idx - nx]) / (dy * dy);
                double d2w_dz2 = (W[idx + sz] - 2.0 * w + W[idx - sz]) * inv_dz2;
                double visc_u = nu * (d2u_dx2 + d2u_dy2 + d2u_dz2);
                double visc_v = nu * (d2v_dx2 + d2v_dy2 + d2v_dz2);
                double visc_w = nu * (d2w_dx2 + d2w_dy2 + d2w_dz2);
                /* compute_source_terms (solver_explicit_euler.c:317-333) */
                double su, sv, sw;
                double x = grid->x[i], y = grid->y[j];
                if (params->source_func) {
                    double zc = (nz > 1 && grid->z) ? grid->z[k] : 0.0;
                    params->source_func(x, y, zc, iter * dt, params->source_context, &su, &sv, &sw);
                } else {
                    su = params->source_amplitude_u * sin(M_PI * y) *
                         exp(-params->source_decay_rate * iter * dt);
                    sv = params->source_amplitude_v * sin(2.0 * M_PI * x) *
                         exp(-params->source_decay_rate * iter * dt);
                    sw = 0.0;
                }
                /* energy_compute_buoyancy (energy_solver.c:185-196) */
                if (params->beta != 0.0) {
                    double dT = field->T[idx] - params->T_ref;
                    su += -params->beta * dT * params->gravity[0];
                    sv += -params->beta * dT * params->gravity[1];
                    sw += -params->beta * dT * params->gravity[2];
                }
                us[idx] = u + dt * (-conv_u + visc_u + su);
                vs[idx] = v + dt * (-conv_v + visc_v + sv);
                ws[idx] = w + dt * (-conv_w + visc_w + sw);
                us[idx] = clampv(us[idx]);
                vs[idx] = clampv(vs[idx]);
                ws[idx] = clampv(ws[idx]);
            }
    copy_boundary_velocities_3d(us, vs, ws, field->u, field->v, field->w, nx, ny, nz);
    double t1 = now_ms();

    double rho = field->rho[0];
    if (rho < 1e-10) rho = 1.0;
    PAR
    for (size_t k = k0; k < k1; k++)
        for (size_t j = 1; j < ny - 1; j++)
            for (size_t i = 1; i < nx - 1; i++) {
                size_t idx = k * sz + j * nx + i;
                double dus = (us[idx + 1] - us[idx - 1]) / (2.0 * dx);
                double dvs = (vs[idx + nx] - vs[idx - nx]) / (2.0 * dy);
                double dws = (ws[idx + sz] - ws[idx - sz]) * inv_2dz;
                double div = dus + dvs + dws;
                rhs[idx] = (g_gpu_rhs ? 1.0 / dt : rho / dt) * div;
            }
    double t2 = now_ms();

    poisson_solver_stats_t pst;
    cfd_status_t ps;
    poisson_solver_params_t capped = oracle_poisson_params_default();
    capped.max_iterations = g_poisson_cap;
    const poisson_solver_params_t* pp = g_poisson_cap > 0 ? &capped : (g_have_pparams ? &g_pparams : NULL);
    if (pkind == ORACLE_POISSON_REDBLACK)
        ps = oracle_redblack_solve(pn, rhs, nx, ny, nz, dx, dy, dz, pp, &pst);
    else if (pkind == ORACLE_POISSON_JACOBI)
        ps = oracle_jacobi_solve(pn, pt, rhs, nx, ny, nz, dx, dy, dz, pp, &pst);
    else
        ps = oracle_cg_solve(pn, rhs, nx, ny, nz, dx, dy, dz, pp, &pst);
    if (g_poisson_cap > 0) { ps = CFD_SUCCESS; pst.status = POISSON_CONVERGED; }
    if (poisson_iters) *poisson_iters = pst.iterations;
    g_last_pst = pst;
    double t3 = now_ms();
    /* poisson_solve_3d returns -1 unless converged (linear_solver.c:691-704) */
    if (!(ps == CFD_SUCCESS && pst.status == POISSON_CONVERGED)) { st = CFD_ERROR_MAX_ITER; goto done; }

    double dt_over_rho = dt / rho;
    PAR
    for (size_t k = k0; k < k1; k++)
        for (size_t j = 1; j < ny - 1; j++)
            for (size_t i = 1; i < nx - 1; i++) {
                size_t idx = k * sz + j * nx + i;
                double dp_dx = (pn[idx + 1] - pn[idx - 1]) / (2.0 * dx);
                double dp_dy = (pn[idx + nx] - pn[idx - nx]) / (2.0 * dy);
                double dp_dz = (pn[idx + sz] - pn[idx - sz]) * inv_2dz;
                field->u[idx] = us[idx] - dt_over_rho * dp_dx;
                field->v[idx] = vs[idx] - dt_over_rho * dp_dy;
                field->w[idx] = ws[idx] - dt_over_rho * dp_dz;
                field->u[idx] = clampv(field->u[idx]);
                field->v[idx] = clampv(field->v[idx]);
                field->w[idx] = clampv(field->w[idx]);
            }
    memcpy(field->p, pn, bytes);
    st = oracle_energy_step(field, grid, params, dt, iter * dt);
    if (st != CFD_SUCCESS) goto done;
    st = oracle_apply_thermal_bcs(field, params);
    if (st != CFD_SUCCESS) goto done;
    copy_boundary_velocities_3d(field->u, field->v, field->w, us, vs, ws, nx, ny, nz);
    for (size_t n = 0; n < total; n++) {
        if (!isfinite(field->u[n]) || !isfinite(field->v[n]) || !isfinite(field->w[n]) ||
            !isfinite(field->p[n])) {
            st = CFD_ERROR_DIVERGED;
            goto done;
        }
    }
    double t4 = now_ms();
    g_phase_ms[0] = t1 - t0;
    g_phase_ms[1] = t2 - t1;
    g_phase_ms[2] = t3 - t2;
    g_phase_ms[3] = t4 - t3;
    if (stats) {
        stats->iterations = 1;
        double mv, mp;
        oracle_max_velocity_pressure(field, &mv, &mp);
        stats->max_velocity = mv;
        stats->max_pressure = mp;
        stats->max_temperature = oracle_max_temperature(field);
    }
done:
    free(us); free(vs); free(ws); free(pn); free(pt); free(rhs);
    return st;
}

/* ------------------------------------------------------------------------ */
/* RK4 (solver_rk4.c:69-259) with the shared momentum RHS                    */
/* (ns_momentum_rhs_scalar.h:49-190) and apply_boundary_conditions          */
/* (solver_explicit_euler.c:231-306)                                         */
/* ------------------------------------------------------------------------ */
#define RK_MAX_D1 100.0    /* MAX_DERIVATIVE_LIMIT */
#define RK_MAX_D2 1000.0   /* MAX_SECOND_DERIVATIVE_LIMIT */
#define RK_MAX_DIV 10.0    /* MAX_DIVERGENCE_LIMIT */
#define RK_P_FACTOR 0.1    /* PRESSURE_UPDATE_FACTOR */

static inline double clampd(double x, double lim) { return fmax(-lim, fmin(lim, x)); }

static void rk_rhs(const flow_field* f, const grid* g, const ns_solver_params_t* prm,
                   double* ru, double* rv, double* rw, double* rp, int iter, double dt) {
    size_t nx = f->nx, ny = f->ny, nz = f->nz, plane = nx * ny;
    size_t sz = (nz > 1) ? plane : 0, k0 = (nz > 1) ? 1 : 0, k1 = (nz > 1) ? nz - 1 : 1;
    double inv_2dz = (nz > 1 && g->dz) ? 1.0 / (2.0 * g->dz[0]) : 0.0;
    double inv_dz2 = (nz > 1 && g->dz) ? 1.0 / (g->dz[0] * g->dz[0]) : 0.0;
    const double *u = f->u, *v = f->v, *w = f->w, *p = f->p, *rho = f->rho, *T = f->T;
    PAR
    for (size_t k = k0; k < k1; k++)
        for (size_t j = 1; j < ny - 1; j++)
            for (size_t i = 1; i < nx - 1; i++) {
                size_t idx = k * sz + j * nx + i;
                if (rho[idx] <= 1e-10 || fabs(g->dx[i]) < 1e-10 || fabs(g->dy[j]) < 1e-10) {
                    ru[idx] = rv[idx] = rw[idx] = rp[idx] = 0.0;
                    continue;
                }
                size_t il = (i > 1) ? idx - 1 : k * sz + j * nx + (nx - 2);
                size_t ir = (i < nx - 2) ? idx + 1 : k * sz + j * nx + 1;
                size_t jd = (j > 1) ? idx - nx : k * sz + (ny - 2) * nx + i;
                size_t ju = (j < ny - 2) ? idx + nx : k * sz + 1 * nx + i;
                size_t kd = (k > 1) ? idx - sz : (nz - 2) * sz + j * nx + i;
                size_t ku = (k < nz - 2) ? idx + sz : 1 * sz + j * nx + i;
                double tdx = 2.0 * g->dx[i], tdy = 2.0 * g->dy[j];
                double dxx = g->dx[i] * g->dx[i], dyy = g->dy[j] * g->dy[j];
                double du_dx = (u[ir] - u[il]) / tdx, du_dy = (u[ju] - u[jd]) / tdy;
                double du_dz = (u[ku] - u[kd]) * inv_2dz;
                double dv_dx = (v[ir] - v[il]) / tdx, dv_dy = (v[ju] - v[jd]) / tdy;
                double dv_dz = (v[ku] - v[kd]) * inv_2dz;
                double dw_dx = (w[ir] - w[il]) / tdx, dw_dy = (w[ju] - w[jd]) / tdy;
                double dw_dz = (w[ku] - w[kd]) * inv_2dz;
                double dp_dx = (p[ir] - p[il]) / tdx, dp_dy = (p[ju] - p[jd]) / tdy;
                double dp_dz = (p[ku] - p[kd]) * inv_2dz;
                double d2u_dx2 = (u[ir] - 2.0 * u[idx] + u[il]) / dxx;
                double d2u_dy2 = (u[ju] - 2.0 * u[idx] + u[jd]) / dyy;
                double d2u_dz2 = (u[ku] - 2.0 * u[idx] + u[kd]) * inv_dz2;
                double d2v_dx2 = (v[ir] - 2.0 * v[idx] + v[il]) / dxx;
                double d2v_dy2 = (v[ju] - 2.0 * v[idx] + v[jd]) / dyy;
                double d2v_dz2 = (v[ku] - 2.0 * v[idx] + v[kd]) * inv_dz2;
                double d2w_dx2 = (w[ir] - 2.0 * w[idx] + w[il]) / dxx;
                double d2w_dy2 = (w[ju] - 2.0 * w[idx] + w[jd]) / dyy;
                double d2w_dz2 = (w[ku] - 2.0 * w[idx] + w[kd]) * inv_dz2;
                double nu = prm->mu / fmax(rho[idx], 1e-10);
                nu = fmin(nu, 1.0);
                du_dx = clampd(du_dx, RK_MAX_D1); du_dy = clampd(du_dy, RK_MAX_D1);
                du_dz = clampd(du_dz, RK_MAX_D1); dv_dx = clampd(dv_dx, RK_MAX_D1);
                dv_dy = clampd(dv_dy, RK_MAX_D1); dv_dz = clampd(dv_dz, RK_MAX_D1);
                dw_dx = clampd(dw_dx, RK_MAX_D1); dw_dy = clampd(dw_dy, RK_MAX_D1);
                dw_dz = clampd(dw_dz, RK_MAX_D1); dp_dx = clampd(dp_dx, RK_MAX_D1);
                dp_dy = clampd(dp_dy, RK_MAX_D1); dp_dz = clampd(dp_dz, RK_MAX_D1);
                d2u_dx2 = clampd(d2u_dx2, RK_MAX_D2); d2u_dy2 = clampd(d2u_dy2, RK_MAX_D2);
                d2u_dz2 = clampd(d2u_dz2, RK_MAX_D2); d2v_dx2 = clampd(d2v_dx2, RK_MAX_D2);
                d2v_dy2 = clampd(d2v_dy2, RK_MAX_D2); d2v_dz2 = clampd(d2v_dz2, RK_MAX_D2);
                d2w_dx2 = clampd(d2w_dx2, RK_MAX_D2); d2w_dy2 = clampd(d2w_dy2, RK_MAX_D2);
                d2w_dz2 = clampd(d2w_dz2, RK_MAX_D2);
                /* compute_source_terms (solver_explicit_euler.c:317-333) + buoyancy */
                double su = prm->source_amplitude_u * sin(M_PI * g->y[j]) *
                            exp(-prm->source_decay_rate * iter * dt);
                double sv = prm->source_amplitude_v * sin(2.0 * M_PI * g->x[i]) *
                            exp(-prm->source_decay_rate * iter * dt);
                double sw = 0.0;
                if (T && prm->beta != 0.0) {
                    double dT = T[idx] - prm->T_ref;
                    su += -prm->beta * dT * prm->gravity[0];
                    sv += -prm->beta * dT * prm->gravity[1];
                    sw += -prm->beta * dT * prm->gravity[2];
                }
                ru[idx] = -u[idx] * du_dx - v[idx] * du_dy - w[idx] * du_dz - dp_dx / rho[idx] +
                          nu * (d2u_dx2 + d2u_dy2 + d2u_dz2) + su;
                rv[idx] = -u[idx] * dv_dx - v[idx] * dv_dy - w[idx] * dv_dz - dp_dy / rho[idx] +
                          nu * (d2v_dx2 + d2v_dy2 + d2v_dz2) + sv;
                rw[idx] = -u[idx] * dw_dx - v[idx] * dw_dy - w[idx] * dw_dz - dp_dz / rho[idx] +
                          nu * (d2w_dx2 + d2w_dy2 + d2w_dz2) + sw;
                double div = du_dx + dv_dy + dw_dz;
                div = fmax(-RK_MAX_DIV, fmin(RK_MAX_DIV, div));
                rp[idx] = -RK_P_FACTOR * rho[idx] * div;
            }
}

/* periodic copies of u,v,w,p,rho,T: x faces, y faces, z faces */
static void rk_apply_periodic(flow_field* f) {
    double* a[6] = {f->u, f->v, f->w, f->p, f->rho, f->T};
    for (int q = 0; q < 6; q++)
        if (a[q]) oracle_bc_periodic_3d(a[q], f->nx, f->ny, f->nz);
}

cfd_status_t oracle_rk4_step(flow_field* field, const grid* grid, const ns_solver_params_t* params,
                             ns_solver_stats_t* stats) {
    if (field->nx < 3 || field->ny < 3 || (field->nz > 1 && field->nz < 3)) return CFD_ERROR_INVALID;
    size_t nx = field->nx, ny = field->ny, nz = field->nz;
    if (nz > 1 && grid->dz)
        for (size_t k = 1; k < nz - 1; k++)
            if (fabs(grid->dz[k] - grid->dz[0]) > 1e-14) return CFD_ERROR_INVALID;
    size_t total = nx * ny * nz, bytes = total * sizeof(double);
    double* buf = (double*)calloc(20 * total, sizeof(double));
    if (!buf) return CFD_ERROR_NOMEM;
    double* K[4][4];
    for (int s = 0; s < 4; s++)
        for (int q = 0; q < 4; q++) K[s][q] = buf + (size_t)(s * 4 + q) * total;
    double* Q0[4];
    for (int q = 0; q < 4; q++) Q0[q] = buf + (size_t)(16 + q) * total;
    double* F[4] = {field->u, field->v, field->w, field->p};
    const double dt = params->dt;
    const int iter = 0; /* rk4_step forces max_iter = 1 (solver_registry.c:756-759) */
    for (int q = 0; q < 4; q++) memcpy(Q0[q], F[q], bytes);
    const double fac[3] = {0.5 * dt, 0.5 * dt, dt};
    for (int s = 0; s < 4; s++) {
        rk_rhs(field, grid, params, K[s][0], K[s][1], K[s][2], K[s][3], iter, dt);
        if (s == 3) break;
        /* apply_stage_update (solver_rk4.c:47-63) */
        for (size_t n = 0; n < total; n++) {
            for (int q = 0; q < 4; q++) F[q][n] = Q0[q][n] + fac[s] * K[s][q][n];
            for (int q = 0; q < 3; q++) F[q][n] = clampv(F[q][n]);
        }
    }
    double sixth_dt = dt / 6.0;
    for (size_t n = 0; n < total; n++) {
        for (int q = 0; q < 4; q++)
            F[q][n] = Q0[q][n] + sixth_dt * (K[0][q][n] + 2.0 * K[1][q][n] + 2.0 * K[2][q][n] +
                                             K[3][q][n]);
        for (int q = 0; q < 3; q++) F[q][n] = clampv(F[q][n]);
    }
    free(buf);
    cfd_status_t st = oracle_energy_step(field, grid, params, dt, iter * dt);
    if (st != CFD_SUCCESS) return st;
    rk_apply_periodic(field);
    st = oracle_apply_thermal_bcs(field, params);
    if (st != CFD_SUCCESS) return st;
    for (size_t n = 0; n < total; n++)
        if (!isfinite(field->u[n]) || !isfinite(field->v[n]) || !isfinite(field->w[n]) ||
            !isfinite(field->p[n]))
            return CFD_ERROR_DIVERGED;
    if (stats) {
        stats->iterations = 1;
        oracle_max_velocity_pressure(field, &stats->max_velocity, &stats->max_pressure);
        stats->max_temperature = oracle_max_temperature(field);
    }
    return CFD_SUCCESS;
}

/* ------------------------------------------------------------------------ */
/* Explicit pressure-relaxation step of the reference device API             */
/* gpu_solver_step (lib/src/solvers/gpu/solver_projection_gpu.cu:523-570):   */
/* kernel_velocity_rhs (:158-205) with inv_rho 1, kernel_velocity_update     */
/* (:207-228), Neumann BC on u,v,w, kernel_compute_divergence (:78-95),      */
/* kernel_pressure_update (:257-269), Neumann BC on p. The reference's        */
/* device BC kernel writes all faces in one launch (its edge cells race);     */
/* the restatement uses the sequential face order of                           */
/* boundary_conditions_core_impl.h:41-85, which every race-free order of     */
/* Neumann copies reproduces.                                                 */
/* ------------------------------------------------------------------------ */
cfd_status_t oracle_gpu_explicit_step(flow_field* f, const grid* g,
                                      const ns_solver_params_t* prm) {
    if (!f || !g || !prm) return CFD_ERROR_INVALID;
    const size_t nx = f->nx, ny = f->ny, nz = f->nz, n = nx * ny * nz;
    const size_t sz = (nz > 1) ? nx * ny : 0;
    const size_t k0 = (nz > 1) ? 1 : 0, k1 = (nz > 1) ? nz - 2 : 0; /* inclusive */
    const double dx = g->dx[0], dy = g->dy[0], dt = prm->dt, nu = prm->mu;
    const double inv_2dx = 0.5 / dx, inv_2dy = 0.5 / dy;
    const double inv_dx2 = 1.0 / (dx * dx), inv_dy2 = 1.0 / (dy * dy);
    const double inv_2dz = (nz > 1) ? 0.5 / g->dz[0] : 0.0;
    const double inv_dz2 = (nz > 1) ? 1.0 / (g->dz[0] * g->dz[0]) : 0.0;
    const double inv_rho = 1.0;
    double* ur = (double*)calloc(n, sizeof(double));
    double* vr = (double*)calloc(n, sizeof(double));
    double* wr = (double*)calloc(n, sizeof(double));
    double* dv = (double*)calloc(n, sizeof(double));
    if (!ur || !vr || !wr || !dv) {
        free(ur); free(vr); free(wr); free(dv);
        return CFD_ERROR_NOMEM;
    }
    double *u = f->u, *v = f->v, *w = f->w, *p = f->p;
    for (size_t k = k0; k <= k1; k++)
        for (size_t j = 1; j < ny - 1; j++)
            for (size_t i = 1; i < nx - 1; i++) {
                size_t idx = k * sz + j * nx + i;
                double u_c = u[idx], v_c = v[idx], w_c = w[idx];
                double du_dx = (u[idx + 1] - u[idx - 1]) * inv_2dx;
                double du_dy = (u[idx + nx] - u[idx - nx]) * inv_2dy;
                double du_dz = (u[idx + sz] - u[idx - sz]) * inv_2dz;
                double d2u = (u[idx + 1] - 2.0 * u_c + u[idx - 1]) * inv_dx2 +
                             (u[idx + nx] - 2.0 * u_c + u[idx - nx]) * inv_dy2 +
                             (u[idx + sz] - 2.0 * u_c + u[idx - sz]) * inv_dz2;
                double dv_dx = (v[idx + 1] - v[idx - 1]) * inv_2dx;
                double dv_dy = (v[idx + nx] - v[idx - nx]) * inv_2dy;
                double dv_dz = (v[idx + sz] - v[idx - sz]) * inv_2dz;
                double d2v = (v[idx + 1] - 2.0 * v_c + v[idx - 1]) * inv_dx2 +
                             (v[idx + nx] - 2.0 * v_c + v[idx - nx]) * inv_dy2 +
                             (v[idx + sz] - 2.0 * v_c + v[idx - sz]) * inv_dz2;
                double dw_dx = (w[idx + 1] - w[idx - 1]) * inv_2dx;
                double dw_dy = (w[idx + nx] - w[idx - nx]) * inv_2dy;
                double dw_dz = (w[idx + sz] - w[idx - sz]) * inv_2dz;
                double d2w = (w[idx + 1] - 2.0 * w_c + w[idx - 1]) * inv_dx2 +
                             (w[idx + nx] - 2.0 * w_c + w[idx - nx]) * inv_dy2 +
                             (w[idx + sz] - 2.0 * w_c + w[idx - sz]) * inv_dz2;
                double dp_dx = (p[idx + 1] - p[idx - 1]) * inv_2dx;
                double dp_dy = (p[idx + nx] - p[idx - nx]) * inv_2dy;
                double dp_dz = (p[idx + sz] - p[idx - sz]) * inv_2dz;
                ur[idx] = -(u_c * du_dx + v_c * du_dy + w_c * du_dz) + nu * d2u - inv_rho * dp_dx;
                vr[idx] = -(u_c * dv_dx + v_c * dv_dy + w_c * dv_dz) + nu * d2v - inv_rho * dp_dy;
                wr[idx] = -(u_c * dw_dx + v_c * dw_dy + w_c * dw_dz) + nu * d2w - inv_rho * dp_dz;
            }
    for (size_t k = k0; k <= k1; k++)
        for (size_t j = 1; j < ny - 1; j++)
            for (size_t i = 1; i < nx - 1; i++) {
                size_t idx = k * sz + j * nx + i;
                u[idx] = clampv(u[idx] + dt * ur[idx]);
                v[idx] = clampv(v[idx] + dt * vr[idx]);
                w[idx] = clampv(w[idx] + dt * wr[idx]);
            }
    oracle_bc_neumann_3d(u, nx, ny, nz);
    oracle_bc_neumann_3d(v, nx, ny, nz);
    oracle_bc_neumann_3d(w, nx, ny, nz);
    for (size_t k = k0; k <= k1; k++)
        for (size_t j = 1; j < ny - 1; j++)
            for (size_t i = 1; i < nx - 1; i++) {
                size_t idx = k * sz + j * nx + i;
                dv[idx] = (u[idx + 1] - u[idx - 1]) * inv_2dx + (v[idx + nx] - v[idx - nx]) * inv_2dy +
                          (w[idx + sz] - w[idx - sz]) * inv_2dz;
            }
    const double ndim = (nz > 1) ? 3.0 : 2.0;
    const double p_relax = 0.1 * dt * (inv_dx2 + inv_dy2 + inv_dz2) / ndim;
    for (size_t k = k0; k <= k1; k++)
        for (size_t j = 1; j < ny - 1; j++)
            for (size_t i = 1; i < nx - 1; i++) {
                size_t idx = k * sz + j * nx + i;
                p[idx] -= p_relax * dv[idx];
            }
    oracle_bc_neumann_3d(p, nx, ny, nz);
    free(ur); free(vr); free(wr); free(dv);
    return CFD_SUCCESS;
}
