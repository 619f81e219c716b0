/*
 * cfd_host.c -- libcfd_host.so: standalone host-side mirror of the reference
 * API around the projection path (see include/cfd_hip/cfd_host.h).
 *
 * This library holds no numerics of the hot path: the only solvers it can
 * create are the ones libcfd_hip.so registers (projection_hip*). Boundary
 * conditions and field initialisation are the host-side helpers reference
 * drivers call between steps.
 */
#define _GNU_SOURCE
#include "cfd_hip/cfd_host.h"
#include "vtk_format.h"

#include <dlfcn.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* ------------------------------------------------------------------------ */
/* thread-local error state (logging.c:13-90)                                */
/* ------------------------------------------------------------------------ */
static __thread cfd_status_t g_last_status = CFD_SUCCESS;
static __thread char g_last_msg[256];

void cfd_set_error(cfd_status_t status, const char* message) {
    g_last_status = status;
    if (message) snprintf(g_last_msg, sizeof(g_last_msg), "%s", message);
    else g_last_msg[0] = '\0';
}

const char* cfd_get_last_error(void) { return g_last_msg[0] ? g_last_msg : NULL; }
cfd_status_t cfd_get_last_status(void) { return g_last_status; }

const char* cfd_get_error_string(cfd_status_t s) {
    switch (s) {
        case CFD_SUCCESS: return "Success";
        case CFD_ERROR: return "Generic error";
        case CFD_ERROR_NOMEM: return "Out of memory";
        case CFD_ERROR_INVALID: return "Invalid argument";
        case CFD_ERROR_IO: return "I/O error";
        case CFD_ERROR_UNSUPPORTED: return "Operation not supported";
        case CFD_ERROR_DIVERGED: return "NSSolver diverged";
        case CFD_ERROR_MAX_ITER: return "Max iterations reached";
        case CFD_ERROR_LIMIT_EXCEEDED: return "Resource limit exceeded";
        case CFD_ERROR_NOT_FOUND: return "Resource not found";
        default: return "Unknown error";
    }
}

void cfd_clear_error(void) {
    g_last_status = CFD_SUCCESS;
    g_last_msg[0] = '\0';
}

/* ------------------------------------------------------------------------ */
/* grid (grid.c:9-127)                                                        */
/* ------------------------------------------------------------------------ */
grid* grid_create(size_t nx, size_t ny, size_t nz, double xmin, double xmax, double ymin,
                  double ymax, double zmin, double zmax) {
    if (nx == 0 || ny == 0 || nz == 0) {
        cfd_set_error(CFD_ERROR_INVALID, "grid dimensions must be positive");
        return NULL;
    }
    if (xmax <= xmin || ymax <= ymin) {
        cfd_set_error(CFD_ERROR_INVALID, "grid bounds invalid (max must be > min)");
        return NULL;
    }
    if (nz > 1 && zmax <= zmin) {
        cfd_set_error(CFD_ERROR_INVALID, "grid z-bounds invalid (zmax must be > zmin when nz > 1)");
        return NULL;
    }
    grid* g = (grid*)calloc(1, sizeof(grid));
    if (!g) return NULL;
    g->nx = nx; g->ny = ny; g->nz = nz;
    g->xmin = xmin; g->xmax = xmax; g->ymin = ymin; g->ymax = ymax;
    g->x = (double*)calloc(nx, sizeof(double));
    g->y = (double*)calloc(ny, sizeof(double));
    g->dx = (double*)calloc(nx > 1 ? nx - 1 : 1, sizeof(double));
    g->dy = (double*)calloc(ny > 1 ? ny - 1 : 1, sizeof(double));
    if (!g->x || !g->y || !g->dx || !g->dy) {
        grid_destroy(g);
        return NULL;
    }
    if (nz > 1) {
        g->zmin = zmin; g->zmax = zmax;
        g->z = (double*)calloc(nz, sizeof(double));
        g->dz = (double*)calloc(nz - 1, sizeof(double));
        if (!g->z || !g->dz) {
            grid_destroy(g);
            return NULL;
        }
        g->stride_z = nx * ny;
        g->inv_dz2 = 0.0;
        g->k_start = 1;
        g->k_end = nz - 1;
    } else {
        g->k_start = 0;
        g->k_end = 1;
    }
    return g;
}

void grid_destroy(grid* g) {
    if (!g) return;
    free(g->x); free(g->y); free(g->dx); free(g->dy); free(g->z); free(g->dz);
    free(g);
}

void grid_initialize_uniform(grid* g) {
    double dx = (g->xmax - g->xmin) / (g->nx - 1);
    double dy = (g->ymax - g->ymin) / (g->ny - 1);
    for (size_t i = 0; i < g->nx; i++) g->x[i] = g->xmin + (i * dx);
    for (size_t j = 0; j < g->ny; j++) g->y[j] = g->ymin + (j * dy);
    for (size_t i = 0; i + 1 < g->nx; i++) g->dx[i] = dx;
    for (size_t j = 0; j + 1 < g->ny; j++) g->dy[j] = dy;
    if (g->nz > 1 && g->z && g->dz) {
        double dz = (g->zmax - g->zmin) / (g->nz - 1);
        for (size_t k = 0; k < g->nz; k++) g->z[k] = g->zmin + (k * dz);
        for (size_t k = 0; k + 1 < g->nz; k++) g->dz[k] = dz;
        g->inv_dz2 = 1.0 / (dz * dz);
    }
}

/* ------------------------------------------------------------------------ */
/* flow field (solver_explicit_euler.c:58-160)                               */
/* ------------------------------------------------------------------------ */
static double* aligned_zeros(size_t n) {
    void* p = NULL;
    size_t bytes = n * sizeof(double);
    if (bytes == 0) bytes = sizeof(double);
    if (posix_memalign(&p, 64, bytes) != 0) return NULL;
    memset(p, 0, bytes);
    return (double*)p;
}

flow_field* flow_field_create(size_t nx, size_t ny, size_t nz) {
    if (nx == 0 || ny == 0 || nz == 0) {
        cfd_set_error(CFD_ERROR_INVALID, "Flow field dimensions must be positive");
        return NULL;
    }
    flow_field* f = (flow_field*)calloc(1, sizeof(flow_field));
    if (!f) return NULL;
    f->nx = nx; f->ny = ny; f->nz = nz;
    size_t n = nx * ny * nz;
    f->u = aligned_zeros(n);
    f->v = aligned_zeros(n);
    f->w = aligned_zeros(n);
    f->p = aligned_zeros(n);
    f->rho = aligned_zeros(n);
    f->T = aligned_zeros(n);
    if (!f->u || !f->v || !f->w || !f->p || !f->rho || !f->T) {
        flow_field_destroy(f);
        return NULL;
    }
    return f;
}

void flow_field_destroy(flow_field* f) {
    if (!f) return;
    free(f->u); free(f->v); free(f->w); free(f->p); free(f->rho); free(f->T);
    free(f);
}

void initialize_flow_field(flow_field* f, const grid* g) {
    size_t nx = f->nx, ny = f->ny, nz = f->nz, plane = nx * ny;
    for (size_t k = 0; k < nz; k++)
        for (size_t j = 0; j < ny; j++)
            for (size_t i = 0; i < nx; i++) {
                size_t idx = k * plane + j * nx + i;
                double x = g->x[i], y = g->y[j];
                f->u[idx] = 1.0 + (0.1 * sin(M_PI * y));
                f->v[idx] = 0.05 * sin(2.0 * M_PI * x);
                f->w[idx] = 0.0;
                f->p[idx] = 1.0;
                f->rho[idx] = 1.0;
                f->T[idx] = 300.0;
                double cx = 1.0, cy = 0.5;
                double r = sqrt(((x - cx) * (x - cx)) + ((y - cy) * (y - cy)));
                if (r < 0.2) {
                    f->p[idx] += 0.1 * exp(-r * r / 0.02);
                    double dp_dx = -0.1 * 2.0 * (x - cx) / 0.02 * exp(-r * r / 0.02);
                    double dp_dy = -0.1 * 2.0 * (y - cy) / 0.02 * exp(-r * r / 0.02);
                    f->u[idx] += -0.1 * dp_dx;
                    f->v[idx] += -0.1 * dp_dy;
                }
            }
}

ns_solver_params_t ns_solver_params_default(void) {
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

ns_solver_stats_t ns_solver_stats_default(void) {
    ns_solver_stats_t s;
    memset(&s, 0, sizeof(s));
    s.status = CFD_SUCCESS;
    return s;
}

/* ------------------------------------------------------------------------ */
/* boundary conditions (boundary_conditions_core_impl.h:41-186)              */
/* ------------------------------------------------------------------------ */
static void bc_neumann(double* f, size_t nx, size_t ny, size_t nz, size_t sz) {
    for (size_t k = 0; k < nz; k++)
        for (size_t j = 0; j < ny; j++) {
            f[k * sz + j * nx] = f[k * sz + j * nx + 1];
            f[k * sz + j * nx + nx - 1] = f[k * sz + j * nx + nx - 2];
        }
    for (size_t k = 0; k < nz; k++)
        for (size_t i = 0; i < nx; i++) {
            f[k * sz + i] = f[k * sz + nx + i];
            f[k * sz + (ny - 1) * nx + i] = f[k * sz + (ny - 2) * nx + i];
        }
    if (nz > 1)
        for (size_t i = 0; i < nx * ny; i++) {
            f[i] = f[sz + i];
            f[(nz - 1) * sz + i] = f[(nz - 2) * sz + i];
        }
}

static void bc_periodic(double* f, size_t nx, size_t ny, size_t nz, size_t sz) {
    for (size_t k = 0; k < nz; k++)
        for (size_t j = 0; j < ny; j++) {
            f[k * sz + j * nx] = f[k * sz + j * nx + nx - 2];
            f[k * sz + j * nx + nx - 1] = f[k * sz + j * nx + 1];
        }
    for (size_t k = 0; k < nz; k++)
        for (size_t i = 0; i < nx; i++) {
            f[k * sz + i] = f[k * sz + (ny - 2) * nx + i];
            f[k * sz + (ny - 1) * nx + i] = f[k * sz + nx + i];
        }
    if (nz > 1)
        for (size_t i = 0; i < nx * ny; i++) {
            f[i] = f[(nz - 2) * sz + i];
            f[(nz - 1) * sz + i] = f[sz + i];
        }
}

static void bc_dirichlet(double* f, size_t nx, size_t ny, size_t nz, size_t sz,
                         const bc_dirichlet_values_t* v) {
    for (size_t k = 0; k < nz; k++)
        for (size_t j = 0; j < ny; j++) {
            f[k * sz + j * nx] = v->left;
            f[k * sz + j * nx + nx - 1] = v->right;
        }
    for (size_t k = 0; k < nz; k++)
        for (size_t i = 0; i < nx; i++) {
            f[k * sz + i] = v->bottom;
            f[k * sz + (ny - 1) * nx + i] = v->top;
        }
    if (nz > 1)
        for (size_t i = 0; i < nx * ny; i++) {
            f[i] = v->back;
            f[(nz - 1) * sz + i] = v->front;
        }
}

cfd_status_t bc_apply_scalar_3d(double* f, size_t nx, size_t ny, size_t nz, size_t sz,
                                bc_type_t type) {
    if (!f || nx < 3 || ny < 3) return CFD_ERROR_INVALID;
    if (nz > 1 && sz == 0) sz = nx * ny;
    if (type == BC_TYPE_NEUMANN) bc_neumann(f, nx, ny, nz, sz);
    else if (type == BC_TYPE_PERIODIC) bc_periodic(f, nx, ny, nz, sz);
    else {
        cfd_set_error(CFD_ERROR_UNSUPPORTED, "bc_apply_scalar_3d: only NEUMANN/PERIODIC in this mirror");
        return CFD_ERROR_UNSUPPORTED;
    }
    return CFD_SUCCESS;
}

cfd_status_t bc_apply_velocity_3d(double* u, double* v, double* w, size_t nx, size_t ny, size_t nz,
                                  size_t sz, bc_type_t type) {
    if (!u || !v || nx < 3 || ny < 3) return CFD_ERROR_INVALID;
    cfd_status_t s = bc_apply_scalar_3d(u, nx, ny, nz, sz, type);
    if (s != CFD_SUCCESS) return s;
    s = bc_apply_scalar_3d(v, nx, ny, nz, sz, type);
    if (s != CFD_SUCCESS) return s;
    if (w && nz > 1) s = bc_apply_scalar_3d(w, nx, ny, nz, sz, type);
    return s;
}

cfd_status_t bc_apply_dirichlet_scalar_3d(double* f, size_t nx, size_t ny, size_t nz, size_t sz,
                                          const bc_dirichlet_values_t* values) {
    if (!f || !values || nx < 3 || ny < 3) return CFD_ERROR_INVALID;
    if (nz > 1 && sz == 0) sz = nx * ny;
    bc_dirichlet(f, nx, ny, nz, sz, values);
    return CFD_SUCCESS;
}

cfd_status_t bc_apply_dirichlet_velocity_3d(double* u, double* v, double* w, size_t nx, size_t ny,
                                            size_t nz, size_t sz,
                                            const bc_dirichlet_values_t* uv,
                                            const bc_dirichlet_values_t* vv,
                                            const bc_dirichlet_values_t* wv) {
    if (!u || !v || !uv || !vv || nx < 3 || ny < 3) return CFD_ERROR_INVALID;
    bc_apply_dirichlet_scalar_3d(u, nx, ny, nz, sz, uv);
    bc_apply_dirichlet_scalar_3d(v, nx, ny, nz, sz, vv);
    if (w && wv && nz > 1) bc_apply_dirichlet_scalar_3d(w, nx, ny, nz, sz, wv);
    return CFD_SUCCESS;
}

/* ------------------------------------------------------------------------ */
/* registry (solver_registry.c:133-494)                                      */
/* ------------------------------------------------------------------------ */
#define MAX_REGISTERED_SOLVERS 32

typedef struct {
    char name[64];
    ns_solver_factory_func factory;
    ns_solver_backend_t backend;
} registry_entry;

struct NSSolverRegistry {
    registry_entry entries[MAX_REGISTERED_SOLVERS];
    int count;
};

static double now_ms(void) {
    struct timeval tv;
    gettimeofday(&tv, NULL);
    return tv.tv_sec * 1000.0 + tv.tv_usec / 1000.0;
}

ns_solver_registry_t* cfd_registry_create(void) {
    return (ns_solver_registry_t*)calloc(1, sizeof(ns_solver_registry_t));
}

void cfd_registry_destroy(ns_solver_registry_t* r) { free(r); }

/* Name suffix -> backend, as the UNPATCHED reference infers it
 * (infer_backend_from_type, solver_registry.c:257-279): only `_gpu` is a GPU
 * name, so `projection_hip` is stored as SCALAR. The one-line patch
 * INTEGRATION.md §1 asks a maintainer to add (a `_hip` clause at :262-265) is
 * switched on with cfd_host_set_hip_patch(1). */
static int g_hip_patch = 0;

void cfd_host_set_hip_patch(int enable) { g_hip_patch = enable ? 1 : 0; }

static ns_solver_backend_t infer_backend(const char* name) {
    if (!name) return NS_SOLVER_BACKEND_SCALAR;
    if (strstr(name, "_gpu")) return NS_SOLVER_BACKEND_CUDA;
    if (g_hip_patch && strstr(name, "_hip")) return NS_SOLVER_BACKEND_CUDA;
    if (strstr(name, "_omp")) return NS_SOLVER_BACKEND_OMP;
    if (strstr(name, "_optimized")) return NS_SOLVER_BACKEND_SIMD;
    return NS_SOLVER_BACKEND_SCALAR;
}

void cfd_registry_register_defaults(ns_solver_registry_t* r) {
    if (!r) return;
    /* plugin lookup: the HIP library registers its solvers when present */
    void (*reg)(ns_solver_registry_t*) =
        (void (*)(ns_solver_registry_t*))dlsym(RTLD_DEFAULT, "cfd_hip_register_solvers");
    if (reg) reg(r);
}

int cfd_registry_register(ns_solver_registry_t* r, const char* name,
                          ns_solver_factory_func factory) {
    if (!r || !name || !factory) {
        cfd_set_error(CFD_ERROR_INVALID, "Invalid arguments for solver registration");
        return -1;
    }
    if (strlen(name) == 0) {
        cfd_set_error(CFD_ERROR_INVALID, "solver type name cannot be empty");
        return -1;
    }
    if (r->count >= MAX_REGISTERED_SOLVERS) {
        cfd_set_error(CFD_ERROR_LIMIT_EXCEEDED, "Max registered solvers limit reached");
        return -1;
    }
    ns_solver_backend_t b = infer_backend(name);
    for (int i = 0; i < r->count; i++)
        if (strcmp(r->entries[i].name, name) == 0) {
            r->entries[i].factory = factory;
            r->entries[i].backend = b;
            return 0;
        }
    snprintf(r->entries[r->count].name, sizeof(r->entries[r->count].name), "%s", name);
    r->entries[r->count].factory = factory;
    r->entries[r->count].backend = b;
    r->count++;
    return 0;
}

int cfd_registry_unregister(ns_solver_registry_t* r, const char* name) {
    if (!r || !name) return -1;
    for (int i = 0; i < r->count; i++)
        if (strcmp(r->entries[i].name, name) == 0) {
            for (int j = i; j < r->count - 1; j++) r->entries[j] = r->entries[j + 1];
            r->count--;
            return 0;
        }
    return -1;
}

int cfd_registry_list(ns_solver_registry_t* r, const char** names, int max_count) {
    if (!r) return 0;
    int n = r->count < max_count ? r->count : max_count;
    if (names)
        for (int i = 0; i < n; i++) names[i] = r->entries[i].name;
    return r->count;
}

int cfd_registry_has(ns_solver_registry_t* r, const char* name) {
    if (!r || !name) return 0;
    for (int i = 0; i < r->count; i++)
        if (strcmp(r->entries[i].name, name) == 0) return 1;
    return 0;
}

const char* cfd_registry_get_description(ns_solver_registry_t* r, const char* name) {
    ns_solver_t* s = cfd_solver_create(r, name);
    if (!s) return NULL;
    const char* d = s->description;
    solver_destroy(s);
    return d;
}

ns_solver_t* cfd_solver_create(ns_solver_registry_t* r, const char* name) {
    if (!r || !name) {
        cfd_set_error(CFD_ERROR_INVALID, "Invalid arguments for solver creation");
        return NULL;
    }
    for (int i = 0; i < r->count; i++)
        if (strcmp(r->entries[i].name, name) == 0) {
            ns_solver_t* s = r->entries[i].factory();
            if (!s && cfd_get_last_status() == CFD_SUCCESS)
                cfd_set_error(CFD_ERROR_NOMEM, "Failed to allocate solver");
            return s;
        }
    char msg[128];
    snprintf(msg, sizeof(msg), "Solver type '%s' not registered", name);
    cfd_set_error(CFD_ERROR_NOT_FOUND, msg);
    return NULL;
}

void solver_destroy(ns_solver_t* s) {
    if (!s) return;
    if (s->destroy) s->destroy(s);
    free(s);
}

cfd_status_t solver_init(ns_solver_t* s, const grid* g, const ns_solver_params_t* p) {
    if (!s) return CFD_ERROR_INVALID;
    if (!s->init) return CFD_SUCCESS;
    return s->init(s, g, p);
}

cfd_status_t solver_step(ns_solver_t* s, flow_field* f, const grid* g,
                         const ns_solver_params_t* p, ns_solver_stats_t* st) {
    if (!s || !f || !g || !p) return CFD_ERROR_INVALID;
    if (!s->step) return CFD_ERROR;
    double t0 = now_ms();
    cfd_status_t status = s->step(s, f, g, p, st);
    double t1 = now_ms();
    if (st) {
        st->elapsed_time_ms = t1 - t0;
        st->status = status;
    }
    return status;
}

cfd_status_t solver_solve(ns_solver_t* s, flow_field* f, const grid* g,
                          const ns_solver_params_t* p, ns_solver_stats_t* st) {
    if (!s || !f || !g || !p) return CFD_ERROR_INVALID;
    if (!s->solve) return CFD_ERROR;
    double t0 = now_ms();
    cfd_status_t status = s->solve(s, f, g, p, st);
    double t1 = now_ms();
    if (st) {
        st->elapsed_time_ms = t1 - t0;
        st->status = status;
    }
    return status;
}

/* solver_registry.c:1600-1621: the GPU backend asks gpu_is_available(), which
 * libcfd_hip.so exports (gpu_device_hip.hip); this mirror has no SIMD / OpenMP
 * solvers of its own. */
int cfd_backend_is_available(ns_solver_backend_t b) {
    if (b == NS_SOLVER_BACKEND_SCALAR) return 1;
    if (b == NS_SOLVER_BACKEND_CUDA) {
        int (*avail)(void) = (int (*)(void))dlsym(RTLD_DEFAULT, "gpu_is_available");
        return avail ? avail() : 0;
    }
    return 0;
}

const char* cfd_backend_get_name(ns_solver_backend_t b) {  /* :1623-1636 */
    switch (b) {
        case NS_SOLVER_BACKEND_SCALAR: return "scalar";
        case NS_SOLVER_BACKEND_SIMD: return "simd";
        case NS_SOLVER_BACKEND_OMP: return "openmp";
        case NS_SOLVER_BACKEND_CUDA: return "cuda";
        default: return "unknown";
    }
}

/* :1638-1667, on the backend stored at registration */
int cfd_registry_list_by_backend(ns_solver_registry_t* r, ns_solver_backend_t backend,
                                 const char** names, int max_count) {
    if (!r) return 0;
    int count = 0;
    for (int i = 0; i < r->count; i++) {
        if (r->entries[i].backend != backend) continue;
        if (!names) {
            count++;
        } else if (count < max_count) {
            names[count++] = r->entries[i].name;
        } else {
            break;
        }
    }
    return count;
}

/* :1669-1694: the backend the NAME implies must be available first */
ns_solver_t* cfd_solver_create_checked(ns_solver_registry_t* r, const char* name) {
    if (!r || !name) {
        cfd_set_error(CFD_ERROR_INVALID, "Invalid arguments for solver creation");
        return NULL;
    }
    ns_solver_backend_t b = infer_backend(name);
    if (!cfd_backend_is_available(b)) {
        char msg[128];
        snprintf(msg, sizeof(msg), "Backend '%s' is not available on this system",
                 cfd_backend_get_name(b));
        cfd_set_error(CFD_ERROR_UNSUPPORTED, msg);
        return NULL;
    }
    return cfd_solver_create(r, name);
}

/* simulation_api.c:452-478: a STATIC name table, not the registry. The
 * reference's own names (CFD_ENABLE_OPENMP build); the HIP names appear only
 * with the INTEGRATION.md §1 patch, mirrored by the same switch. */
static const char* const s_solver_names[] = {
    "explicit_euler", "explicit_euler_optimized", "projection", "projection_optimized",
    "explicit_euler_gpu", "projection_gpu", "explicit_euler_omp", "projection_omp",
    "projection_hip", "projection_hip_rbsor", "projection_hip_jacobi", "rk4_hip",
    "projection_hip_cg1",
};

int simulation_list_solvers(const char** names, int max_count) {
    const int total = (int)(sizeof(s_solver_names) / sizeof(s_solver_names[0]));
    const int n = g_hip_patch ? total : total - 5;
    if (names && max_count > 0) {
        int fill = n < max_count ? n : max_count;
        for (int i = 0; i < fill; i++) names[i] = s_solver_names[i];
    }
    return n;
}

/* ------------------------------------------------------------------------ */
/* simulation API subset (simulation_api.c:24-251)                           */
/* ------------------------------------------------------------------------ */
simulation_data* init_simulation_with_solver(size_t nx, size_t ny, size_t nz, double xmin,
                                             double xmax, double ymin, double ymax, double zmin,
                                             double zmax, const char* solver_type) {
    if (!solver_type) {
        cfd_set_error(CFD_ERROR_INVALID, "solver type must not be NULL");
        return NULL;
    }
    if (nx == 0 || ny == 0 || nz == 0) {
        cfd_set_error(CFD_ERROR_INVALID, "Simulation grid dimensions must be positive");
        return NULL;
    }
    if (xmax <= xmin || ymax <= ymin || (nz > 1 && zmax <= zmin)) {
        cfd_set_error(CFD_ERROR_INVALID, "Simulation bounds invalid");
        return NULL;
    }
    simulation_data* s = (simulation_data*)calloc(1, sizeof(simulation_data));
    if (!s) return NULL;
    snprintf(s->output_base_dir, sizeof(s->output_base_dir), "../../artifacts");
    s->grid = grid_create(nx, ny, nz, xmin, xmax, ymin, ymax, zmin, zmax);
    if (!s->grid) goto fail;
    grid_initialize_uniform(s->grid);
    s->field = flow_field_create(nx, ny, nz);
    if (!s->field) goto fail;
    initialize_flow_field(s->field, s->grid);
    s->params = ns_solver_params_default();
    s->params.dt = 0.001;
    s->params.cfl = 0.2;
    s->params.mu = 0.01;
    s->params.max_iter = 1;
    s->last_stats = ns_solver_stats_default();
    s->registry = cfd_registry_create();
    if (!s->registry) goto fail;
    cfd_registry_register_defaults(s->registry);
    s->solver = cfd_solver_create(s->registry, solver_type);
    if (!s->solver) goto fail;
    solver_init(s->solver, s->grid, &s->params); /* return ignored, simulation_api.c:115 */
    return s;
fail:
    if (s->registry) cfd_registry_destroy(s->registry);
    flow_field_destroy(s->field);
    grid_destroy(s->grid);
    free(s);
    return NULL;
}

void free_simulation(simulation_data* s) {
    if (!s) return;
    if (s->solver) solver_destroy(s->solver);
    if (s->registry) cfd_registry_destroy(s->registry);
    free(s->run_prefix);
    flow_field_destroy(s->field);
    grid_destroy(s->grid);
    free(s);
}

cfd_status_t run_simulation_step(simulation_data* s) {
    if (!s || !s->solver) return CFD_ERROR_INVALID;
    s->params.dt = 0.005; /* fixed dt (simulation_api.c:191) */
    cfd_status_t st = solver_step(s->solver, s->field, s->grid, &s->params, &s->last_stats);
    if (st != CFD_SUCCESS) return st;
    s->current_time += s->params.dt;
    return CFD_SUCCESS;
}

cfd_status_t run_simulation_solve(simulation_data* s) {
    if (!s || !s->solver) return CFD_ERROR_INVALID;
    s->params.dt = 0.005;
    cfd_status_t st = solver_solve(s->solver, s->field, s->grid, &s->params, &s->last_stats);
    s->current_time += s->params.dt * s->last_stats.iterations;
    return st;
}

const ns_solver_stats_t* simulation_get_stats(const simulation_data* s) {
    return s ? &s->last_stats : NULL;
}

/* ------------------------------------------------------------------------ */
/* Poisson solver interface (linear_solver.c:25-535), GPU backend only       */
/* ------------------------------------------------------------------------ */
poisson_solver_params_t poisson_solver_params_default(void) {
    /* linear_solver.c:37-47 */
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

poisson_solver_stats_t poisson_solver_stats_default(void) {
    /* linear_solver.c:49-57 */
    poisson_solver_stats_t s;
    memset(&s, 0, sizeof(s));
    s.status = POISSON_ERROR;
    return s;
}

static int hip_device_visible(void) {
    int (*avail)(void) = (int (*)(void))dlsym(RTLD_DEFAULT, "hip_projection_available");
    return avail ? avail() : 0;
}

bool poisson_solver_backend_available(poisson_solver_backend_t backend) {
    /* linear_solver.c:105-131, for a library whose only solvers are the HIP ones */
    if (backend == POISSON_BACKEND_GPU || backend == POISSON_BACKEND_AUTO)
        return hip_device_visible() != 0;
    return false;
}

poisson_solver_t* poisson_solver_create(poisson_solver_method_t method,
                                        poisson_solver_backend_t backend) {
    /* linear_solver.c:150-235: no silent fallbacks; NULL when the pair is absent */
    if (backend == POISSON_BACKEND_AUTO) backend = POISSON_BACKEND_GPU;
    if (backend != POISSON_BACKEND_GPU) return NULL;
    const char* factory = NULL;
    switch (method) {
        case POISSON_METHOD_JACOBI: factory = "create_jacobi_gpu_solver"; break;
        case POISSON_METHOD_REDBLACK_SOR: factory = "create_redblack_gpu_solver"; break;
        case POISSON_METHOD_CG: factory = "create_cg_gpu_solver"; break;
        default: return NULL; /* SOR / Gauss-Seidel / BiCGSTAB / multigrid: no GPU form */
    }
    poisson_solver_t* (*fn)(void) = (poisson_solver_t * (*)(void)) dlsym(RTLD_DEFAULT, factory);
    if (!fn) {
        cfd_set_error(CFD_ERROR_UNSUPPORTED, "libcfd_hip.so (GPU Poisson backend) is not loaded");
        return NULL;
    }
    return fn();
}

cfd_status_t poisson_solver_init(poisson_solver_t* solver, size_t nx, size_t ny, size_t nz,
                                 double dx, double dy, double dz,
                                 const poisson_solver_params_t* params) {
    /* linear_solver.c:237-282 */
    if (!solver) return CFD_ERROR_INVALID;
    if (nx < 3 || ny < 3 || (nz > 1 && nz < 3)) return CFD_ERROR_INVALID;
    solver->nx = nx;
    solver->ny = ny;
    solver->nz = nz;
    solver->dx = dx;
    solver->dy = dy;
    solver->dz = dz;
    solver->params = params ? *params : poisson_solver_params_default();
    if (solver->method == POISSON_METHOD_JACOBI && params == NULL)
        solver->params.max_iterations = 2000;
    if (solver->init) return solver->init(solver, nx, ny, nz, dx, dy, dz, &solver->params);
    return CFD_SUCCESS;
}

void poisson_solver_destroy(poisson_solver_t* solver) {
    /* linear_solver.c:284-294 */
    if (!solver) return;
    if (solver->destroy) solver->destroy(solver);
    free(solver);
}

cfd_status_t poisson_solver_solve(poisson_solver_t* solver, double* x, double* x_temp,
                                  const double* rhs, poisson_solver_stats_t* stats) {
    /* linear_solver.c:487-509 (every GPU solver has its own solve) */
    if (!solver) return CFD_ERROR_INVALID;
    if (!solver->solve) return CFD_ERROR_UNSUPPORTED;
    double t0 = now_ms();
    cfd_status_t st = solver->solve(solver, x, x_temp, rhs, stats);
    if (stats) stats->elapsed_time_ms = now_ms() - t0;
    return st;
}

cfd_status_t poisson_solver_iterate(poisson_solver_t* solver, double* x, double* x_temp,
                                    const double* rhs, double* residual) {
    /* linear_solver.c:511-527 */
    if (!solver || !x || !rhs) return CFD_ERROR_INVALID;
    if (!solver->iterate) return CFD_ERROR_UNSUPPORTED;
    return solver->iterate(solver, x, x_temp, rhs, residual);
}

/* ------------------------------------------------------------------------ */
/* legacy VTK output (vtk_output.c:110-275)                                  */
/* ------------------------------------------------------------------------ */
void write_vtk_output(const char* filename, const char* field_name, const double* data, size_t nx,
                      size_t ny, size_t nz, double xmin, double xmax, double ymin, double ymax,
                      double zmin, double zmax) {
    if (!filename || !field_name || !data ||
        !vtk_grid_ok(nx, ny, nz, xmin, xmax, ymin, ymax, zmin, zmax))
        return;
    FILE* fp = fopen(filename, "w");
    if (!fp) {
        cfd_set_error(CFD_ERROR_IO, "Failed to open VTK output file");
        return;
    }
    vtk_header(fp, "CFD Framework Output", nx, ny, nz, xmin, xmax, ymin, ymax, zmin, zmax);
    fprintf(fp, "\nPOINT_DATA %zu\n", nx * ny * nz);
    vtk_scalars(fp, field_name, data, nx * ny * nz);
    fclose(fp);
}

void write_vtk_vector_output(const char* filename, const char* field_name, const double* u_data,
                             const double* v_data, const double* w_data, size_t nx, size_t ny,
                             size_t nz, double xmin, double xmax, double ymin, double ymax,
                             double zmin, double zmax) {
    if (!filename || !field_name || !u_data || !v_data ||
        !vtk_grid_ok(nx, ny, nz, xmin, xmax, ymin, ymax, zmin, zmax))
        return;
    FILE* fp = fopen(filename, "w");
    if (!fp) {
        cfd_set_error(CFD_ERROR_IO, "Failed to open VTK vector output file");
        return;
    }
    vtk_header(fp, "CFD Framework Vector Output", nx, ny, nz, xmin, xmax, ymin, ymax, zmin, zmax);
    fprintf(fp, "\nPOINT_DATA %zu\n", nx * ny * nz);
    vtk_vectors(fp, field_name, u_data, v_data, w_data, nx * ny * nz);
    fclose(fp);
}

void write_vtk_flow_field(const char* filename, const flow_field* field, size_t nx, size_t ny,
                          size_t nz, double xmin, double xmax, double ymin, double ymax,
                          double zmin, double zmax) {
    if (!filename || !field || !vtk_grid_ok(nx, ny, nz, xmin, xmax, ymin, ymax, zmin, zmax))
        return;
    if (vtk_write_flow_field_file(filename, field->u, field->v, field->w, field->p, field->rho,
                                  field->T, nx, ny, nz, xmin, xmax, ymin, ymax, zmin,
                                  zmax) != 0)
        cfd_set_error(CFD_ERROR_IO, "Failed to open VTK flow field output file");
}
