// gpu_device_hip.hip -- the reference's device API (cfd/core/gpu_device.h,
// implemented in lib/src/solvers/gpu/solver_projection_gpu.cu:294-770 and
// solver_rk_gpu.cu:546-553) on top of the persistent hip_proj context.
//
// gpu_solver_step is the reference's explicit pressure-relaxation step
// (solver_projection_gpu.cu:523-570):
//   rhs   = -(u.grad)u + nu lap u - grad p          (kernel_velocity_rhs :158-205, inv_rho 1)
//   u     = clamp(u + dt rhs)                        (kernel_velocity_update :207-228)
//   Neumann BC on u, v, w                            (bc_apply_velocity_3d_gpu)
//   div   = div u                                    (kernel_compute_divergence :78-95)
//   p    -= 0.1 dt (1/dx^2 + 1/dy^2 + 1/dz^2)/ndim * div   (kernel_pressure_update :257-269)
//   Neumann BC on p                                  (bc_apply_scalar_3d_gpu)
// Here it is two fused sweeps: k_gs_momentum (RHS + update, written to the
// u*/v*/w* buffers so the stencil never reads a cell it already advanced --
// the reference gets the same effect from separate rhs arrays), the boundary
// gathers, and k_gs_pressure (divergence + pressure update in one pass).
// Every per-cell expression keeps the reference kernels' operation order
// (-ffp-contract=off), so the fields are bitwise the reference GPU's.
#include "ctx.hpp"

#include "cfd_hip/gpu_device.h"

#include <new>

extern "C" __attribute__((visibility("hidden"))) cfd_status_t hip_proj_step_iter_internal(
    hip_proj_ctx_t* c, flow_field* f, const grid* g, const ns_solver_params_t* prm,
    ns_solver_stats_t* stats, int n_steps);
extern "C" __attribute__((visibility("hidden"))) cfd_status_t hip_rk4_step_iter_internal(
    hip_proj_ctx_t* c, flow_field* f, const grid* g, const ns_solver_params_t* prm,
    ns_solver_stats_t* stats, int n_steps);

namespace {

constexpr double GS_MAX_VELOCITY = 100.0;  // MAX_VELOCITY of the reference kernels

struct GsCoef {
    double inv_2dx, inv_2dy, inv_2dz;
    double inv_dx2, inv_dy2, inv_dz2;
    double nu, dt, p_relax;
};

__device__ __forceinline__ double gs_clamp(double v) {
    return fmax(-GS_MAX_VELOCITY, fmin(GS_MAX_VELOCITY, v));
}

// kernel_velocity_rhs + kernel_velocity_update, interior cells; boundary
// cells of the outputs are rewritten by the Neumann gathers that follow.
__global__ __launch_bounds__(256) void k_gs_momentum(Geo g, GsCoef q,
                                                     const double* __restrict__ U,
                                                     const double* __restrict__ V,
                                                     const double* __restrict__ W,
                                                     const double* __restrict__ P,
                                                     double* __restrict__ Uo,
                                                     double* __restrict__ Vo,
                                                     double* __restrict__ Wo) {
    const int i = blockIdx.x * 64 + (threadIdx.x & 63);
    const int j = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int k = blockIdx.z;
    if (i < 1 || i > g.nx - 2 || j < 1 || j > g.ny - 2 || k < g.k0 || k >= g.k1) return;
    const long long idx = cidx(g, i, j, k);
    const long long px = g.px, sz = g.sz;
    const double u_c = U[idx], v_c = V[idx], w_c = W[idx];

    const double du_dx = (U[idx + 1] - U[idx - 1]) * q.inv_2dx;
    const double du_dy = (U[idx + px] - U[idx - px]) * q.inv_2dy;
    const double du_dz = (U[idx + sz] - U[idx - sz]) * q.inv_2dz;
    const double d2u = (U[idx + 1] - 2.0 * u_c + U[idx - 1]) * q.inv_dx2 +
                       (U[idx + px] - 2.0 * u_c + U[idx - px]) * q.inv_dy2 +
                       (U[idx + sz] - 2.0 * u_c + U[idx - sz]) * q.inv_dz2;
    const double dv_dx = (V[idx + 1] - V[idx - 1]) * q.inv_2dx;
    const double dv_dy = (V[idx + px] - V[idx - px]) * q.inv_2dy;
    const double dv_dz = (V[idx + sz] - V[idx - sz]) * q.inv_2dz;
    const double d2v = (V[idx + 1] - 2.0 * v_c + V[idx - 1]) * q.inv_dx2 +
                       (V[idx + px] - 2.0 * v_c + V[idx - px]) * q.inv_dy2 +
                       (V[idx + sz] - 2.0 * v_c + V[idx - sz]) * q.inv_dz2;
    const double dw_dx = (W[idx + 1] - W[idx - 1]) * q.inv_2dx;
    const double dw_dy = (W[idx + px] - W[idx - px]) * q.inv_2dy;
    const double dw_dz = (W[idx + sz] - W[idx - sz]) * q.inv_2dz;
    const double d2w = (W[idx + 1] - 2.0 * w_c + W[idx - 1]) * q.inv_dx2 +
                       (W[idx + px] - 2.0 * w_c + W[idx - px]) * q.inv_dy2 +
                       (W[idx + sz] - 2.0 * w_c + W[idx - sz]) * q.inv_dz2;
    const double dp_dx = (P[idx + 1] - P[idx - 1]) * q.inv_2dx;
    const double dp_dy = (P[idx + px] - P[idx - px]) * q.inv_2dy;
    const double dp_dz = (P[idx + sz] - P[idx - sz]) * q.inv_2dz;

    const double inv_rho = 1.0;  // gpu_solver_step passes 1.0 (:537)
    const double ru = -(u_c * du_dx + v_c * du_dy + w_c * du_dz) + q.nu * d2u - inv_rho * dp_dx;
    const double rv = -(u_c * dv_dx + v_c * dv_dy + w_c * dv_dz) + q.nu * d2v - inv_rho * dp_dy;
    const double rw = -(u_c * dw_dx + v_c * dw_dy + w_c * dw_dz) + q.nu * d2w - inv_rho * dp_dz;
    Uo[idx] = gs_clamp(u_c + q.dt * ru);
    Vo[idx] = gs_clamp(v_c + q.dt * rv);
    Wo[idx] = gs_clamp(w_c + q.dt * rw);
}

// kernel_compute_divergence + kernel_pressure_update on the advanced velocity
// (boundary values already Neumann-updated), interior cells.
__global__ __launch_bounds__(256) void k_gs_pressure(Geo g, GsCoef q,
                                                     const double* __restrict__ U,
                                                     const double* __restrict__ V,
                                                     const double* __restrict__ W,
                                                     double* __restrict__ P) {
    const int i = blockIdx.x * 64 + (threadIdx.x & 63);
    const int j = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int k = blockIdx.z;
    if (i < 1 || i > g.nx - 2 || j < 1 || j > g.ny - 2 || k < g.k0 || k >= g.k1) return;
    const long long idx = cidx(g, i, j, k);
    const double div = (U[idx + 1] - U[idx - 1]) * q.inv_2dx +
                       (V[idx + g.px] - V[idx - g.px]) * q.inv_2dy +
                       (W[idx + g.sz] - W[idx - g.sz]) * q.inv_2dz;
    P[idx] -= q.p_relax * div;
}

}  // namespace

struct gpu_solver_context_t {
    hip_proj_ctx_t* pc = nullptr;
    gpu_config_t cfg{};
    gpu_solver_stats_t stats{};
    hipEvent_t e0 = nullptr, e1 = nullptr;
};

extern "C" {

gpu_config_t gpu_config_default(void) {
    // solver_projection_gpu.cu:294-308
    gpu_config_t c;
    memset(&c, 0, sizeof(c));
    c.enable_gpu = 1;
    c.min_grid_size = 10000;
    c.min_steps = 10;
    c.block_size_x = 16;
    c.block_size_y = 16;
    c.poisson_max_iter = 1000;
    c.poisson_tolerance = 1e-3;
    c.persistent_memory = 1;
    c.async_transfers = 1;
    c.sync_after_kernel = 0;
    c.verbose = 0;
    return c;
}

int gpu_is_available(void) { return hip_projection_available(); }

int gpu_get_device_info(gpu_device_info_t* info, int max_devices) {
    // solver_projection_gpu.cu:327-352
    int n = 0;
    if (!info || max_devices <= 0 || hipGetDeviceCount(&n) != hipSuccess) return 0;
    int cur = 0;
    hipGetDevice(&cur);
    const int count = std::min(n, max_devices);
    for (int i = 0; i < count; ++i) {
        hipDeviceProp_t prop;
        memset(&info[i], 0, sizeof(info[i]));
        if (hipGetDeviceProperties(&prop, i) != hipSuccess) continue;
        info[i].device_id = i;
        snprintf(info[i].name, sizeof(info[i].name), "%s",
                 prop.name[0] ? prop.name : prop.gcnArchName);
        info[i].total_memory = prop.totalGlobalMem;
        info[i].compute_capability_major = prop.major;
        info[i].compute_capability_minor = prop.minor;
        info[i].multiprocessor_count = prop.multiProcessorCount;
        info[i].max_threads_per_block = prop.maxThreadsPerBlock;
        info[i].warp_size = prop.warpSize;
        info[i].is_available = 1;
        size_t fr = 0, tot = 0;
        if (hipSetDevice(i) == hipSuccess && hipMemGetInfo(&fr, &tot) == hipSuccess)
            info[i].free_memory = fr;
    }
    hipSetDevice(cur);
    return count;
}

cfd_status_t gpu_select_device(int device_id) {
    if (hipSetDevice(device_id) == hipSuccess) return CFD_SUCCESS;
    (void)hipGetLastError();  // do not leave the failed call as the thread's last error
    return CFD_ERROR;
}

int gpu_should_use(const gpu_config_t* config, size_t nx, size_t ny, size_t nz, int num_steps) {
    // solver_projection_gpu.cu:358-373
    if (!config || !config->enable_gpu) return 0;
    if (!gpu_is_available()) return 0;
    if (nx < 3 || ny < 3 || nz == 0 || nz == 2) return 0;
    if (ny > SIZE_MAX / nx || nz > SIZE_MAX / (nx * ny)) return 0;
    if (nx * ny * nz < config->min_grid_size) return 0;
    if (num_steps < config->min_steps) return 0;
    return 1;
}

void gpu_solver_destroy(gpu_solver_context_t* ctx) {
    if (!ctx) return;
    if (ctx->pc) hip_proj_destroy(ctx->pc);
    if (ctx->e0) hipEventDestroy(ctx->e0);
    if (ctx->e1) hipEventDestroy(ctx->e1);
    delete ctx;
}

gpu_solver_context_t* gpu_solver_create(size_t nx, size_t ny, size_t nz,
                                        const gpu_config_t* config) {
    // solver_projection_gpu.cu:375-446 (validation and messages)
    if (!gpu_is_available()) return nullptr;
    if (nx < 3 || ny < 3 || nz == 0) {
        set_err(CFD_ERROR_INVALID, "GPU solver requires nx>=3, ny>=3, nz>=1");
        return nullptr;
    }
    if (nz == 2) {
        set_err(CFD_ERROR_INVALID, "GPU solver requires nz==1 (2D) or nz>=3 (3D), got nz==2");
        return nullptr;
    }
    if (ny > SIZE_MAX / nx || nz > SIZE_MAX / (nx * ny)) {
        set_err(CFD_ERROR_INVALID, "Grid dimensions too large: nx*ny*nz overflows");
        return nullptr;
    }
    gpu_solver_context_t* ctx = new (std::nothrow) gpu_solver_context_t();
    if (!ctx) return nullptr;
    ctx->cfg = config ? *config : gpu_config_default();
    hip_proj_config_t pcfg = hip_proj_config_default();
    pcfg.poisson_tolerance = ctx->cfg.poisson_tolerance;
    pcfg.poisson_abs_tolerance = 0.0;
    pcfg.poisson_max_iter = ctx->cfg.poisson_max_iter;
    pcfg.rhs_density = 0;
    pcfg.poisson_fail_fatal = 0;
    pcfg.verbose = ctx->cfg.verbose;
    ctx->pc = hip_proj_create(nx, ny, nz, &pcfg);
    if (!ctx->pc || hipEventCreate(&ctx->e0) != hipSuccess ||
        hipEventCreate(&ctx->e1) != hipSuccess) {
        gpu_solver_destroy(ctx);
        return nullptr;
    }
    ctx->stats.memory_allocated = hip_proj_device_bytes(ctx->pc);
    return ctx;
}

cfd_status_t gpu_solver_upload(gpu_solver_context_t* ctx, const flow_field* field) {
    // solver_projection_gpu.cu:478-505: w / T absent -> zero-filled
    if (!ctx || !field) return CFD_ERROR_INVALID;
    hip_proj_ctx* c = ctx->pc;
    if (field->nx != c->nx || field->ny != c->ny || field->nz != c->nz) return CFD_ERROR_INVALID;
    HIP_TRY(hipEventRecord(ctx->e0, c->stream));
    ST_TRY(hip_proj_set_field(c, HIP_FIELD_U, field->u));
    ST_TRY(hip_proj_set_field(c, HIP_FIELD_V, field->v));
    if (field->w) ST_TRY(hip_proj_set_field(c, HIP_FIELD_W, field->w));
    else ST_TRY(hip_proj_fill_field(c, HIP_FIELD_W, 0.0));
    ST_TRY(hip_proj_set_field(c, HIP_FIELD_P, field->p));
    if (field->T) ST_TRY(hip_proj_set_field(c, HIP_FIELD_T, field->T));
    c->rho0 = field->rho ? field->rho[0] : 1.0;
    HIP_TRY(hipEventRecord(ctx->e1, c->stream));
    HIP_TRY(hipEventSynchronize(ctx->e1));
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ctx->e0, ctx->e1) == hipSuccess) ctx->stats.transfer_time_ms += ms;
    return CFD_SUCCESS;
}

cfd_status_t gpu_solver_download(gpu_solver_context_t* ctx, flow_field* field) {
    // solver_projection_gpu.cu:507-521
    if (!ctx || !field) return CFD_ERROR_INVALID;
    hip_proj_ctx* c = ctx->pc;
    if (field->nx != c->nx || field->ny != c->ny || field->nz != c->nz) return CFD_ERROR_INVALID;
    HIP_TRY(hipEventRecord(ctx->e0, c->stream));
    ST_TRY(hip_proj_get_field(c, HIP_FIELD_U, field->u));
    ST_TRY(hip_proj_get_field(c, HIP_FIELD_V, field->v));
    if (field->w) ST_TRY(hip_proj_get_field(c, HIP_FIELD_W, field->w));
    ST_TRY(hip_proj_get_field(c, HIP_FIELD_P, field->p));
    if (field->T && c->T) ST_TRY(hip_proj_get_field(c, HIP_FIELD_T, field->T));
    HIP_TRY(hipEventRecord(ctx->e1, c->stream));
    HIP_TRY(hipEventSynchronize(ctx->e1));
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ctx->e0, ctx->e1) == hipSuccess) ctx->stats.transfer_time_ms += ms;
    return CFD_SUCCESS;
}

cfd_status_t gpu_solver_step(gpu_solver_context_t* ctx, const grid* g,
                             const ns_solver_params_t* params, gpu_solver_stats_t* stats) {
    // solver_projection_gpu.cu:523-570
    if (!ctx || !g || !params) return CFD_ERROR_INVALID;
    hip_proj_ctx* c = ctx->pc;
    if (!g->dx || !g->dy || (c->nz > 1 && !g->dz)) return CFD_ERROR_INVALID;
    HIP_TRY(hipSetDevice(c->device));
    const bool is3d = c->nz > 1;
    const double dx = g->dx[0], dy = g->dy[0], dt = params->dt;
    GsCoef q;
    q.inv_2dx = 0.5 / dx;
    q.inv_2dy = 0.5 / dy;
    q.inv_dx2 = 1.0 / (dx * dx);
    q.inv_dy2 = 1.0 / (dy * dy);
    q.inv_2dz = is3d ? 0.5 / g->dz[0] : 0.0;
    q.inv_dz2 = is3d ? 1.0 / (g->dz[0] * g->dz[0]) : 0.0;
    q.nu = params->mu;
    q.dt = dt;
    const double ndim = is3d ? 3.0 : 2.0;
    q.p_relax = 0.1 * dt * (q.inv_dx2 + q.inv_dy2 + q.inv_dz2) / ndim;

    const dim3 cg = cell_grid(c);
    const DirVals dv{};
    (void)hipGetLastError();  // launch errors below are this step's own
    HIP_TRY(hipEventRecord(ctx->e0, c->stream));
    hipLaunchKernelGGL(k_gs_momentum, cg, dim3(256), 0, c->stream, c->geo, q, c->u, c->v, c->w,
                       c->p, c->us, c->vs, c->ws);
    // the advanced velocity becomes the field; its boundary is the Neumann
    // gather of its own interior (bc_apply_velocity_3d_gpu, BC_TYPE_NEUMANN)
    std::swap(c->u, c->us);
    std::swap(c->v, c->vs);
    std::swap(c->w, c->ws);
    launch_bc(c, c->u, 0, dv);
    launch_bc(c, c->v, 0, dv);
    launch_bc(c, c->w, 0, dv);
    hipLaunchKernelGGL(k_gs_pressure, cg, dim3(256), 0, c->stream, c->geo, q, c->u, c->v, c->w,
                       c->p);
    launch_bc(c, c->p, 0, dv);
    HIP_TRY(hipGetLastError());
    HIP_TRY(hipEventRecord(ctx->e1, c->stream));
    HIP_TRY(hipEventSynchronize(ctx->e1));
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, ctx->e0, ctx->e1) == hipSuccess) ctx->stats.kernel_time_ms += ms;
    ctx->stats.kernels_launched += 6;
    if (stats) *stats = ctx->stats;
    return CFD_SUCCESS;
}

gpu_solver_stats_t gpu_solver_get_stats(const gpu_solver_context_t* ctx) {
    if (!ctx) {
        gpu_solver_stats_t e;
        memset(&e, 0, sizeof(e));
        return e;
    }
    return ctx->stats;
}

void gpu_solver_reset_stats(gpu_solver_context_t* ctx) {
    if (!ctx) return;
    const size_t mem = ctx->stats.memory_allocated;  // preserved across reset (:585)
    memset(&ctx->stats, 0, sizeof(ctx->stats));
    ctx->stats.memory_allocated = mem;
}

cfd_status_t solve_navier_stokes_gpu(flow_field* field, const grid* g,
                                     const ns_solver_params_t* params,
                                     const gpu_config_t* config) {
    // solver_projection_gpu.cu:590-612
    if (!field || !g || !params) return CFD_ERROR_INVALID;
    gpu_config_t cfg = config ? *config : gpu_config_default();
    if (!gpu_should_use(&cfg, field->nx, field->ny, field->nz, params->max_iter)) return CFD_ERROR;
    gpu_solver_context_t* ctx = gpu_solver_create(field->nx, field->ny, field->nz, &cfg);
    if (!ctx) return CFD_ERROR_NOMEM;
    if (gpu_solver_upload(ctx, field) != CFD_SUCCESS) {
        gpu_solver_destroy(ctx);
        return CFD_ERROR;
    }
    gpu_solver_stats_t st;
    for (int it = 0; it < params->max_iter; ++it)
        if (gpu_solver_step(ctx, g, params, &st) != CFD_SUCCESS) break;
    gpu_solver_download(ctx, field);
    gpu_solver_destroy(ctx);
    return CFD_SUCCESS;
}

cfd_status_t solve_projection_method_gpu(flow_field* field, const grid* g,
                                         const ns_solver_params_t* params,
                                         const gpu_config_t* config) {
    // solver_projection_gpu.cu:617-770: the reference GPU's settings on the
    // projection_hip step (Poisson tol/cap from the config, absolute 0, a
    // capped solve non-fatal, RHS div/dt, no default source term)
    if (!field || !g || !params) return CFD_ERROR_INVALID;
    gpu_config_t cfg = config ? *config : gpu_config_default();
    if (!gpu_should_use(&cfg, field->nx, field->ny, field->nz, params->max_iter)) return CFD_ERROR;
    gpu_solver_context_t* ctx = gpu_solver_create(field->nx, field->ny, field->nz, &cfg);
    if (!ctx) return CFD_ERROR_NOMEM;
    ns_solver_params_t prm = *params;
    prm.source_amplitude_u = 0.0;  // kernel_predictor has no source term (:98-155)
    prm.source_amplitude_v = 0.0;
    cfd_status_t s = CFD_SUCCESS;
    // gpu_solver_upload zero-fills d_T when the field has none (:491-495), so
    // buoyancy / energy then act on T = 0 instead of failing
    if (!field->T && (prm.beta != 0.0 || prm.alpha > 0.0))
        s = hip_proj_fill_field(ctx->pc, HIP_FIELD_T, 0.0);
    if (s == CFD_SUCCESS)
        s = hip_proj_step_iter_internal(ctx->pc, field, g, &prm, nullptr, params->max_iter);
    gpu_solver_destroy(ctx);
    // the reference has no NaN scan and returns CFD_SUCCESS after its loop
    // (:762-769); a non-finite field is downloaded here as there
    if (s == CFD_ERROR_DIVERGED) s = CFD_SUCCESS;
    return s;
}

static cfd_status_t not_on_path(const char* what) {
    set_err(CFD_ERROR_UNSUPPORTED, what);
    return CFD_ERROR_UNSUPPORTED;
}

cfd_status_t solve_explicit_euler_method_gpu(flow_field*, const grid*, const ns_solver_params_t*,
                                             const gpu_config_t*) {
    return not_on_path("GPU explicit Euler solver: not provided by the MI355X projection library");
}

cfd_status_t solve_rk2_method_gpu(flow_field*, const grid*, const ns_solver_params_t*,
                                  const gpu_config_t*) {
    return not_on_path("GPU RK2 solver: not provided by the MI355X projection library");
}

cfd_status_t solve_rk4_method_gpu(flow_field* field, const grid* g,
                                  const ns_solver_params_t* params, const gpu_config_t* config) {
    // solver_rk_gpu.cu:260-553 (order 4): params->max_iter RK4 steps
    if (!field || !g || !params) return CFD_ERROR_INVALID;
    gpu_config_t cfg = config ? *config : gpu_config_default();
    if (!gpu_should_use(&cfg, field->nx, field->ny, field->nz, params->max_iter)) return CFD_ERROR;
    hip_proj_config_t pcfg = hip_proj_config_default();
    hip_proj_ctx_t* pc = hip_proj_create(field->nx, field->ny, field->nz, &pcfg);
    if (!pc) return CFD_ERROR_NOMEM;
    cfd_status_t s = hip_rk4_step_iter_internal(pc, field, g, params, nullptr, params->max_iter);
    hip_proj_destroy(pc);
    return s;
}

}  // extern "C"
