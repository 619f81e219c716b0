// rk4_hip.hip -- the RK4 integrator on a hip_proj
// context: rk4_impl (solver_rk4.c:69-259) with max_iter = 1 per step.
//
// Per step: four fused stage kernels (k_rk_stage: RHS + stage update +
// running k1 + 2k2 + 2k3 sum, the stage derivatives stay in registers), the
// energy equation on the new velocity, the periodic boundary copies of
// apply_boundary_conditions (solver_explicit_euler.c:231-306) on u,v,w,p,
// rho,T, the thermal BCs, then one stats / NaN pass. Stage states ping-pong
// between the context's CG work arrays (u*,v*,w*,p_new and r,p_a,p_b,x_tmp);
// the final update is written in place over u,v,w,p.
#include "ctx.hpp"

static cfd_status_t ensure_rk(hip_proj_ctx* c) {
    const size_t n = field_elems(c);
    for (int q = 0; q < 4; ++q)
        if (!c->rk_acc[q]) ST_TRY(dalloc(c, &c->rk_acc[q], n));
    if (!c->xt) ST_TRY(dalloc(c, &c->xt, n));
    if (!c->dxa) ST_TRY(dalloc(c, &c->dxa, c->nx));
    if (!c->dya) ST_TRY(dalloc(c, &c->dya, c->ny));
    if (!c->rho) {
        // no per-cell density supplied: uniform rho0 (what set_density sets)
        ST_TRY(dalloc(c, &c->rho, n));
        double* h = nullptr;
        HIP_TRY(hipHostMalloc((void**)&h, n * sizeof(double), hipHostMallocDefault));
        for (size_t e = 0; e < n; ++e) h[e] = c->rho0;
        hipError_t e1 = hipMemcpyAsync(c->rho, h, n * sizeof(double), hipMemcpyHostToDevice,
                                       c->stream);
        hipError_t e2 = hipStreamSynchronize(c->stream);
        hipHostFree(h);
        HIP_TRY(e1);
        HIP_TRY(e2);
    }
    return CFD_SUCCESS;
}

template <int S>
static void launch_stage(hip_proj_ctx* c, bool buoy, const RkCoef& rc, const Fld4& cur,
                         const Fld4& q0, const Fld4& acc, const Fld4& out) {
    // x-pair stage kernel (default); CFD_HIP_RK_PAIR=0 selects the per-cell one
    const bool pair = c->env.rk_pair;
    if (pair) {
        const dim3 g2((unsigned)((c->nx + 127) / 128), (unsigned)((c->ny + 3) / 4),
                      (unsigned)c->nz);
        if (buoy)
            hipExtLaunchKernelGGL((k_rk_stage2<S, true>), g2, dim3(256), 0, c->stream, c->ta,
                                  c->tb, 0, c->geo, rc, cur, q0, acc, out, c->rho, c->T, c->dxa,
                                  c->dya, c->src_u_row, c->src_v_col);
        else
            hipExtLaunchKernelGGL((k_rk_stage2<S, false>), g2, dim3(256), 0, c->stream, c->ta,
                                  c->tb, 0, c->geo, rc, cur, q0, acc, out, c->rho, c->T, c->dxa,
                                  c->dya, c->src_u_row, c->src_v_col);
        return;
    }
    const dim3 grid = cell_grid(c);
    if (buoy)
        hipExtLaunchKernelGGL((k_rk_stage<S, true>), grid, dim3(256), 0, c->stream, c->ta, c->tb,
                              0, c->geo, rc, cur, q0, acc, out, c->rho, c->T, c->dxa, c->dya,
                              c->src_u_row, c->src_v_col);
    else
        hipExtLaunchKernelGGL((k_rk_stage<S, false>), grid, dim3(256), 0, c->stream, c->ta,
                              c->tb, 0, c->geo, rc, cur, q0, acc, out, c->rho, c->T, c->dxa,
                              c->dya, c->src_u_row, c->src_v_col);
}

static cfd_status_t rk4_step_impl(hip_proj_ctx* c, const grid* g, const ns_solver_params_t* prm,
                                  ns_solver_stats_t* stats, int iter) {
    if (!c) return CFD_ERROR_INVALID;
    if (c->nranks > 1) {
        set_err(CFD_ERROR_UNSUPPORTED, "rk4_hip: Z-slab decomposition is not supported");
        return CFD_ERROR_UNSUPPORTED;
    }
    ST_TRY(ctx_validate_params(c, g, prm));
    HIP_TRY(hipSetDevice(c->device));
    const bool buoy = (prm->beta != 0.0);
    const bool energy = (prm->alpha > 0.0);
    if ((buoy || energy) && !c->have_T) {
        set_err(CFD_ERROR_INVALID, "rk4_hip: buoyancy / energy equation need the T field");
        return CFD_ERROR_INVALID;
    }
    ST_TRY(ensure_rk(c));
    const size_t nx = c->nx, ny = c->ny, nz = c->nzg;
    const double dt = prm->dt;

    // per-index spacing and compute_source_terms tables (iter-dependent decay),
    // evaluated on the host with the reference's libm expressions
    HIP_TRY(hipMemcpyAsync(c->dxa, g->dx, nx * sizeof(double), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->dya, g->dy, ny * sizeof(double), hipMemcpyHostToDevice, c->stream));
    ST_TRY(upload_source_tables(c, g, prm, iter));

    RkCoef rc;
    rc.inv_2dz = (nz > 1 && g->dz) ? 1.0 / (2.0 * g->dz[0]) : 0.0;
    rc.inv_dz2 = (nz > 1 && g->dz) ? 1.0 / (g->dz[0] * g->dz[0]) : 0.0;
    rc.mu = prm->mu;
    rc.beta = prm->beta;
    rc.T_ref = prm->T_ref;
    rc.g0 = prm->gravity[0];
    rc.g1 = prm->gravity[1];
    rc.g2 = prm->gravity[2];
    const Fld4 q0{{c->u, c->v, c->w, c->p}};
    const Fld4 a{{c->us, c->vs, c->ws, c->pn}};
    const Fld4 b{{c->r, c->pa, c->pb, c->xt}};
    const Fld4 acc{{c->rk_acc[0], c->rk_acc[1], c->rk_acc[2], c->rk_acc[3]}};
    timed(c, HIP_KT_RK_STAGE, [&] {
        rc.fac = 0.5 * dt;
        launch_stage<0>(c, buoy, rc, q0, q0, acc, a);
    });
    timed(c, HIP_KT_RK_STAGE, [&] { launch_stage<1>(c, buoy, rc, a, q0, acc, b); });
    timed(c, HIP_KT_RK_STAGE, [&] {
        rc.fac = dt;
        launch_stage<2>(c, buoy, rc, b, q0, acc, a);
    });
    timed(c, HIP_KT_RK_STAGE, [&] {
        rc.fac = dt / 6.0;
        launch_stage<3>(c, buoy, rc, a, q0, acc, q0);
    });
    HIP_TRY(hipGetLastError());
    c->cg_scratch_dirty = 1;  // r, p_a, p_b now hold stage values at the walls

    hipLaunchKernelGGL(k_init_red, dim3(1), dim3(64), 0, c->stream, c->red);
    if (energy) ST_TRY(ctx_energy_step(c, g, prm, false));  // solver_rk4.c:213-221
    // apply_boundary_conditions: periodic copies of every field (x, y, z faces)
    for (double* f : {c->u, c->v, c->w, c->p, c->rho, c->T})
        if (f) launch_bc(c, f, 1, DirVals{});
    if (c->T) c->T_dirty = 1;
    if (energy) ST_TRY(ctx_apply_thermal_bcs(c, prm->thermal_bc, nz > 1));  // :228-232
    const dim3 cg = cell_grid(c);
    hipLaunchKernelGGL(k_vel_stats, cg, dim3(256), 0, c->stream, c->geo, c->u, c->v, c->w, c->p,
                       c->red);
    ctx_queue_max_T(c);
    HIP_TRY(hipMemcpyAsync(c->h_red, c->red, 8 * sizeof(unsigned long long),
                           hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    flush_timing(c);
    if (c->h_red[5]) {
        set_err(CFD_ERROR_DIVERGED, "NaN/Inf detected in energy_step_explicit");
        return CFD_ERROR_DIVERGED;
    }
    if (c->have_T && c->T_dirty) {
        c->max_T = ord_dec(c->h_red[3]);
        c->T_dirty = 0;
    }
    if (stats) {
        stats->iterations = 1;
        stats->max_velocity = std::sqrt(ord_dec(c->h_red[0]));  // red[0]: max |u|^2
        stats->max_pressure = ord_dec(c->h_red[1]);
        stats->max_temperature = c->have_T ? c->max_T : 0.0;
    }
    if (c->h_red[2]) {
        set_err(CFD_ERROR_DIVERGED, "rk4_hip: NaN/Inf in the flow field");
        return CFD_ERROR_DIVERGED;
    }
    return CFD_SUCCESS;
}

// Host-buffer path for hip_rk4_step and the rk4_hip plugin (n steps, source
// iteration index 0..n-1 like rk4_impl's loop).
extern "C" __attribute__((visibility("hidden"))) cfd_status_t hip_rk4_step_iter_internal(
    hip_proj_ctx_t* c, flow_field* f, const grid* g, const ns_solver_params_t* prm,
    ns_solver_stats_t* stats, int n_steps) {
    if (!c || !f || !g || !prm) return CFD_ERROR_INVALID;
    if (f->nx < 3 || f->ny < 3 || (f->nz > 1 && f->nz < 3)) return CFD_ERROR_INVALID;
    ST_TRY(ctx_validate_params(c, g, prm));
    if (n_steps <= 0) return CFD_SUCCESS;
    c->resident = 0;
    const int ids[4] = {HIP_FIELD_U, HIP_FIELD_V, HIP_FIELD_W, HIP_FIELD_P};
    double* hf[4] = {f->u, f->v, f->w, f->p};
    for (int q = 0; q < 4; ++q) ST_TRY(hip_proj_set_field(c, ids[q], hf[q]));
    if (f->rho) ST_TRY(hip_proj_set_field(c, HIP_FIELD_RHO, f->rho));
    if (f->T) ST_TRY(hip_proj_set_field(c, HIP_FIELD_T, f->T));
    cfd_status_t s = CFD_SUCCESS;
    for (int it = 0; it < n_steps; ++it) {
        s = rk4_step_impl(c, g, prm, stats, it);
        if (s != CFD_SUCCESS) break;
    }
    if (s == CFD_SUCCESS || s == CFD_ERROR_DIVERGED) {
        for (int q = 0; q < 4; ++q) ST_TRY(hip_proj_get_field(c, ids[q], hf[q]));
        if (f->rho) ST_TRY(hip_proj_get_field(c, HIP_FIELD_RHO, f->rho));
        if (f->T) ST_TRY(hip_proj_get_field(c, HIP_FIELD_T, f->T));
    }
    return s;
}

extern "C" {

cfd_status_t hip_rk4_step_device(hip_proj_ctx_t* c, const grid* g, const ns_solver_params_t* prm,
                                 ns_solver_stats_t* stats) {
    GroupHostLock hl_(c);
    return rk4_step_impl(c, g, prm, stats, 0);
}

cfd_status_t hip_rk4_step(hip_proj_ctx_t* c, flow_field* f, const grid* g,
                          const ns_solver_params_t* prm, ns_solver_stats_t* stats) {
    GroupHostLock hl_(c);
    return hip_rk4_step_iter_internal(c, f, g, prm, stats, 1);
}

}  // extern "C"
