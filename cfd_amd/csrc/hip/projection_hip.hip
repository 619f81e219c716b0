// projection_hip.hip -- device context and step orchestration behind the
// C-ABI of include/cfd_hip/projection_hip.h.
//
// One context = one device, one HIP stream, all fields resident in HBM with a
// padded row pitch. A step is: predictor -> (p_new = p) -> pressure solve on
// p_new with the divergence right-hand side fused into the CG setup ->
// corrector + boundary restore + NaN scan + stats -> swap(p, p_new).
// The CG loop keeps alpha/beta/convergence on the device (CgState) and the
// host only polls a pinned copy of the state every few iterations, so there
// is no host round trip per iteration (the reference GPU path does two per
// iteration, poisson_cg_gpu_solve.cuh:189-203).
#include "ctx.hpp"

#include <array>
#include "rb2.hpp"
#include "ccf.hpp"

template <int TY, bool FIRST, bool DIST, int FL, bool FOLD>
static void launch_cgA_t(hip_proj_ctx* c, const Lap& L, const double* r, const double* po,
                         double* pn, int it, const PFold& fd) {
    hipExtLaunchKernelGGL((k_cgA<TY, FIRST, DIST, FL, FOLD>), dim3(sweep_grid(c)), dim3(64 * TY),
                          0, c->stream, c->ta, c->tb, 0, c->sgeo, L, r, po, pn, c->st, c->partials,
                          c->counter, it, c->dsum, mbox(c), fd);
}

// Sweep B operands: p = p_it (stencil) and r.
struct BArgs {
    const double* p;
    double* r;
};

template <int TY, bool DIST, int FL>
static void launch_cgB_t(hip_proj_ctx* c, const SGeo& sg, const Lap& L, const BArgs& a, int it) {
    const unsigned nb = (unsigned)(sg.tiles_x * sg.tiles_y * sg.tiles_z);
    // sweep B marches z downwards on one device in 3-D (r03: it starts on the
    // planes sweep A touched last, in the Infinity Cache; 512^3 sweep B
    // 0.551 -> 0.539 ms, CG iteration 1.355 -> 1.335 ms, profiles/r03_rev.jsonl);
    // CFD_HIP_CGB_REV=0 restores the upward march
    if (!DIST && c->env.cgb_rev && c->geo.sz && sg.kmode == 0) {
        hipExtLaunchKernelGGL((k_cgB<TY, DIST, FL, true>), dim3(nb), dim3(64 * TY), 0, c->stream,
                              c->ta, c->tb, 0, sg, L, a.p, a.r, c->st, c->partials, c->counter,
                              it, c->dsum, mbox(c));
        return;
    }
    hipExtLaunchKernelGGL((k_cgB<TY, DIST, FL>), dim3(nb), dim3(64 * TY), 0, c->stream, c->ta,
                          c->tb, 0, sg, L, a.p, a.r, c->st, c->partials, c->counter, it,
                          c->dsum, mbox(c));
}

// fd.x == nullptr: no fold this iteration
template <int TY, int FL>
static void launch_cgA_f(hip_proj_ctx* c, bool first, const Lap& L, const double* r,
                         const double* po, double* pn, int it, const PFold& fd) {
    const bool d = dist(c);
    if (first) d ? launch_cgA_t<TY, true, true, FL, false>(c, L, r, po, pn, it, fd)
                 : launch_cgA_t<TY, true, false, FL, false>(c, L, r, po, pn, it, fd);
    // the fold sweep streams 4 more fields: without the plane prefetch's
    // second register bundle it fits without spilling
    else if (fd.x) d ? launch_cgA_t<TY, false, true, (FL & ~SW_PREFETCH), true>(c, L, r, po, pn, it, fd)
                     : launch_cgA_t<TY, false, false, (FL & ~SW_PREFETCH), true>(c, L, r, po, pn, it, fd);
    else d ? launch_cgA_t<TY, false, true, FL, false>(c, L, r, po, pn, it, fd)
           : launch_cgA_t<TY, false, false, FL, false>(c, L, r, po, pn, it, fd);
}

template <int TY, int FL>
static void launch_cgB_f(hip_proj_ctx* c, const SGeo& sg, const Lap& L, const BArgs& a, int it) {
    if (dist(c)) launch_cgB_t<TY, true, FL>(c, sg, L, a, it);
    else launch_cgB_t<TY, false, FL>(c, sg, L, a, it);
}

template <int TY>
static void launch_cgA_v(hip_proj_ctx* c, bool first, const Lap& L, const double* r,
                         const double* po, double* pn, int it, const PFold& fd) {
    switch (c->sweep_variant) {
        case 1: return launch_cgA_f<TY, 1>(c, first, L, r, po, pn, it, fd);
        case 2: return launch_cgA_f<TY, 2>(c, first, L, r, po, pn, it, fd);
        case 3: return launch_cgA_f<TY, 3>(c, first, L, r, po, pn, it, fd);
        case 4: return launch_cgA_f<TY, 4>(c, first, L, r, po, pn, it, fd);
        case 7: return launch_cgA_f<TY, 7>(c, first, L, r, po, pn, it, fd);
        case 15: return launch_cgA_f<TY, 15>(c, first, L, r, po, pn, it, fd);
                 [[fallthrough]];
        case 23: if constexpr (TY == 16) return launch_cgA_f<TY, 23>(c, first, L, r, po, pn, it, fd);
                 [[fallthrough]];
        case 31: if constexpr (TY == 16) return launch_cgA_f<TY, 31>(c, first, L, r, po, pn, it, fd);
                 [[fallthrough]];
        default: return launch_cgA_f<TY, 0>(c, first, L, r, po, pn, it, fd);
    }
}

template <int TY>
static void launch_cgB_v(hip_proj_ctx* c, const SGeo& sg, const Lap& L, const BArgs& a, int it) {
    switch (c->sweep_variant) {
        case 1: return launch_cgB_f<TY, 1>(c, sg, L, a, it);
        case 2: return launch_cgB_f<TY, 2>(c, sg, L, a, it);
        case 3: return launch_cgB_f<TY, 3>(c, sg, L, a, it);
        case 4: return launch_cgB_f<TY, 4>(c, sg, L, a, it);
        case 7: return launch_cgB_f<TY, 7>(c, sg, L, a, it);
        case 15: return launch_cgB_f<TY, 15>(c, sg, L, a, it);
                 [[fallthrough]];
        case 23: if constexpr (TY == 16) return launch_cgB_f<TY, 23>(c, sg, L, a, it);
                 [[fallthrough]];
        case 31: if constexpr (TY == 16) return launch_cgB_f<TY, 31>(c, sg, L, a, it);
                 [[fallthrough]];
        default: return launch_cgB_f<TY, 0>(c, sg, L, a, it);
    }
}

// sweep_ty 8 or 16 (any sweep_variant), 4 (variant 0 only)
static void launch_cgA(hip_proj_ctx* c, bool first, const Lap& L, const double* r,
                       const double* po, double* pn, int it, const PFold& fd) {
    if (c->sweep_ty == 4) return launch_cgA_f<4, 0>(c, first, L, r, po, pn, it, fd);
    if (c->sweep_ty == 16) return launch_cgA_v<16>(c, first, L, r, po, pn, it, fd);
    return launch_cgA_v<8>(c, first, L, r, po, pn, it, fd);
}

static void launch_cgB(hip_proj_ctx* c, const SGeo& sg, const Lap& L, const BArgs& a, int it) {
    if (c->sweep_ty == 4) return launch_cgB_f<4, 0>(c, sg, L, a, it);
    if (c->sweep_ty == 16) return launch_cgB_v<16>(c, sg, L, a, it);
    return launch_cgB_v<8>(c, sg, L, a, it);
}

// Chronopoulos-Gear CG launches (cg_variant 1)
template <bool FIRST, bool FOLD>
static void launch_cc1_t(hip_proj_ctx* c, double* pn, const double* po, const PPrev& pv, double* x,
                         int it) {
    const unsigned n = (unsigned)(c->px / 2) * (unsigned)(c->ny - 2) *
                       (unsigned)(c->sgeo.k1 - c->sgeo.k0);
    const unsigned nb = std::max(1u, std::min((n + 255) / 256, (unsigned)c->grid_cap * 4));
    hipExtLaunchKernelGGL((k_cc1<FIRST, FOLD>), dim3(nb), dim3(256), 0, c->stream, c->ta, c->tb, 0,
                          c->sgeo, c->r, c->cw, c->cs, po, pn, pv, x, c->st, it);
}

static void launch_cc1(hip_proj_ctx* c, double* pn, const double* po, const PPrev& pv, double* x,
                       int it) {
    const bool fold = (it % CG_XFOLD) == CG_XFOLD - 1;
    if (it == 0) launch_cc1_t<true, false>(c, pn, po, pv, x, it);
    else if (fold) launch_cc1_t<false, true>(c, pn, po, pv, x, it);
    else launch_cc1_t<false, false>(c, pn, po, pv, x, it);
}

template <int TY, bool DIST, bool INIT, bool WST>
static void launch_cc2_t(hip_proj_ctx* c, const SGeo& g, const Lap& L, int it, const double* r) {
    const unsigned nb = (unsigned)(g.tiles_x * g.tiles_y * g.tiles_z);
    hipExtLaunchKernelGGL((k_cc2<TY, DIST, INIT, WST>), dim3(nb), dim3(64 * TY), 0,
                          c->stream, c->ta, c->tb, 0, g, L, r, c->cw, c->st, c->partials,
                          c->counter, it, c->dsum, mbox(c));
}

template <int TY, bool WST>
static void launch_cc2_w(hip_proj_ctx* c, const SGeo& g, const Lap& L, int it, bool init,
                         const double* r) {
    if (dist(c)) init ? launch_cc2_t<TY, true, true, WST>(c, g, L, it, r)
                      : launch_cc2_t<TY, true, false, WST>(c, g, L, it, r);
    else init ? launch_cc2_t<TY, false, true, WST>(c, g, L, it, r)
              : launch_cc2_t<TY, false, false, WST>(c, g, L, it, r);
}

template <int TY>
static void launch_cc2_ty(hip_proj_ctx* c, const SGeo& g, const Lap& L, int it, bool init,
                          const double* r, bool wst) {
    wst ? launch_cc2_w<TY, true>(c, g, L, it, init, r)
        : launch_cc2_w<TY, false>(c, g, L, it, init, r);
}

// w = A r (stored for k_cc1 when wst) and the iteration's one reduction, over
// the planes of g (c->sgeo: all of them; c->cc2_edge: a slab's edge planes)
static void launch_cc2(hip_proj_ctx* c, const Lap& L, int it, bool init, const double* r,
                       bool wst, const SGeo* gp = nullptr) {
    const SGeo& g = gp ? *gp : c->sgeo;
    if (c->sweep_ty == 16) return launch_cc2_ty<16>(c, g, L, it, init, r, wst);
    if (c->sweep_ty == 4) return launch_cc2_ty<4>(c, g, L, it, init, r, wst);
    return launch_cc2_ty<8>(c, g, L, it, init, r, wst);
}

// k_ccf (ccf.hpp): cg_variant 1's whole iteration in one z-march; r_it is in
// c->r for even it and in c->r2 for odd it
// Z-slabs (NOC): the march stops after r_{it+1} (and p_it, also on the halo
// planes); the r halo and k_cc2 (w = A r in registers, the one reduction)
// follow
static const double* ccf_r0(const hip_proj_ctx* c, int it) { return (it & 1) ? c->r2 : c->r; }
static double* ccf_r1(hip_proj_ctx* c, int it) { return (it & 1) ? c->r : c->r2; }

template <bool FIRST, bool FOLD, bool NOC>
static void launch_ccf_t(hip_proj_ctx* c, const SGeo& g, const Lap& L, double* pn,
                         const double* po, const PPrev& pv, double* x, int it, int xmap,
                         hipStream_t s) {
    // clock sample on one launch in eight while timing (iterations 5 and 7
    // mod 8: a plain and a fold launch)
    unsigned long long* clk = (c->timing && c->clk && (it & 5) == 5) ? c->clk : nullptr;
    hipExtLaunchKernelGGL((k_ccf<FIRST, FOLD, NOC>), dim3(g.tiles_x * g.tiles_y * g.tiles_z),
                          dim3(1024), 0, s, c->ta, c->tb, 0, g, L, ccf_r0(c, it),
                          ccf_r1(c, it), po, pn, pv, x, c->st, c->partials, c->counter, it, xmap,
                          dist(c) ? 1 : 0, c->dsum, mbox(c), clk);
}

template <bool NOC>
static void launch_ccf_n(hip_proj_ctx* c, const SGeo& g, const Lap& L, double* pn,
                         const double* po, const PPrev& pv, double* x, int it, int xmap,
                         hipStream_t s) {
    const bool fold = (it % CG_XFOLD) == CG_XFOLD - 1;
    if (it == 0) launch_ccf_t<true, false, NOC>(c, g, L, pn, po, pv, x, it, xmap, s);
    else if (fold) launch_ccf_t<false, true, NOC>(c, g, L, pn, po, pv, x, it, xmap, s);
    else launch_ccf_t<false, false, NOC>(c, g, L, pn, po, pv, x, it, xmap, s);
}

// g: c->ccgeo (the whole march), or on Z-slabs c->cc_edge / c->cc_int. noc:
// the march stops after r_{it+1} (Z-slab edge planes, or a whole slab of < 3
// planes), else it also forms w and the dot products (one device; a slab's
// interior planes in the fused form)
static void launch_ccf(hip_proj_ctx* c, const SGeo& g, const Lap& L, double* pn,
                       const double* po, const PPrev& pv, double* x, int it, bool noc,
                       hipStream_t s = nullptr) {
    const int xmap = c->env.ccf_xmap;
    if (!s) s = c->stream;
    if (noc) launch_ccf_n<true>(c, g, L, pn, po, pv, x, it, xmap, s);
    else launch_ccf_n<false>(c, g, L, pn, po, pv, x, it, xmap, s);
}

// ---------------------------------------------------------------------------
// pressure solvers on ctx->pn
// ---------------------------------------------------------------------------
enum RhsSource { RHS_FROM_VELOCITY, RHS_FROM_ARRAY };

static cfd_status_t cg_solve(hip_proj_ctx* c, double dx, double dy, double dz,
                             const DivCoef& dc, RhsSource src, double rel_tol, double abs_tol,
                             int max_iter, int check_interval, bool final_bc) {
    const Lap L = make_lap(dx, dy, dz);
    const int G = tile_grid(c);
    const DirVals dv{};
    const bool D = dist(c);
    double* x = c->pn;
    if (c->cg_scratch_dirty) {  // after RK4 stages (rk4_hip.hip): walls of r / p ring to 0
        for (double* f : {c->r, c->pa, c->pb, c->pc4, c->pd4, c->r2})
            if (f) HIP_TRY(hipMemsetAsync(f, 0, field_elems(c) * sizeof(double), c->stream));
        c->cg_scratch_dirty = 0;
    }
    ST_TRY(halo(c, {x}));
    // poisson_solver_apply_bc(x) at solve start (linear_solver_cg.c:320); a
    // caller override runs on the host around the device solve instead
    const bool neumann = (c->poisson_bc == HIP_POISSON_BC_NEUMANN);
    if (neumann) launch_bc(c, x, 0, dv);
    timed(c, HIP_KT_CG_SETUP, [&] {
        const double* rhs_in = (src == RHS_FROM_VELOCITY) ? nullptr : c->rhs;
        if (src == RHS_FROM_VELOCITY) {
            if (D)
                hipExtLaunchKernelGGL((k_cg_setup<true, false, true, true>), dim3(G), dim3(NT), 0,
                                   c->stream, c->ta, c->tb, 0, c->geo, L, dc, c->us, c->vs, c->ws, nullptr, x,
                                   c->r, c->st, c->partials, c->counter, rel_tol, abs_tol,
                                   max_iter, check_interval, c->dsum, mbox(c));
            else
                hipExtLaunchKernelGGL((k_cg_setup<true, false, true, false>), dim3(G), dim3(NT), 0,
                                   c->stream, c->ta, c->tb, 0, c->geo, L, dc, c->us, c->vs, c->ws, nullptr, x,
                                   c->r, c->st, c->partials, c->counter, rel_tol, abs_tol,
                                   max_iter, check_interval, c->dsum, (Mbox*)nullptr);
        } else {
            if (D)
                hipExtLaunchKernelGGL((k_cg_setup<false, false, true, true>), dim3(G), dim3(NT), 0,
                                   c->stream, c->ta, c->tb, 0, c->geo, L, dc, nullptr, nullptr, nullptr,
                                   (double*)rhs_in, x, c->r, c->st, c->partials, c->counter,
                                   rel_tol, abs_tol, max_iter, check_interval, c->dsum, mbox(c));
            else
                hipExtLaunchKernelGGL((k_cg_setup<false, false, true, false>), dim3(G), dim3(NT), 0,
                                   c->stream, c->ta, c->tb, 0, c->geo, L, dc, nullptr, nullptr, nullptr,
                                   (double*)rhs_in, x, c->r, c->st, c->partials, c->counter,
                                   rel_tol, abs_tol, max_iter, check_interval, c->dsum, (Mbox*)nullptr);
        }
    });
    if (D && !mbox(c)) {
        ST_TRY(reduce_dot(c));
        hipExtLaunchKernelGGL(k_finish_setup, dim3(1), dim3(64), 0, c->stream, c->ta, c->tb, 0,
                              c->st, c->dsum + 1, rel_tol, abs_tol, max_iter, check_interval);
    }
    if (D) ST_TRY(halo(c, {c->r}));
    double* P[CG_XFOLD] = {c->pa, c->pb, c->pc4, c->pd4};
    // one CG iteration: sweep A (+ all-reduce of (p,Ap); on slabs A also
    // forms p on the halo planes), sweep B (+ all-reduce of (r,r), halo of r)
    auto iterate = [&](int it) -> cfd_status_t {
        double* pnew = P[it % CG_XFOLD];
        double* pold = P[(it + CG_XFOLD - 1) % CG_XFOLD];
        // x += alpha_j p_j of iterations it-4 .. it-1, folded by sweep A
        const bool fold = it > 0 && (it % CG_XFOLD) == 0;
        const PFold fd{P[(it + 1) % CG_XFOLD], P[(it + 2) % CG_XFOLD], fold ? x : nullptr};
        const BArgs ba{pnew, c->r};
        const int kb = HIP_KT_CG_SWEEP_B;
        const int ka = fold ? HIP_KT_CG_SWEEP_BX : HIP_KT_CG_SWEEP_A;
        timed(c, ka, [&] { launch_cgA(c, it == 0, L, c->r, pold, pnew, it, fd); }, it);
        if (D && !mbox(c)) {
            ST_TRY(timed_span(c, c->stream, HIP_KT_ALLREDUCE, [&] {
                ST_TRY(reduce_dot(c));
                hipLaunchKernelGGL(k_finish_A, dim3(1), dim3(64), 0, c->stream, c->st,
                                   c->dsum + 1, it, fold ? 1 : 0);
                return CFD_SUCCESS;
            }, it));
        }
        if (!D) timed(c, kb, [&] { launch_cgB(c, c->sgeo, L, ba, it); }, it);
        if (D) {
            // r's halo goes out on the side stream (halo communicator) as soon
            // as the two slab-edge planes of the new r exist: sweep B runs them
            // first, then the interior planes overlap the exchange; the (r,r)
            // all-reduce follows on the main stream; the next sweep A waits
            // for both
            if (c->split_b) launch_cgB(c, c->sg_edge, L, ba, it);
            else timed(c, kb, [&] { launch_cgB(c, c->sgeo, L, ba, it); }, it);
            HIP_TRY(hipEventRecord(c->ev_b, c->stream));
            HIP_TRY(hipStreamWaitEvent(c->hstream, c->ev_b, 0));
            double* rr[1] = {c->r};
            ST_TRY(timed_span(c, c->hstream, HIP_KT_HALO, [&] {
                return c->comm->halo(c->hstream, rr, 1, c->ps, (int)c->nz, false);
            }, it));
            HIP_TRY(hipEventRecord(c->ev_h, c->hstream));
            if (c->split_b) timed(c, kb, [&] { launch_cgB(c, c->sg_int, L, ba, it); }, it);
            if (!mbox(c)) {
                ST_TRY(timed_span(c, c->stream, HIP_KT_ALLREDUCE, [&] {
                    ST_TRY(reduce_dot(c));
                    hipLaunchKernelGGL(k_finish_B, dim3(1), dim3(64), 0, c->stream, c->st,
                                       c->dsum + 1, it);
                    return CFD_SUCCESS;
                }, it));
            }
            HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_h, 0));
        }
        return CFD_SUCCESS;
    };
    // Chronopoulos-Gear (cg_variant 1): k_cc1 (pointwise) -> halo of r ->
    // k_cc2 (w = A r and both dots, ONE reduction / all-reduce)
    const bool cc = (c->cfg.cg_variant == 1);
    // 3-D: the fused iteration (k_ccf; on Z-slabs + the r halo + k_cc2);
    // CFD_HIP_CCF = 0 keeps k_cc1 + k_cc2 (c->env: read at context creation)
    const bool ccf = cc && c->ccgeo.tiles_x > 0 && !c->env.ccf_off;
    auto reduce_cc = [&](int it, bool init) -> cfd_status_t {
        if (!D || mbox(c)) return CFD_SUCCESS;
        return timed_span(c, c->stream, HIP_KT_ALLREDUCE, [&] {
            ST_TRY(c->comm->allreduce_sum(c->stream, c->dsum, c->dsum + 2, 2));
            hipLaunchKernelGGL(k_finish_cc, dim3(1), dim3(64), 0, c->stream, c->st, c->dsum + 2,
                               it, (it % CG_XFOLD) == CG_XFOLD - 1 ? 1 : 0, init ? 1 : 0);
            return CFD_SUCCESS;
        }, it);
    };
    auto iterate_cc = [&](int it) -> cfd_status_t {
        double* pnew = P[it % CG_XFOLD];
        double* pold = P[(it + CG_XFOLD - 1) % CG_XFOLD];
        PPrev pv;
        for (int q = 0; q < CG_XFOLD - 1; ++q) pv.q[q] = P[(it + 1 + q) % CG_XFOLD];
        // the fold launches (x += the four pending alpha p, every 4th) time
        // apart from the plain ones
        const int kcf = (it > 0 && (it % CG_XFOLD) == CG_XFOLD - 1) ? HIP_KT_CC_FOLD
                                                                     : HIP_KT_CC_FUSED;
        if (ccf && !D) {
            timed(c, kcf,
                  [&] { launch_ccf(c, c->ccgeo, L, pnew, pold, pv, x, it, false); }, it);
            return CFD_SUCCESS;
        }
        if (ccf) {
            // Z-slabs: r_{it+1} on the two edge planes first; its halo then
            // travels on the side stream (halo communicator) while the march
            // covers the interior planes; the SpMV + reduction wait for it.
            // Fused form (default): the interior march also forms w and the
            // dot products of planes k0 + 1 .. k1 - 2, so k_cc2 covers only the
            // two edge planes (whose w needs the neighbours' r) and completes
            // the shared reduction; CFD_HIP_CCF_SLAB_FUSED=0: k_cc2 over every
            // plane (r04)
            double* r1 = ccf_r1(c, it);
            if (c->cc_edge.tiles_x > 0) {
                const bool fused = c->cc2_edge.tiles_x > 0;
                if (c->env.ccf_edge_side) {
                    // r06: the edge planes' march runs on the side stream,
                    // beside the interior march instead of before it: the
                    // two read only r_it and p_{it-1} and write disjoint
                    // planes of p_it, r_{it+1} and x (the interior march
                    // forms the edge planes' r_{it+1} it needs itself), so
                    // only the halo waits for the edge launch. The side
                    // stream first waits for the main stream (the previous
                    // iteration's reduction: alpha, beta)
                    HIP_TRY(hipEventRecord(c->ev_b, c->stream));
                    HIP_TRY(hipStreamWaitEvent(c->hstream, c->ev_b, 0));
                    launch_ccf(c, c->cc_edge, L, pnew, pold, pv, x, it, true, c->hstream);
                } else {
                    launch_ccf(c, c->cc_edge, L, pnew, pold, pv, x, it, true);
                    HIP_TRY(hipEventRecord(c->ev_b, c->stream));
                    HIP_TRY(hipStreamWaitEvent(c->hstream, c->ev_b, 0));
                }
                double* rr[1] = {r1};
                ST_TRY(timed_span(c, c->hstream, HIP_KT_HALO, [&] {
                    return c->comm->halo(c->hstream, rr, 1, c->ps, (int)c->nz, false);
                }, it));
                HIP_TRY(hipEventRecord(c->ev_h, c->hstream));
                timed(c, kcf,
                      [&] { launch_ccf(c, fused ? c->cc_int_red : c->cc_int, L, pnew, pold, pv,
                                       x, it, !fused); }, it);
                HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_h, 0));
                timed(c, HIP_KT_CC_SPMV, [&] {
                    launch_cc2(c, L, it, false, r1, false, fused ? &c->cc2_edge : nullptr);
                }, it);
            } else {
                timed(c, kcf,
                      [&] { launch_ccf(c, c->ccgeo, L, pnew, pold, pv, x, it, true); }, it);
                ST_TRY(timed_span(c, c->stream, HIP_KT_HALO, [&] { return halo(c, {r1}); }, it));
                timed(c, HIP_KT_CC_SPMV, [&] { launch_cc2(c, L, it, false, r1, false); }, it);
            }
            return reduce_cc(it, false);
        }
        timed(c, HIP_KT_CC_UPDATE, [&] { launch_cc1(c, pnew, pold, pv, x, it); }, it);
        if (D)
            ST_TRY(timed_span(c, c->stream, HIP_KT_HALO,
                              [&] { return halo(c, {c->r}); }, it));
        timed(c, HIP_KT_CC_SPMV, [&] { launch_cc2(c, L, it, false, c->r, true); }, it);
        return reduce_cc(it, false);
    };
    if (cc) {
        const size_t n = field_elems(c);
        if (!ccf && !c->cw) ST_TRY(dalloc(c, &c->cw, n));
        if (!ccf && !c->cs) ST_TRY(dalloc(c, &c->cs, n));
        if (ccf && !c->r2) ST_TRY(dalloc(c, &c->r2, n));
        // w_0 = A r_0 and alpha_0 (the textbook's first (p, Ap) with p_0 =
        // r_0); the fused iteration needs no stored w
        timed(c, HIP_KT_CC_SPMV, [&] { launch_cc2(c, L, -1, true, c->r, !ccf); });
        ST_TRY(reduce_cc(-1, true));
    }
    auto step_it = [&](int it) { return cc ? iterate_cc(it) : iterate(it); };
    // small grids: the whole solve in one cooperative launch (k_cg_small);
    // CFD_HIP_CG_SMALL = 0 never, 1 up to 64 x 256 x 16 interior cells,
    // default up to CG_SMALL_CELLS
    bool small_done = false;
    const long long ncell = (long long)(c->nx - 2) * (long long)(c->ny - 2) *
                            (long long)(c->geo.k1 - c->geo.k0);
    {
        const int mode = c->env.cg_small;
        const long long cap = (mode == 1) ? (long long)CGS_MAX_WG * CGS_THREADS * 16
                                          : (mode == 0 ? 0 : CG_SMALL_CELLS);
        if (!D && !cc && max_iter > 0 && ncell > 0 && ncell <= cap) {
            int rate_khz = 0;
            hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, c->device);
            long long ticks = (long long)std::max(rate_khz, 1000) * 1000LL * 20;  // 20 s
            unsigned nbw = (unsigned)std::min<long long>(
                CGS_MAX_WG, (ncell + CGS_THREADS - 1) / CGS_THREADS);
            Geo geo = c->geo;
            Lap lap = L;
            double* xx = x;
            unsigned* barp = c->counter + 8;
            void* args[] = {&geo, &lap, &xx, &c->r, &c->pa, &c->pb, &c->st, &c->partials,
                            &barp, &ticks};
            ST_TRY(timed_span(c, c->stream, HIP_KT_CG_SMALL, [&]() -> cfd_status_t {
                HIP_TRY(hipMemsetAsync(barp, 0, sizeof(unsigned), c->stream));
                if (hipLaunchCooperativeKernel((const void*)k_cg_small, dim3(nbw),
                                               dim3(CGS_THREADS), args, 0,
                                               c->stream) == hipSuccess)
                    small_done = true;
                else
                    (void)hipGetLastError();  // not co-resident here: the sweep loop
                return CFD_SUCCESS;
            }));
        }
    }
    int it = 0;
    if (max_iter > 0 && !small_done) {
        ST_TRY(step_it(0));
        it = 1;
    }
    // Host polls a pinned copy of the device state once per chunk, one chunk
    // behind (double-buffered), so the stream never drains while it waits.
    // Every rank sees the same all-reduced state and leaves at the same chunk.
    int chunk = 8;
    const int chunk_max = std::max(1, c->cfg.poll_interval);
    int slot = 0, prev = -1;
    while (it < max_iter && !small_done) {
        const int n = std::min(chunk, max_iter - it);
        for (int q = 0; q < n; ++q, ++it) ST_TRY(step_it(it));
        HIP_TRY(hipMemcpyAsync(&c->h_state[slot], c->st, sizeof(CgState), hipMemcpyDeviceToHost,
                               c->stream));
        HIP_TRY(hipEventRecord(c->ev_poll[slot], c->stream));
        if (prev >= 0) {
            HIP_TRY(hipEventSynchronize(c->ev_poll[prev]));
            if (c->h_state[prev].done) break;
        }
        prev = slot;
        slot ^= 1;
        chunk = std::min(chunk * 2, chunk_max);
    }
    PRing pr;
    for (int q = 0; q < CG_XFOLD; ++q) pr.p[q] = P[q];
    hipExtLaunchKernelGGL(k_cg_finalize, dim3(G), dim3(NT), 0, c->stream, c->ta, c->tb, 0, c->geo, pr, x,
                       c->st);
    HIP_TRY(hipMemcpyAsync(&c->h_state[2], c->st, sizeof(CgState), hipMemcpyDeviceToHost,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const CgState& s = c->h_state[2];
    flush_timing(c, s.iterations);
    if (s.status == ST_COMM_TIMEOUT) {
        set_err(CFD_ERROR, small_done
                               ? "projection_hip: small-grid CG grid barrier timed out"
                               : "projection_hip: slab all-reduce timed out (a rank stopped)");
        return CFD_ERROR;
    }
    const bool stagnated = (s.status == ST_STAGNATED);
    // final poisson_solver_apply_bc (cg.c:447); the breakdown exit skips it.
    if (final_bc && neumann && !stagnated && !(s.iterations == 0 && s.status == ST_CONVERGED))
        launch_bc(c, x, 0, dv);
    ST_TRY(halo(c, {x}));
    c->pstats.status = (poisson_solver_status_t)s.status;
    c->pstats.iterations = s.iterations;
    c->pstats.initial_residual = s.res0;
    c->pstats.final_residual = s.res;
    return (s.status == ST_CONVERGED) ? CFD_SUCCESS : CFD_ERROR_MAX_ITER;
}

static double optimal_omega(size_t nx, size_t ny, size_t nz, double dx, double dy, double dz) {
    // linear_solver_internal.h:184-220
    double inv_dx2 = 1.0 / (dx * dx), inv_dy2 = 1.0 / (dy * dy);
    double inv_dz2 = (dz > 0.0) ? (1.0 / (dz * dz)) : 0.0;
    double num = cos(M_PI / (double)(nx - 1)) * inv_dx2 + cos(M_PI / (double)(ny - 1)) * inv_dy2;
    double den = inv_dx2 + inv_dy2;
    if (nz > 1 && inv_dz2 > 0.0) {
        num += cos(M_PI / (double)(nz - 1)) * inv_dz2;
        den += inv_dz2;
    }
    double rj = num / den;
    return 2.0 / (1.0 + sqrt(1.0 - (rj * rj)));
}

static cfd_status_t residual_linf(hip_proj_ctx* c, const double* x, const ResCoef& rc, double* out) {
    const int G = tile_grid(c);
    hipExtLaunchKernelGGL(k_init_red, dim3(1), dim3(64), 0, c->stream, c->ta, c->tb, 0, c->red);
    timed(c, HIP_KT_RESIDUAL, [&] {
        hipExtLaunchKernelGGL(k_residual_linf, dim3(G), dim3(NT), 0, c->stream, c->ta, c->tb, 0, c->geo, rc, x, c->rhs,
                           c->red + 4);
    });
    cfd_status_t st;
    const unsigned long long* red = reduce_red(c, &st);
    if (st != CFD_SUCCESS) return st;
    HIP_TRY(hipMemcpyAsync(c->h_red, red, 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    *out = ord_dec(c->h_red[4]);
    return CFD_SUCCESS;
}

static cfd_status_t ensure_aux(hip_proj_ctx* c, bool need_rhs, bool need_xt);
static_assert(sizeof(RxState) <= sizeof(CgState), "RxState polls through the CgState slots");

// One k_rb1 sweep on one device (3-D): xi -> xo (one RB-SOR iteration with
// its Neumann shell when neu_fold), the L-inf residual of xi decided on `st`
// as sweep `it` of the fused loop.
static void rb1_sweep_single(hip_proj_ctx* c, const RelaxCoef& rc, const double* xi, double* xo,
                             int it, RxState* st, bool neu_fold) {
    constexpr int FLR = SW_NT_STORE | SW_PREFETCH | SW_EDGE1;
    const unsigned nb1 = (unsigned)(c->rgeo.tiles_x * c->rgeo.tiles_y * c->rgeo.tiles_z);
    // register-ring prefetch (default); CFD_HIP_RB1_PF=0 selects the
    // end-of-step loads (experiments)
    const bool rb1_pf = c->env.rb1_pf;
    // memory hints of k_rb1 / k_rb1m (SW_* bits): FLR = 13, NT stores
    // of Y and plain rhs loads (r03: the NT rhs loads of 15 made the
    // neighbouring tiles re-fetch the rhs halo rows; 512^3 0.744 ->
    // 0.726 ms, 1024^2 x 512 2.925 -> 2.85 ms, fetch 19.6 -> 18.7
    // B/cell, profiles/r03_rbfl.jsonl)
    // odd iterations march z downwards (REV), so each sweep starts on
    // the planes the previous one wrote last, in the Infinity Cache;
    // bitwise either way (kernels.hpp rb1_body). CFD_HIP_RB1_ALT=0:
    // every iteration upwards
    const bool rev = c->env.rb1_alt && rb1_pf && (it & 1);
#define RB1_LAUNCH(TCV, PFV)                                                                   \
    hipExtLaunchKernelGGL((k_rb1<FLR, TCV, PFV>), dim3(nb1), dim3(1024), 0, c->stream, c->ta, \
                          c->tb, 0, c->rgeo, rc, xi, xo, c->rhs, st, c->partials,            \
                          c->counter, it, (const double*)nullptr, 0, 0, (Mbox*)nullptr,      \
                          (unsigned long long*)nullptr, neu_fold ? 1 : 0)
    if (c->rb_strip_tc && rb1_pf) {
        // full-width tiles and the narrow strip in one grid
        const SGeo& gm = c->rg_main;
        const SGeo& gs = c->rg_strip;
        const int nbm = gm.tiles_x * gm.tiles_y * gm.tiles_z;
        const unsigned nbt = (unsigned)(nbm + gs.tiles_x * gs.tiles_y * gs.tiles_z);
        timed(c, HIP_KT_RELAX, [&] {
            auto go = [&](auto kern) {
                hipExtLaunchKernelGGL(kern, dim3(nbt), dim3(1024), 0, c->stream, c->ta,
                                      c->tb, 0, gm, gs, nbm, rc, xi, xo, c->rhs, st,
                                      c->partials, c->counter, it, neu_fold ? 1 : 0);
            };
            if (rev) go(k_rb1m<FLR, 16, true>);
            else go(k_rb1m<FLR, 16>);
        }, it);
    } else
    timed(c, HIP_KT_RELAX, [&] {
        if (!rb1_pf) RB1_LAUNCH(64, false);
        else if (c->rb1_tc == 32) RB1_LAUNCH(32, true);
        else if (c->rb1_tc == 16) RB1_LAUNCH(16, true);
        else if (rev)
            hipExtLaunchKernelGGL((k_rb1<FLR, 64, true, false, true>), dim3(nb1),
                                  dim3(1024), 0, c->stream, c->ta, c->tb, 0, c->rgeo, rc,
                                  xi, xo, c->rhs, st, c->partials, c->counter, it,
                                  (const double*)nullptr, 0, 0, (Mbox*)nullptr,
                                  (unsigned long long*)nullptr, neu_fold ? 1 : 0);
        else RB1_LAUNCH(64, true);
    });
#undef RB1_LAUNCH
}


// Two RB-SOR iterations per sweep (k_rb2, rb2.hpp) on one device in 3-D with
// the Neumann shell, check_interval 1 (the reference default): the fused
// loop of relax_solve_fused with sweep 0 a k_rb1 sweep (the exact initial
// residual), then k_rb2 sweeps s = 1, 3, 5, ... (iterate s -> s + 2, the
// decisions on iterates s and s + 1). The host logs every launch (iterate,
// kind, buffers), so after the loop stops it finds the decided iterate: the
// input of a launch (intact) or the middle iterate of a k_rb2 sweep, which it
// recomputes with one k_rb1 sweep from that sweep's input. With apx (the
// product form) the device may also stop on
//  - ST_RB2_AMBIG (an approximate residual within its bound of the
//    threshold): the host computes that iterate's exact residual and resumes
//    the loop from the iterate with it as an override;
//  - ST_RB2_UNCERT (a value outside the certified range): the host resumes
//    from that sweep's input with k_rb1 sweeps for the rest of the solve;
// and the final residual is recomputed exactly. Iterates, iteration counts,
// statuses and residuals are those of relax_solve_fused.
static cfd_status_t relax_solve_rb2(hip_proj_ctx* c, const RelaxCoef& rc, double rel_tol,
                                    double abs_tol, int max_iter, bool apx) {
    ST_TRY(ensure_aux(c, true, true));
    if (!c->rxst) HIP_TRY(hipMalloc((void**)&c->rxst, sizeof(RxState)));
    if (!c->rxst2) HIP_TRY(hipMalloc((void**)&c->rxst2, sizeof(RxState)));
    if (!c->rb2dec) HIP_TRY(hipMalloc((void**)&c->rb2dec, sizeof(Rb2Dec)));
    Rb2Coef cf;
    cf.rc = rc;
    cf.k2 = 2.0 * (rc.rdx2 + rc.rdy2 + rc.inv_dz2);
    cf.slow = 0x1p-900;
    cf.nif = -rc.inv_factor;
    double escale = 1.0, mlim = 0x1p800;
    if (c->env.rb2_test) {  // tests: force the host paths
        const int v = c->env.rb2_test;
        if (v == 1) escale = 1e300;  // every approximate decision ambiguous
        if (v == 2) mlim = 0.0;      // every sweep uncertified
        if (v == 3) cf.slow = 1e300; // every SOR update in the reference's arithmetic
    }
    hipExtLaunchKernelGGL(k_rb2_dec_init, dim3(1), dim3(64), 0, c->stream, c->ta, c->tb, 0,
                          (Rb2Dec*)c->rb2dec, rc.rdx2 + rc.rdy2 + rc.inv_dz2, escale, mlim);
    // the fast division's range argument (rb2.hpp rb2_sorc) needs 1 <= 1/d^2 <= 2^60
    if (!(rc.rdx2 >= 1.0 && rc.rdy2 >= 1.0 && rc.rdx2 <= 0x1p60 && rc.rdy2 <= 0x1p60))
        apx = false;
    constexpr int FLR = SW_NT_STORE | SW_PREFETCH | SW_EDGE1;
    const SGeo& g2 = c->r2geo;
    const int xmap = c->env.rb2_xmap;
    const unsigned nb2 = (unsigned)(g2.tiles_x * g2.tiles_y * g2.tiles_z);
    hipExtLaunchKernelGGL(k_rx_init, dim3(1), dim3(64), 0, c->stream, c->ta, c->tb, 0, c->rxst,
                          rel_tol, abs_tol, max_iter, 1);
    if (apx) {
        const int nbm = (int)std::min<long long>(4LL * c->grid_cap,
                                                 ((long long)c->nx * c->ny * c->nz + 255) / 256);
        hipExtLaunchKernelGGL(k_rb2_bmax, dim3(std::max(1, nbm)), dim3(256), 0, c->stream,
                              c->ta, c->tb, 0, c->geo, (const double*)c->rhs, c->rxst);
    }
    struct Launch {
        int s, kind;  // kind 1: k_rb1 (iterate s -> s + 1), 2: k_rb2 (s -> s + 2)
        double *x, *y;
    };
    std::vector<Launch> log;
    double* bx = c->pn;
    double* by = c->xt;
    int cur = 0;
    bool exact_mode = false, force_certx = false;
    int n_ambig = 0, n_uncert = 0;
    auto launch = [&]() {
        if (cur == 0 || exact_mode) {
            rb1_sweep_single(c, rc, bx, by, cur, c->rxst, true);
            log.push_back({cur, 1, bx, by});
            cur += 1;
        } else {
            const int certx = (force_certx || log.empty() || log.back().kind == 1) ? 1 : 0;
            force_certx = false;
            if (apx && certx) {  // X's own values: max |X| for the sweep's range test
                // (an error here is sticky: the loop's next HIP_TRY reports it)
                (void)hipMemsetAsync(&c->rxst->xmax, 0, sizeof(double), c->stream);
                const int nbm = (int)std::min<long long>(
                    4LL * c->grid_cap, ((long long)c->nx * c->ny * c->nz + 255) / 256);
                hipExtLaunchKernelGGL(k_rb2_xmax, dim3(std::max(1, nbm)), dim3(256), 0,
                                      c->stream, c->ta, c->tb, 0, c->geo, (const double*)bx,
                                      c->rxst);
            }
            timed(c, HIP_KT_RELAX2, [&] {
                if (apx)
                    hipExtLaunchKernelGGL((k_rb2<true, FLR>), dim3(nb2), dim3(1024), 0, c->stream,
                                          c->ta, c->tb, 0, g2, cf, (const double*)bx, by,
                                          (const double*)c->rhs, c->rxst, c->partials,
                                          c->counter, cur, certx, xmap,
                                          (const Rb2Dec*)c->rb2dec);
                else
                    hipExtLaunchKernelGGL((k_rb2<false, FLR>), dim3(nb2), dim3(1024), 0,
                                          c->stream, c->ta, c->tb, 0, g2, cf, (const double*)bx,
                                          by, (const double*)c->rhs, c->rxst, c->partials,
                                          c->counter, cur, certx, xmap,
                                          (const Rb2Dec*)c->rb2dec);
            }, cur);
            log.push_back({cur, 2, bx, by});
            cur += 2;
        }
        std::swap(bx, by);
    };
    // the middle iterate of k_rb2 launch L, recomputed into L.y (one k_rb1
    // sweep on a scratch state that never decides)
    auto recompute_mid = [&](const Launch& L) {
        hipExtLaunchKernelGGL(k_rx_init, dim3(1), dim3(64), 0, c->stream, c->ta, c->tb, 0,
                              c->rxst2, 0.0, 0.0, 0x7fffffff, 1);
        rb1_sweep_single(c, rc, L.x, L.y, 1, c->rxst2, true);
    };
    auto find = [&](int t, int* kind_mid) -> int {  // log index holding iterate t
        for (int q = (int)log.size() - 1; q >= 0; --q) {
            if (log[q].s == t) {
                *kind_mid = 0;
                return q;
            }
            if (log[q].kind == 2 && log[q].s + 1 == t) {
                *kind_mid = 1;
                return q;
            }
        }
        return -1;
    };
    const ResCoef resc{rc.dx2, rc.dy2, rc.inv_dz2};
    static_assert(sizeof(RxState) <= sizeof(CgState), "h_state holds RxState copies");
    RxState* hs = reinterpret_cast<RxState*>(c->h_state);
    for (;;) {
        int chunk = 8, slot = 0, prev = -1;
        const int chunk_max = std::max(1, c->cfg.poll_interval);
        while (cur <= max_iter) {
            const int target = cur + chunk;  // iterates launched this chunk
            while (cur <= max_iter && cur < target) launch();
            HIP_TRY(hipMemcpyAsync(&hs[slot], c->rxst, sizeof(RxState), hipMemcpyDeviceToHost,
                                   c->stream));
            HIP_TRY(hipEventRecord(c->ev_poll[slot], c->stream));
            if (prev >= 0) {
                HIP_TRY(hipEventSynchronize(c->ev_poll[prev]));
                if (hs[prev].done) break;
            }
            prev = slot;
            slot ^= 1;
            chunk = std::min(chunk * 2, chunk_max);
        }
        HIP_TRY(hipMemcpyAsync(&hs[2], c->rxst, sizeof(RxState), hipMemcpyDeviceToHost,
                               c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        const RxState r = hs[2];
        if (!r.done) {
            set_err(CFD_ERROR, "relaxation (k_rb2): device loop ended without a decision");
            return CFD_ERROR;
        }
        int mid = 0;
        const int li = find(r.res_it, &mid);
        if (li < 0) {
            set_err(CFD_ERROR, "relaxation (k_rb2): decided iterate not in the launch log");
            return CFD_ERROR;
        }
        const Launch L = log[li];
        if (r.status == ST_RB2_UNCERT) {
            ++n_uncert;
            // rerun from this sweep's input with k_rb1 sweeps
            log.resize(li);
            exact_mode = true;
            bx = L.x;
            by = L.y;
            cur = L.s;
            hipExtLaunchKernelGGL(k_rb2_resume, dim3(1), dim3(64), 0, c->stream, c->ta, c->tb,
                                  0, c->rxst, -1, 0.0);
            continue;
        }
        double* xt = mid ? L.y : L.x;
        if (mid) recompute_mid(L);
        if (r.status == ST_RB2_AMBIG) {
            ++n_ambig;
            double m = 0.0;
            ST_TRY(residual_linf(c, xt, resc, &m));
            log.resize(li);
            force_certx = true;  // the next sweep's input came from a recompute
            bx = xt;
            by = mid ? L.x : L.y;
            cur = r.res_it;
            hipExtLaunchKernelGGL(k_rb2_resume, dim3(1), dim3(64), 0, c->stream, c->ta, c->tb,
                                  0, c->rxst, r.res_it, m);
            continue;
        }
        flush_timing(c);
        double res = r.res;
        if (!r.res_exact) ST_TRY(residual_linf(c, xt, resc, &res));
        if (c->env.rb2_log) {  // diagnostics: the loop's launches and stops
            int n1 = 0, n2 = 0;
            for (const Launch& q : log) (q.kind == 1 ? n1 : n2)++;
            fprintf(stderr, "rb2: iterations %d status %d, k_rb1 %d k_rb2 %d launches, "
                    "%d ambiguous, %d uncertified, res_it %d\n", r.iterations, r.status, n1, n2,
                    n_ambig, n_uncert, r.res_it);
        }
        if (xt != c->pn) std::swap(c->pn, c->xt);
        c->pstats.initial_residual = r.res0;
        c->pstats.iterations = r.iterations;
        c->pstats.final_residual = res;
        c->pstats.status = (poisson_solver_status_t)r.status;
        return (r.status == ST_CONVERGED) ? CFD_SUCCESS : CFD_ERROR_MAX_ITER;
    }
}

// Fused relaxation loop (single device, 16-row sweep tiles): the iteration's
// sweeps, boundary shell and convergence test all run on the device (k_rx,
// kernels.hpp); the host polls the state one chunk behind, like cg_solve.
// Same iterates, residuals, iteration counts and statuses as relax_solve's
// two-pass form below.
static cfd_status_t relax_solve_fused(hip_proj_ctx* c, int method, const RelaxCoef& rc,
                                      double rel_tol, double abs_tol, int max_iter,
                                      int check_interval) {
    ST_TRY(ensure_aux(c, true, true));
    if (!c->rxst) HIP_TRY(hipMalloc((void**)&c->rxst, sizeof(RxState)));
    double* X[2] = {c->pn, c->xt};
    const bool D = dist(c);
    Mbox* mb = mbox(c);
    // Z-slabs without a device mailbox: residual max through RCCL (red[6] -> redg[6])
    unsigned long long* dred = c->red + 6;
    unsigned long long* gred = D ? c->redg + 6 : nullptr;
    const unsigned nb = (unsigned)sweep_grid(c);
    const unsigned TH = 64u * (unsigned)c->sweep_ty;
    constexpr int FL = SW_NT_STORE | SW_NT_LOAD | SW_PREFETCH | SW_EDGE1;
    // k_rb1: plain rhs loads (its tiles' rhs halo rows are re-read by the
    // neighbouring tile; see the one-device launch below)
    constexpr int FLR = SW_NT_STORE | SW_PREFETCH | SW_EDGE1;
    auto sweep = [&](int mode, const double* xi, double* xo, int it) {
        timed(c, HIP_KT_RELAX, [&] {
#define RX_LAUNCH(TYV, M, DV)                                                                  \
    hipExtLaunchKernelGGL((k_rx<TYV, M, FL, DV>), dim3(nb), dim3(TH), 0, c->stream, c->ta,     \
                          c->tb, 0, c->sgeo, rc, xi, xo, c->rhs, c->rxst, c->partials,        \
                          c->counter, it, mb, dred)
#define RX_MODES(TYV, DV)                                 \
    if (mode == RX_RED) RX_LAUNCH(TYV, RX_RED, DV);       \
    else if (mode == RX_BLACK) RX_LAUNCH(TYV, RX_BLACK, DV); \
    else RX_LAUNCH(TYV, RX_JACOBI, DV)
            if (c->sweep_ty == 16) {
                if (D) { RX_MODES(16, true); } else { RX_MODES(16, false); }
            } else {
                if (D) { RX_MODES(8, true); } else { RX_MODES(8, false); }
            }
#undef RX_MODES
#undef RX_LAUNCH
        });
    };
    // the residual sweep's all-ranks max when there is no device mailbox
    auto finish = [&](int it) -> cfd_status_t {
        if (!D || mb) return CFD_SUCCESS;
        ST_TRY(c->comm->allreduce_max_u64(c->stream, dred, gred, 1));
        hipExtLaunchKernelGGL(k_rx_finish, dim3(1), dim3(64), 0, c->stream, c->ta, c->tb, 0,
                              c->rxst, gred, it);
        return CFD_SUCCESS;
    };
    // one-pass RB-SOR (k_rb1) on a single device in 3-D; relax_two_pass = 2
    // forces the two colour sweeps of k_rx
    // one-pass RB-SOR (k_rb1) in 3-D, on one device or on Z-slabs (there with
    // the edge planes' R exchanged first); relax_two_pass = 2 forces the two
    // colour sweeps of k_rx
    const bool single = method == HIP_POISSON_REDBLACK && c->nz > 1 &&
                        c->cfg.relax_two_pass == 0;
    // k_rb1 writes the iteration's Neumann shell itself (no k_rx_shell);
    // CFD_HIP_RB1_FOLD=0 keeps the separate shell launch (A/B)
    const bool neu_fold = single && c->env.rb1_fold && c->poisson_bc == HIP_POISSON_BC_NEUMANN;
    // two iterations per sweep on one device (rb2.hpp): CFD_HIP_RB2 = 1 (the
    // default: certified fast arithmetic), 2 (the reference's arithmetic
    // throughout), 0 (one iteration per sweep, k_rb1)
    const int rb2_env = c->env.rb2;
    if (neu_fold && !D && check_interval == 1 && rb2_env != 0 && c->r2geo.tiles_x > 0)
        return relax_solve_rb2(c, rc, rel_tol, abs_tol, max_iter, rb2_env != 2);
    ST_TRY(halo(c, {c->pn}));
    hipExtLaunchKernelGGL(k_rx_init, dim3(1), dim3(64), 0, c->stream, c->ta, c->tb, 0, c->rxst,
                          rel_tol, abs_tol, max_iter, check_interval);
    // Halo exchanges are host-launched and run even after the device decided
    // to stop; they then copy the neighbours' final owned planes into the
    // result's halo planes, which is what they hold anyway.
    auto iterate = [&](int it) -> cfd_status_t {
        double* xi = X[it & 1];
        double* xo = X[(it + 1) & 1];
        if (single && D) {
            // R of the own edge planes -> the neighbours' halo planes of RH
            // (the CG residual array, free during a relaxation solve), then
            // the one-pass sweep with R on the halo planes taken from RH
            double* RH = c->r;
            c->cg_scratch_dirty = 1;
            const long long plane = (long long)c->nx * (long long)c->ny;
            const unsigned ne = (unsigned)std::min<long long>((2 * plane + 255) / 256,
                                                              (long long)c->grid_cap * 4);
            timed(c, HIP_KT_RELAX, [&] {
                hipExtLaunchKernelGGL(k_rb_edge_r, dim3(ne), dim3(256), 0, c->stream, c->ta,
                                      c->tb, 0, c->rgeo, rc, xi, c->rhs, RH);
            }, it);
            auto rb1 = [&](const SGeo& sg) {
                const unsigned nbx = (unsigned)(sg.tiles_x * sg.tiles_y * sg.tiles_z);
                timed(c, HIP_KT_RELAX, [&] {
                    hipExtLaunchKernelGGL((k_rb1<FLR, 64, true, true>), dim3(nbx), dim3(1024), 0,
                                          c->stream, c->ta, c->tb, 0, sg, rc, xi, xo, c->rhs,
                                          c->rxst, c->partials, c->counter, it, (const double*)RH,
                                          c->geo.lo_face ? 0 : 1, c->geo.hi_face ? 0 : 1, mb,
                                          dred, neu_fold ? 1 : 0);
                }, it);
            };
            // exchange of `f`'s edge planes on the side stream (halo
            // communicator), ordered after the main stream's work so far
            auto side_halo = [&](double* f) -> cfd_status_t {
                HIP_TRY(hipEventRecord(c->ev_b, c->stream));
                HIP_TRY(hipStreamWaitEvent(c->hstream, c->ev_b, 0));
                double* ff[1] = {f};
                ST_TRY(timed_span(c, c->hstream, HIP_KT_HALO, [&] {
                    return c->comm->halo(c->hstream, ff, 1, c->ps, (int)c->nz, false);
                }, it));
                HIP_TRY(hipEventRecord(c->ev_h, c->hstream));
                return CFD_SUCCESS;
            };
            if (c->split_rb) {
                // R's edge planes travel while interior part 1 (which needs no
                // halo R) runs; the edge planes of Y follow, and their exchange
                // overlaps interior part 2 and the residual's all-reduce. The
                // three launches write disjoint planes of Y and share one
                // L-inf reduction, so Y and the decision are the one-launch ones.
                ST_TRY(side_halo(RH));
                rb1(c->rg_in1);
                HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_h, 0));
                rb1(c->rg_edge);
                ST_TRY(side_halo(xo));
                rb1(c->rg_in2);
                if (!mb)
                    ST_TRY(timed_span(c, c->stream, HIP_KT_ALLREDUCE, [&] { return finish(it); },
                                      it));
                HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_h, 0));
            } else {
                // same collective order as the split form (R halo, Y halo,
                // residual max): the in-process group pairs its ranks' calls
                // by order, and a slab of < 4 planes runs this form beside
                // split neighbours
                ST_TRY(timed_span(c, c->stream, HIP_KT_HALO, [&] { return halo(c, {RH}); }, it));
                rb1(c->rgeo);
                ST_TRY(timed_span(c, c->stream, HIP_KT_HALO, [&] { return halo(c, {xo}); }, it));
                if (!mb)
                    ST_TRY(timed_span(c, c->stream, HIP_KT_ALLREDUCE, [&] { return finish(it); },
                                      it));
            }
        } else if (single) {
            rb1_sweep_single(c, rc, xi, xo, it, c->rxst, neu_fold);
        } else if (method == HIP_POISSON_REDBLACK) {
            sweep(RX_RED, xi, xo, it);
            ST_TRY(finish(it));
            hipExtLaunchKernelGGL(k_rx_shell, dim3(shell_blocks(c)), dim3(256), 0, c->stream,
                                  c->ta, c->tb, 0, c->geo, c->rxst, xi, xo, 0);
            ST_TRY(halo(c, {xo}));  // the black pass reads the neighbours' red cells
            sweep(RX_BLACK, nullptr, xo, it);
        } else {
            sweep(RX_JACOBI, xi, xo, it);
            ST_TRY(finish(it));
        }
        if (D && !single)
            ST_TRY(timed_span(c, c->stream, HIP_KT_HALO, [&] { return halo(c, {xo}); }, it));
        // the iteration's apply_bc: Neumann (linear_solver_redblack.c:139,
        // linear_solver_jacobi.c:118), or the caller's fixed boundary values,
        // or x's own boundary kept
        if (!neu_fold) {
            const double* shell_src = (c->poisson_bc == HIP_POISSON_BC_FIXED) ? c->bcfix : xi;
            const int shell_mode = (c->poisson_bc == HIP_POISSON_BC_NEUMANN) ? 1 : 0;
            hipExtLaunchKernelGGL(k_rx_shell, dim3(shell_blocks(c)), dim3(256), 0, c->stream,
                                  c->ta, c->tb, 0, c->geo, c->rxst, shell_src, xo, shell_mode);
        }
        return CFD_SUCCESS;
    };
    // iterations 0..max_iter: sweep it also yields the residual after it - 1
    // iterations, so the last launch only completes the final test
    static_assert(sizeof(RxState) <= sizeof(CgState), "h_state holds RxState copies");
    RxState* hs = reinterpret_cast<RxState*>(c->h_state);  // pinned, >= 3 RxState
    int it = 0, chunk = 8, slot = 0, prev = -1;
    const int chunk_max = std::max(1, c->cfg.poll_interval);
    while (it <= max_iter) {
        const int n = std::min(chunk, max_iter + 1 - it);
        for (int q = 0; q < n; ++q, ++it) ST_TRY(iterate(it));
        HIP_TRY(hipMemcpyAsync(&hs[slot], c->rxst, sizeof(RxState), hipMemcpyDeviceToHost,
                               c->stream));
        HIP_TRY(hipEventRecord(c->ev_poll[slot], c->stream));
        if (prev >= 0) {
            HIP_TRY(hipEventSynchronize(c->ev_poll[prev]));
            if (hs[prev].done) break;
        }
        prev = slot;
        slot ^= 1;
        chunk = std::min(chunk * 2, chunk_max);
    }
    HIP_TRY(hipMemcpyAsync(&hs[2], c->rxst, sizeof(RxState), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    flush_timing(c);
    const RxState& r = hs[2];
    if (r.status == ST_COMM_TIMEOUT) {
        set_err(CFD_ERROR, "relaxation: slab all-reduce timed out (a rank stopped)");
        return CFD_ERROR;
    }
    if (!r.done) {
        set_err(CFD_ERROR, "relaxation: device loop ended without a decision");
        return CFD_ERROR;
    }
    if (r.result == 1) std::swap(c->pn, c->xt);
    c->pstats.initial_residual = r.res0;
    c->pstats.iterations = r.iterations;
    c->pstats.final_residual = r.res;
    c->pstats.status = (poisson_solver_status_t)r.status;
    return (r.status == ST_CONVERGED) ? CFD_SUCCESS : CFD_ERROR_MAX_ITER;
}

// Relaxation methods driven by the common loop (linear_solver.c:397-485):
// L-infinity residual before the loop and every check_interval iterations.
static cfd_status_t relax_solve(hip_proj_ctx* c, int method, double dx, double dy, double dz,
                                double rel_tol, double abs_tol, int max_iter, int check_interval,
                                double omega_in) {
    const int G = tile_grid(c);
    RelaxCoef rc;
    rc.dx2 = dx * dx;
    rc.dy2 = dy * dy;
    rc.inv_dz2 = (dz > 0.0) ? (1.0 / (dz * dz)) : 0.0;
    rc.inv_factor = 1.0 / (2.0 * (1.0 / rc.dx2 + 1.0 / rc.dy2 + rc.inv_dz2));
    rc.omega = (omega_in <= 0.0) ? optimal_omega(c->nx, c->ny, c->nzg, dx, dy, dz) : omega_in;
    rc.rdx2 = 1.0 / rc.dx2;
    rc.rdy2 = 1.0 / rc.dy2;
    if ((c->sweep_ty == 16 || c->sweep_ty == 8) && max_iter > 0 &&
        (c->cfg.relax_two_pass != 1 || c->poisson_bc != HIP_POISSON_BC_NEUMANN))
        return relax_solve_fused(c, method, rc, rel_tol, abs_tol, max_iter, check_interval);
    ResCoef res_c{rc.dx2, rc.dy2, rc.inv_dz2};
    const DirVals dv{};
    // caller boundary modes (hip_proj_poisson_solve_ex): the iteration's
    // apply_bc copies the shell from bcfix (FIXED) or keeps x's own (NONE);
    // k_rx_shell does the copy, gated on an RxState that k_rx_init leaves
    // undecided
    const bool neumann_bc = c->poisson_bc == HIP_POISSON_BC_NEUMANN;
    if (!neumann_bc) {
        if (!c->rxst) HIP_TRY(hipMalloc((void**)&c->rxst, sizeof(RxState)));
        hipExtLaunchKernelGGL(k_rx_init, dim3(1), dim3(64), 0, c->stream, c->ta, c->tb, 0,
                              c->rxst, rel_tol, abs_tol, max_iter, check_interval);
    }
    ST_TRY(halo(c, {c->pn}));
    double res0 = 0.0;
    cfd_status_t s = residual_linf(c, c->pn, res_c, &res0);
    if (s != CFD_SUCCESS) return s;
    double tol = rel_tol * res0;
    if (tol < abs_tol) tol = abs_tol;
    c->pstats.initial_residual = res0;
    if (res0 < abs_tol) {
        c->pstats.status = POISSON_CONVERGED;
        c->pstats.iterations = 0;
        c->pstats.final_residual = res0;
        return CFD_SUCCESS;
    }
    int iter;
    bool conv = false;
    double res = res0;
    for (iter = 0; iter < max_iter; ++iter) {
        if (method == HIP_POISSON_REDBLACK) {
            timed(c, HIP_KT_RELAX, [&] {
                hipExtLaunchKernelGGL(k_rb_pass, dim3(G), dim3(NT), 0, c->stream, c->ta, c->tb, 0, c->geo, rc, c->pn,
                                   c->rhs, 1);
            });
            ST_TRY(halo(c, {c->pn}));  // the black pass reads the neighbours' red cells
            timed(c, HIP_KT_RELAX, [&] {
                hipExtLaunchKernelGGL(k_rb_pass, dim3(G), dim3(NT), 0, c->stream, c->ta, c->tb, 0, c->geo, rc, c->pn,
                                   c->rhs, 0);
            });
        } else {
            timed(c, HIP_KT_RELAX, [&] {
                hipExtLaunchKernelGGL(k_jacobi, dim3(G), dim3(NT), 0, c->stream, c->ta, c->tb, 0, c->geo, rc, c->pn,
                                   c->xt, c->rhs);
            });
            // memcpy(x, x_temp) + BC == swap buffers then BC (all boundary
            // cells are rewritten by the Neumann gather; with a caller mode
            // the shell is copied below)
            std::swap(c->pn, c->xt);
        }
        ST_TRY(halo(c, {c->pn}));
        if (neumann_bc) {
            launch_bc(c, c->pn, 0, dv);
        } else if (c->poisson_bc == HIP_POISSON_BC_FIXED || method != HIP_POISSON_REDBLACK) {
            // FIXED: the caller's values; NONE + Jacobi: the iterate's previous
            // boundary (now in xt), as the fused loop keeps it. NONE + RB-SOR
            // updates in place and never writes the shell.
            const double* src = (c->poisson_bc == HIP_POISSON_BC_FIXED) ? c->bcfix : c->xt;
            hipExtLaunchKernelGGL(k_rx_shell, dim3(shell_blocks(c)), dim3(256), 0, c->stream,
                                  c->ta, c->tb, 0, c->geo, c->rxst, src, c->pn, 0);
        }
        if (iter % check_interval == 0) {
            s = residual_linf(c, c->pn, res_c, &res);
            if (s != CFD_SUCCESS) return s;
            if (res < tol || res < abs_tol) {
                conv = true;
                break;
            }
        }
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    flush_timing(c);
    c->pstats.iterations = iter + 1;
    c->pstats.final_residual = res;
    c->pstats.status = conv ? POISSON_CONVERGED : POISSON_MAX_ITER;
    return conv ? CFD_SUCCESS : CFD_ERROR_MAX_ITER;
}

static cfd_status_t ensure_aux(hip_proj_ctx* c, bool need_rhs, bool need_xt) {
    const size_t n = field_elems(c);
    if (need_rhs && !c->rhs) {
        cfd_status_t s = dalloc(c, &c->rhs, n);
        if (s != CFD_SUCCESS) return s;
    }
    if (need_xt && !c->xt) {
        cfd_status_t s = dalloc(c, &c->xt, n);
        if (s != CFD_SUCCESS) return s;
    }
    return CFD_SUCCESS;
}

cfd_status_t ctx_validate_params(const hip_proj_ctx* c, const grid* g,
                                    const ns_solver_params_t* prm) {
    if (!g || !prm) return CFD_ERROR_INVALID;
    if (g->nx != c->nx || g->ny != c->ny || g->nz != c->nzg) {
        set_err(CFD_ERROR_INVALID, "projection_hip: grid does not match the context");
        return CFD_ERROR_INVALID;
    }
    if (g->nz > 1 && g->dz) {
        for (size_t k = 1; k < g->nz - 1; k++)
            if (fabs(g->dz[k] - g->dz[0]) > 1e-14) {  // solver_projection.c:59-66
                set_err(CFD_ERROR_INVALID, "projection_hip: non-uniform dz");
                return CFD_ERROR_INVALID;
            }
    }
    if (prm->source_func) {
        set_err(CFD_ERROR_UNSUPPORTED,
                "projection_hip: host source_func callbacks cannot run on the device");
        return CFD_ERROR_UNSUPPORTED;
    }
    if (prm->alpha > 0.0) {
        if (prm->heat_source_func) {  // host callback (gpu_shared_kernels.cuh:271-276)
            set_err(CFD_ERROR_UNSUPPORTED,
                    "projection_hip: host heat_source_func callbacks cannot run on the device");
            return CFD_ERROR_UNSUPPORTED;
        }
        const ns_thermal_bc_config_t& t = prm->thermal_bc;
        auto ok = [](bc_type_t b) {
            return b == BC_TYPE_PERIODIC || b == BC_TYPE_NEUMANN || b == BC_TYPE_DIRICHLET;
        };
        if (!ok(t.left) || !ok(t.right) || !ok(t.bottom) || !ok(t.top) ||
            (g->nz > 1 && (!ok(t.front) || !ok(t.back)))) {  // energy_solver.c:230-241
            set_err(CFD_ERROR_INVALID,
                    "energy_apply_thermal_bcs: unsupported thermal BC type on a face "
                    "(only PERIODIC, NEUMANN, DIRICHLET are valid)");
            return CFD_ERROR_INVALID;
        }
        if (c->nranks > 1 && ((t.back == BC_TYPE_PERIODIC) != (t.front == BC_TYPE_PERIODIC))) {
            set_err(CFD_ERROR_UNSUPPORTED,
                    "projection_hip: Z-slabs need periodic thermal BCs on both z faces or neither");
            return CFD_ERROR_UNSUPPORTED;
        }
    }
    return CFD_SUCCESS;
}

// ---------------------------------------------------------------------------
// C-ABI
// ---------------------------------------------------------------------------
extern "C" {

hip_proj_config_t hip_proj_config_default(void) {
    hip_proj_config_t c;
    memset(&c, 0, sizeof(c));
    c.device = -1;
    c.poisson_method = HIP_POISSON_CG;
    c.poisson_tolerance = 1e-6;
    c.poisson_abs_tolerance = 1e-10;
    c.poisson_max_iter = 5000;
    c.poisson_check_interval = 1;
    c.sor_omega = 0.0;
    c.poll_interval = 64;
    c.kchunk = 0;
    c.verbose = 0;
    c.sweep_rows = 16;   // tools/sweep_bench.py at 512^3: 16 rows + NT hints fastest
    // r01c / r01e sweep_bench at 512^3 (profiles/r01e_sweep_variants.jsonl)
    c.sweep_variant = SW_NT_STORE | SW_NT_LOAD | SW_PREFETCH | SW_EDGE1;
    c.rhs_density = 1;
    c.poisson_fail_fatal = 1;
    c.relax_two_pass = 0;
    c.sweep_variant_fold = 0;
    c.dirty_faces = 0;
    c.dirty_sync_interval = 0;
    c.cg_variant = 0;
    return c;
}

int hip_projection_available(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n > 0 ? 1 : 0;
}

static void free_ctx(hip_proj_ctx* c) {
    if (!c) return;
    if (c->stream) hipStreamSynchronize(c->stream);
    for (void* b : c->allocs) hipFree(b);
    if (c->st) hipFree(c->st);
    if (c->rxst) hipFree(c->rxst);
    if (c->rxst2) hipFree(c->rxst2);
    if (c->rb2dec) hipFree(c->rb2dec);
    if (c->partials) hipFree(c->partials);
    if (c->counter) hipFree(c->counter);
    if (c->red) hipFree(c->red);
    if (c->redg) hipFree(c->redg);
    if (c->dsum) hipFree(c->dsum);
    if (c->clk) hipFree(c->clk);
    if (c->h_state) hipHostFree(c->h_state);
    if (c->h_red) hipHostFree(c->h_red);
    if (c->h_src) hipHostFree(c->h_src);
    if (c->ev_src) hipEventDestroy(c->ev_src);
    if (c->shell_host) hipHostFree(c->shell_host);
    if (c->shell_dev) hipFree(c->shell_dev);
    for (int i = 0; i < 2; i++)
        if (c->ev_poll[i]) hipEventDestroy(c->ev_poll[i]);
    for (auto e : c->ev_pool) hipEventDestroy(e);
    if (c->ev_b) hipEventDestroy(c->ev_b);
    if (c->ev_h) hipEventDestroy(c->ev_h);
    if (c->hstream) {
        hipStreamSynchronize(c->hstream);
        hipStreamDestroy(c->hstream);
    }
    if (c->stream) hipStreamDestroy(c->stream);
    delete c;
}

// k_ccf's z layers over P planes: runs of kc, and with tail_layers > 0 the
// last tail_layers layers runs of kc2 (< kc) covering the remaining planes,
// so the workgroups dispatched last are short and the launch's tail (each CU
// idles while the last workgroups finish) shrinks. tail_layers = 0: every
// layer kc.
static void ccf_layout(SGeo& g, int P, int kc, int kc2, int tail_layers) {
    kc = std::max(1, std::min(kc, P));
    g.kc = kc;
    g.kc2 = kc;
    g.nz1 = g.tiles_z = (P + kc - 1) / kc;
    if (tail_layers <= 0 || kc2 <= 0 || kc2 >= kc) return;
    const int tail = std::min(P, tail_layers * kc2);
    const int bulk = P - tail;
    if (bulk <= 0) return;
    g.kc2 = kc2;
    g.nz1 = (bulk + kc - 1) / kc;
    // the bulk's last layer may be partial: the tail then starts at nz1 kc,
    // past the bulk, and covers P - nz1 kc planes
    const int rest = std::max(0, P - g.nz1 * kc);
    g.tiles_z = g.nz1 + (rest + kc2 - 1) / kc2;
}

static cfd_status_t init_ctx(hip_proj_ctx* c, size_t nx, size_t ny, size_t nz) {
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
    hipDeviceProp_t prop;
    HIP_TRY(hipGetDeviceProperties(&prop, c->device));
    c->grid_cap = std::max(64, prop.multiProcessorCount * 8);
    // field k starts k x 4 KiB into its allocation (r06): the march reads
    // r_it and p_{it-1} and writes p_it and r_{it+1} at equal offsets of
    // different fields, and with every field 2 MiB-aligned those streams meet
    // on the same HBM channels. 512^3 k_ccf, one box, four interleaved
    // rounds: 1.026-1.055 ms per iteration against 1.039-1.089 unstaggered
    // (2 / 1 / 8 KiB: 1.029-1.059 / 1.028-1.067 / 1.029-1.079,
    // profiles/r06l_ccf_stagger_ab.jsonl; r06k another box, same order).
    // Textbook CG's sweeps measured 0.8 % slower staggered (1.302-1.335 vs
    // 1.292-1.302 ms, r06m, where the march gained 1.044-1.048 vs
    // 1.038-1.062, profiles/r06m_stagger_both_cg_ab.jsonl), so the stagger
    // is the single-reduction contexts' default only.
    // CFD_HIP_FIELD_STAGGER=N overrides (0: aligned fields)
    c->stagger_bytes = (c->cfg.cg_variant == 1) ? 4096 : 0;
    if (const char* e = getenv("CFD_HIP_FIELD_STAGGER")) c->stagger_bytes = (size_t)atol(e) / 256 * 256;
    {
        auto ienv = [](const char* name, int dflt) {
            const char* e = getenv(name);
            return e ? atoi(e) : dflt;
        };
        c->env.ccf_off = ienv("CFD_HIP_CCF", 1) == 0;
        c->env.cg_small = ienv("CFD_HIP_CG_SMALL", -1);
        c->env.rb2_test = ienv("CFD_HIP_RB2_TEST", 0);
        c->env.rb2_xmap = ienv("CFD_HIP_RB2_XMAP", 0);
        c->env.rb2_log = getenv("CFD_HIP_RB2_LOG") != nullptr;
        c->env.rb2 = ienv("CFD_HIP_RB2", 1);
        c->env.ccf_xmap = ienv("CFD_HIP_CCF_XMAP", 0);
        c->env.cgb_rev = ienv("CFD_HIP_CGB_REV", 1) != 0;
        c->env.rb1_pf = ienv("CFD_HIP_RB1_PF", 1) != 0;
        c->env.rb1_alt = ienv("CFD_HIP_RB1_ALT", 1) != 0;
        c->env.rb1_fold = ienv("CFD_HIP_RB1_FOLD", 1) != 0;
        c->env.rk_pair = ienv("CFD_HIP_RK_PAIR", 1) != 0;
        c->env.alloc_contig = getenv("CFD_HIP_ALLOC") && strcmp(getenv("CFD_HIP_ALLOC"), "contig") == 0;
        c->env.ccf_edge_side = ienv("CFD_HIP_CCF_EDGE_SIDE", 1) != 0;
    }
    c->nx = nx;
    c->ny = ny;
    c->nz = nz;
    c->px = (long long)((nx + 7) / 8 * 8);
    // CFD_HIP_ROW_PAD=N (experiments, r06): N more doubles per row (a
    // multiple of 8), so that rows do not start on 4 KiB boundaries
    if (const char* e = getenv("CFD_HIP_ROW_PAD")) c->px += (long long)(std::max(0, atoi(e)) / 8 * 8);
    c->ps = c->px * (long long)ny;
    Geo& g = c->geo;
    g.nx = (int)nx;
    g.ny = (int)ny;
    g.nz = (int)nz;
    g.px = c->px;
    g.ps = c->ps;
    g.sz = (nz > 1) ? c->ps : 0;
    g.k0 = (nz > 1) ? 1 : 0;
    g.k1 = (nz > 1) ? (int)nz - 1 : 1;
    g.lo_face = (c->rank == 0) ? 1 : 0;
    g.hi_face = (c->rank == c->nranks - 1) ? 1 : 0;
    g.kofs = (int)c->kofs;
    const int nint_k = g.k1 - g.k0;
    int kc = 0;
    if (kc <= 0) {
        // enough tiles to fill every CU several times, long z runs otherwise
        long long xy_tiles = (long long)((nx + TX - 1) / TX) * (long long)((ny + TY - 1) / TY);
        long long want = 4LL * c->grid_cap;
        kc = (int)std::max<long long>(8, (xy_tiles * nint_k + want - 1) / want);
        kc = std::min(kc, std::max(1, nint_k));
    }
    g.kc = std::max(1, kc);
    g.tiles_x = (int)((nx + TX - 1) / TX);
    g.tiles_y = (int)((ny + TY - 1) / TY);
    g.tiles_z = (nint_k + g.kc - 1) / g.kc;

    // row-pair CG sweeps: 128 x TY x kc tiles (kernels.hpp, k_cgA / k_cgB)
    c->sweep_ty = (c->cfg.sweep_rows == 4 || c->cfg.sweep_rows == 16) ? c->cfg.sweep_rows : 8;
    {   // variants built: 0-3 (memory hints), 4 and 7 (+ plane prefetch)
        const int v = c->cfg.sweep_variant & 63;
        if (v == 15 && c->sweep_ty >= 8) c->sweep_variant = v;
        else if ((v == 23 || v == 31) && c->sweep_ty == 16) c->sweep_variant = v;
        else c->sweep_variant = (v & SW_PREFETCH) ? ((v & 3) == 3 ? 7 : 4) : (v & 3);
    }
    {
        const int vf = c->cfg.sweep_variant_fold;
        c->sweep_variant_fold = (c->sweep_ty == 16 && (vf == 3 || vf == 11 || vf == 15)) ? vf : 0;
    }
    SGeo& sg = c->sgeo;
    sg.nx = g.nx;
    sg.ny = g.ny;
    sg.nz = g.nz;
    sg.px = g.px;
    sg.ps = g.ps;
    sg.sz = g.sz;
    sg.k0 = g.k0;
    sg.k1 = g.k1;
    sg.kofs = g.kofs;
    sg.tiles_x = (int)((nx + 127) / 128);
    sg.tiles_y = (int)((ny + c->sweep_ty - 1) / c->sweep_ty);
    if (c->cfg.kchunk > 0) {
        sg.kc = c->cfg.kchunk;
    } else {
        // long z runs (each chunk re-reads two planes), shortened (down to
        // 4) until every CU has a workgroup: a thin slab or a mid-size grid
        // must still fill all 256 CUs. r01f at 512^3: 256-plane runs (256
        // workgroups) beat 64 by ~2 %; one 8-rank slab: 32 beat 16
        // (profiles/r01f_sweep_*). r02b: the floor was 16, which left 96^3 /
        // 128^3 at 36 / 64 workgroups; 4 takes a CG iteration from 53 to
        // 25 us / 58 to 33 us there (profiles/r02_small_grids.jsonl)
        sg.kc = 256;
        const long long want = c->grid_cap / 8;
        while (sg.kc > 4 &&
               (long long)sg.tiles_x * sg.tiles_y * ((nint_k + sg.kc - 1) / sg.kc) < want)
            sg.kc /= 2;
    }
    sg.kc = std::max(1, std::min(sg.kc, nint_k));
    sg.tiles_z = (nint_k + sg.kc - 1) / sg.kc;
    int n_partials = std::max(c->grid_cap, sg.tiles_x * sg.tiles_y * sg.tiles_z);
    // single-pass RB-SOR tiling (k_rb1): 124 x 12 cells written per 128 x 16 loaded
    {
        SGeo& rg = c->rgeo;
        rg = sg;
        // tile width: TC = 64 (128 x 16 cells loaded, 124 x 12 written). The
        // narrower tiles (32: 64 x 32, 16: 32 x 64) need ~20 % fewer
        // workgroups at 512^3 and 1024^2 x 512 but mask their halo rows per
        // lane instead of skipping whole waves, and measured slower (0.846 /
        // 1.022 vs 0.734 ms at 512^3, profiles/r02_rb_tile_width.jsonl);
        // CFD_HIP_RB1_TC = 32 / 16 selects them (experiments)
        int tc = 64;
        if (const char* e = getenv("CFD_HIP_RB1_TC")) {
            const int v = atoi(e);
            if (v == 64 || v == 32 || v == 16) tc = v;
        }
        c->rb1_tc = tc;
        const int ox = 2 * tc - 4, oy = 1024 / tc - 4;
        rg.tiles_x = (int)((nx - 1 + ox - 1) / ox);
        rg.tiles_y = (int)((ny - 1 + oy - 1) / oy);
        rg.kc = 64;
        if (const char* e = getenv("CFD_HIP_RB1_KC")) rg.kc = std::max(1, atoi(e));  // experiments
        while (rg.kc > 16 &&
               (long long)rg.tiles_x * rg.tiles_y * ((nint_k + rg.kc - 1) / rg.kc) < 512)
            rg.kc /= 2;
        // small grids: shorter runs (each costs a two-plane prologue) only
        // while fewer than half the CUs have a workgroup (r02b: 96^3 31 ->
        // 17 us per iteration at 4 planes; 128^3, 176 workgroups at 16
        // planes, is slower at 8 or 4; profiles/r02_small_grids.jsonl)
        while (rg.kc > 4 &&
               (long long)rg.tiles_x * rg.tiles_y * ((nint_k + rg.kc - 1) / rg.kc) < 128)
            rg.kc /= 2;
        rg.kc = std::max(1, std::min(rg.kc, nint_k));
        rg.tiles_z = (nint_k + rg.kc - 1) / rg.kc;
        n_partials = std::max(n_partials, rg.tiles_x * rg.tiles_y * rg.tiles_z);
        // two RB-SOR iterations per sweep (k_rb2, rb2.hpp): 64 x 32 cells
        // loaded, 56 x 24 written; one device, 3-D. Four partials per
        // workgroup (two maxima, the value range).
        SGeo& r2 = c->r2geo;
        r2 = rg;
        r2.tiles_x = r2.tiles_y = r2.tiles_z = 0;
        if (c->nranks == 1 && nz > 1 && nx >= 8 && ny >= 8) {
            r2.xofs = 0;
            r2.tiles_x = (int)((nx - 1 + RB2_OX - 1) / RB2_OX);
            r2.tiles_y = (int)((ny - 1 + RB2_OY - 1) / RB2_OY);
            // 128-plane z runs: the 6-plane pipeline fill is 4.7 % of a run
            // (1024^2 x 512: 2.16 -> 2.05 ms per iteration against 64;
            // 32: 2.34, profiles/r04_rb2_kc.jsonl)
            r2.kc = 128;
            // deep grids with many columns: three runs per column (1024^2 x
            // 512: 170 planes, 2451 workgroups, 1.735-1.739 vs 1.748-1.751 ms
            // per iteration against 128 in four same-box pairs on two boxes;
            // 255: 1.78-1.80, 510: 2.02; profiles/r05as_rb2_kc_ab.jsonl)
            if (nint_k >= 384 &&
                3LL * r2.tiles_x * r2.tiles_y >= 8LL * std::max(1, c->grid_cap / 8))
                r2.kc = (nint_k + 2) / 3;
            if (const char* e = getenv("CFD_HIP_RB2_KC")) r2.kc = std::max(1, atoi(e));
            while (r2.kc > 4 &&
                   (long long)r2.tiles_x * r2.tiles_y * ((nint_k + r2.kc - 1) / r2.kc) < 512)
                r2.kc /= 2;
            r2.kc = std::max(1, std::min(r2.kc, nint_k));
            r2.tiles_z = (nint_k + r2.kc - 1) / r2.kc;
            n_partials = std::max(n_partials, 2 * r2.tiles_x * r2.tiles_y * r2.tiles_z);
        }
        // the fused single-reduction CG iteration (k_ccf, ccf.hpp): 64 x 32
        // cells loaded, 60 x 28 written; one device, 3-D
        SGeo& cg = c->ccgeo;
        cg = rg;
        cg.tiles_x = cg.tiles_y = cg.tiles_z = 0;
        if (nz >= 3 && nx >= 4 && ny >= 4) {
            cg.xofs = 0;
            cg.tiles_x = (int)((nx - 1 + CCF_OX - 1) / CCF_OX);
            cg.tiles_y = (int)((ny - 1 + CCF_OY - 1) / CCF_OY);
            // z-run length: 24 planes on deep grids, 16 on thin ones (r05;
            // r04 had 32). 512^3 on one device: 24 at 1.048-1.049 vs 32's
            // 1.059 ms per iteration in every stable pair on two boxes (20 and
            // 28 equal to 24, 40 slower; profiles/r05ao_ccf_kc_ab.jsonl). The
            // rank-0 slab shapes of 2 / 4 / 8 ranks, 512^2 x 257 / 130 / 66:
            // 16 at 0.600-0.604 / 0.316-0.319 / 0.171 ms against 24's 0.613-
            // 0.615 / 0.317-0.318 / 0.169 and 32's 0.627-0.630 / 0.334-0.335 /
            // 0.197 (profiles/r05at_ccf_kc_thin_ab.jsonl)
            // r06: one device always 24 (256^3: 0.151-0.157 vs 16's 0.159-0.168
            // ms per iteration in three same-box pairs, profiles/r06c_ccf_kc_256_ab.jsonl;
            // the 16 of r05 was measured on 512^2 slab shapes only);
            // Z-slabs: 16, and 11 on slabs of <= 100 planes (512^2 x 66, the
            // 8-rank slab: 0.1615-0.1678 vs 16's 0.1706-0.1712, 13 0.1637-0.1693,
            // 21 0.168, 32 0.189-0.197; profiles/r06c_ccf_kc_slab8_ab.jsonl)
            cg.kc = (c->nranks == 1) ? 24 : (nint_k <= 100 ? 11 : 16);
            const char* ekc = getenv("CFD_HIP_CCF_KC");  // experiments
            if (ekc) cg.kc = std::max(1, atoi(ekc));
            const bool kc_fixed = getenv("CFD_HIP_CCF_KC_FIXED") != nullptr;
            while (!kc_fixed && cg.kc > 4 &&
                   (long long)cg.tiles_x * cg.tiles_y * ((nint_k + cg.kc - 1) / cg.kc) < 512)
                cg.kc /= 2;
            // tail layers of shorter runs (experiments: CFD_HIP_CCF_TAIL = layers,
            // CFD_HIP_CCF_KC2 = their run length; default off)
            const int tail_l = getenv("CFD_HIP_CCF_TAIL") ? atoi(getenv("CFD_HIP_CCF_TAIL")) : 0;
            const int kc2 = getenv("CFD_HIP_CCF_KC2") ? atoi(getenv("CFD_HIP_CCF_KC2")) : cg.kc / 2;
            c->ccf_tail = tail_l;
            c->ccf_kc2 = kc2;
            ccf_layout(cg, nint_k, cg.kc, kc2, tail_l);
            n_partials = std::max(n_partials, cg.tiles_x * cg.tiles_y * cg.tiles_z);
            // Z-slabs of >= 3 planes: the edge planes' launch (kmode 1) and
            // the interior planes' (kmode 2), so the r halo overlaps the latter
            c->cc_edge = c->cc_int = cg;
            c->cc_edge.tiles_x = c->cc_int.tiles_x = 0;
            if (c->nranks > 1 && nint_k >= 3) {
                SGeo& e = c->cc_edge;
                SGeo& m = c->cc_int;
                e = m = cg;
                e.kmode = 1;
                e.kc = 1;
                e.tiles_z = 2;
                m.kmode = 2;
                m.kt0 = cg.k0 + 1;
                m.kt1 = cg.k1 - 1;
                ccf_layout(m, m.kt1 - m.kt0, cg.kc, c->ccf_kc2, c->ccf_tail);
                // fused form: the interior march with stage c (cc_int_red)
                // and k_cc2 on the two edge planes (cc2_edge, the row-pair
                // tiling of k_cc2 in kmode 1) share one reduction, the
                // interior workgroups' partials first
                const char* ef = getenv("CFD_HIP_CCF_SLAB_FUSED");
                if (!(ef && atoi(ef) == 0)) {
                    SGeo& ir = c->cc_int_red;
                    SGeo& ee = c->cc2_edge;
                    ir = m;
                    ee = sg;
                    ee.kmode = 1;
                    ee.kc = 1;
                    ee.tiles_z = 2;
                    const int ni = ir.tiles_x * ir.tiles_y * ir.tiles_z;
                    const int ne = ee.tiles_x * ee.tiles_y * ee.tiles_z;
                    ir.part_ofs = 0;
                    ee.part_ofs = ni;
                    ir.part_total = ee.part_total = ni + ne;
                    n_partials = std::max(n_partials, ni + ne);
                }
            }
        }
        // the last x tile of a TC-64 launch is partial unless 124 divides the
        // row: its workgroups run a full tile's steps for a few columns
        // (512^3: 14 of 124). Up to 28 such columns run instead as a strip
        // of TC-16 tiles (28 columns x 60 rows, 4.8x fewer workgroups) in
        // the same grid (k_rb1m). CFD_HIP_RB1_STRIP=0: off.
        const char* estrip = getenv("CFD_HIP_RB1_STRIP");
        c->rb_strip_tc = 0;
        if (tc == 64 && c->nranks == 1 && !(estrip && atoi(estrip) == 0)) {
            const int T = (int)(nx / 124), R = (int)nx - 124 * T;
            // TC-32 strips (R in 29..60) measured slower (1024^2 x 512: 2.96 vs
            // 2.93 ms); TC-16 ones faster (512^3: 0.734 vs 0.760 ms,
            // profiles/r03_rb1_strip.jsonl)
            // R = 1 (nx = 124 T + 1): the T full tiles already store every
            // pair (cell nx - 1 is the Neumann mirror), so no strip
            const int stc = (R >= 2 && R <= 28) ? 16 : 0;
            if (stc) {
                c->rb_strip_tc = stc;
                SGeo& m = c->rg_main;
                SGeo& q = c->rg_strip;
                m = rg;
                m.tiles_x = T;
                q = rg;
                q.xofs = 124 * T;
                q.tiles_x = 1;
                const int oy = 1024 / stc - 4;
                q.tiles_y = (int)((ny - 1 + oy - 1) / oy);
                q.kc = std::max(1, std::min(rg.kc, nint_k));
                q.tiles_z = (nint_k + q.kc - 1) / q.kc;
                // one grid (k_rb1m): partial slot = blockIdx.x, total = gridDim.x
                m.part_ofs = q.part_ofs = 0;
                m.part_total = q.part_total = 0;
                n_partials = std::max(n_partials, m.tiles_x * m.tiles_y * m.tiles_z +
                                                      q.tiles_x * q.tiles_y * q.tiles_z);
            }
        }
        // Z-slabs: output planes k0+1 .. k1-2 split into two halves around
        // the edge planes (relax_solve_fused); CFD_HIP_RB_SPLIT=0 keeps the
        // one-launch iteration with blocking exchanges (A/B)
        const char* es = getenv("CFD_HIP_RB_SPLIT");
        c->split_rb = (c->nranks > 1 && nint_k >= 4 && !(es && atoi(es) == 0)) ? 1 : 0;
        if (c->split_rb) {
            const int a0 = g.k0 + 1, a1 = g.k1 - 1;  // interior output planes [a0, a1)
            const int mid = a0 + (a1 - a0) / 2;
            auto range = [&](SGeo& q, int lo, int hi) {
                q = rg;
                q.kmode = 2;
                q.kt0 = lo;
                q.kt1 = hi;
                q.kc = std::max(1, std::min(rg.kc, hi - lo));
                q.tiles_z = (hi - lo + q.kc - 1) / q.kc;
            };
            range(c->rg_in1, a0, mid);
            range(c->rg_in2, mid, a1);
            c->rg_edge = rg;
            c->rg_edge.kmode = 1;
            c->rg_edge.kc = 1;
            c->rg_edge.tiles_z = 2;
            const int xy = rg.tiles_x * rg.tiles_y;
            const int n1 = xy * c->rg_in1.tiles_z, ne = xy * 2, n2 = xy * c->rg_in2.tiles_z;
            c->rg_in1.part_ofs = 0;
            c->rg_edge.part_ofs = n1;
            c->rg_in2.part_ofs = n1 + ne;
            c->rg_in1.part_total = c->rg_edge.part_total = c->rg_in2.part_total = n1 + ne + n2;
            n_partials = std::max(n_partials, n1 + ne + n2);
        }
    }
    {   // predictor / corrector: 128 x PR_TY x kc tiles, >= ~8 workgroups per CU
        SGeo& pg = c->pgeo;
        pg = sg;
        pg.kmode = 0;
        pg.tiles_x = (int)((nx + 127) / 128);
        pg.tiles_y = (int)((ny + PR_TY - 1) / PR_TY);
        const long long xy = (long long)pg.tiles_x * pg.tiles_y;
        const long long zt = std::max(1LL, (4LL * c->grid_cap / PR_TY + xy - 1) / xy);
        pg.kc = (int)std::max<long long>(1, (nint_k + zt - 1) / zt);
        pg.tiles_z = (nint_k + pg.kc - 1) / pg.kc;
        // k_pred3 / k_corr3: the CG sweeps' 128 x 16 tiles, long z runs
        // shortened until every CU has a workgroup (one 1024-thread
        // workgroup per CU: 110 KB of LDS)
        SGeo& p3 = c->pgeo16;
        p3 = sg;
        p3.kmode = 0;
        p3.tiles_x = (int)((nx + 127) / 128);
        p3.tiles_y = (int)((ny + PC_TY - 1) / PC_TY);
        p3.kc = 256;
        while (p3.kc > 4 && (long long)p3.tiles_x * p3.tiles_y * ((nint_k + p3.kc - 1) / p3.kc) <
                                c->grid_cap / 8)
            p3.kc /= 2;
        p3.kc = std::max(1, std::min(p3.kc, nint_k));
        p3.tiles_z = (nint_k + p3.kc - 1) / p3.kc;
        // default k_pred3 / k_corr3 (r03: predictor 1.47 -> 1.25 ms, fetch
        // 45.7 -> 25.6 B/cell at 512^3, profiles/r03_pc3.jsonl);
        // CFD_HIP_PC3=0 selects k_pred2 / k_corr2
        c->pc3 = 1;
        if (const char* e = getenv("CFD_HIP_PC3")) {  // A/B: k_pred3 / k_corr3 (ctx.hpp)
            const int v = atoi(e);
            c->pc3 = (v == 1 || v == 2 || v == 4) ? v : 0;
        }
    }
    c->split_b = (c->nranks > 1 && nint_k >= 3) ? 1 : 0;
    if (c->split_b) {
        // sweep B on slabs: the two edge planes (what the neighbours need)
        // first, then planes k0+1 .. k1-1; one reduction over both launches
        SGeo& e = c->sg_edge;
        SGeo& m = c->sg_int;
        e = sg;
        e.kmode = 1;
        e.kc = 1;
        e.tiles_z = 2;
        m = sg;
        m.k0 = sg.k0 + 1;
        m.k1 = sg.k1 - 1;
        m.kc = std::max(1, std::min(sg.kc, m.k1 - m.k0));
        m.tiles_z = (m.k1 - m.k0 + m.kc - 1) / m.kc;
        const int ne = e.tiles_x * e.tiles_y * e.tiles_z;
        const int nm = m.tiles_x * m.tiles_y * m.tiles_z;
        e.part_ofs = 0;
        m.part_ofs = ne;
        e.part_total = m.part_total = ne + nm;
        n_partials = std::max(n_partials, ne + nm);
    }

    const size_t n = field_elems(c);
    double** fields[] = {&c->u, &c->v, &c->w, &c->p, &c->us, &c->vs, &c->ws, &c->pn,
                         &c->r, &c->pa, &c->pb, &c->pc4, &c->pd4};
    for (double** f : fields) {
        cfd_status_t s = dalloc(c, f, n);
        if (s != CFD_SUCCESS) return s;
    }
    if (dalloc(c, &c->src_u_row, ny) != CFD_SUCCESS) return CFD_ERROR;
    if (dalloc(c, &c->src_v_col, nx) != CFD_SUCCESS) return CFD_ERROR;
    HIP_TRY(hipHostMalloc((void**)&c->h_src, (nx + ny) * sizeof(double), hipHostMallocDefault));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_src, hipEventDisableTiming));
    HIP_TRY(hipMalloc((void**)&c->st, sizeof(CgState)));
    HIP_TRY(hipMemsetAsync(c->st, 0, sizeof(CgState), c->stream));
    // x2: the single-reduction CG reduces two values per workgroup
    // k_cg_small indexes its two partial slots by CGS_MAX_WG whatever the CU count
    n_partials = std::max(n_partials, CGS_MAX_WG);
    HIP_TRY(hipMalloc((void**)&c->partials, 2 * sizeof(double) * n_partials));
    HIP_TRY(hipMalloc((void**)&c->counter, 64));
    HIP_TRY(hipMemsetAsync(c->counter, 0, 64, c->stream));
    HIP_TRY(hipMalloc((void**)&c->red, 8 * sizeof(unsigned long long)));
    HIP_TRY(hipMalloc((void**)&c->redg, 8 * sizeof(unsigned long long)));
    HIP_TRY(hipMalloc((void**)&c->clk, 4 * sizeof(unsigned long long)));
    HIP_TRY(hipMemsetAsync(c->clk, 0, 4 * sizeof(unsigned long long), c->stream));
    HIP_TRY(hipMalloc((void**)&c->dsum, 4 * sizeof(double)));
    HIP_TRY(hipMemsetAsync(c->dsum, 0, 4 * sizeof(double), c->stream));
    HIP_TRY(hipHostMalloc((void**)&c->h_state, 3 * sizeof(CgState), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&c->h_red, 8 * sizeof(unsigned long long), hipHostMallocDefault));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_poll[0], hipEventDisableTiming));
    HIP_TRY(hipEventCreateWithFlags(&c->ev_poll[1], hipEventDisableTiming));
    if (c->nranks > 1) {
        HIP_TRY(hipStreamCreateWithFlags(&c->hstream, hipStreamNonBlocking));
        HIP_TRY(hipEventCreateWithFlags(&c->ev_b, hipEventDisableTiming));
        HIP_TRY(hipEventCreateWithFlags(&c->ev_h, hipEventDisableTiming));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    return CFD_SUCCESS;
}

// ---------------------------------------------------------------------------
// Placement draws of the single-reduction CG's fields (r06). The march
// (k_ccf) streams r_it and p_{it-1} in and p_it and r_{it+1} out at equal
// offsets of different fields, and how fast it runs depends on where the
// allocator placed those fields: in one process, six 512^3 contexts created
// one after another ran 1.034-1.222 ms per iteration, each one stable to
// 0.2 % (tools/alloc_lottery.py, profiles/r06s_alloc_lottery.jsonl; textbook
// CG's sweeps spread 2.5 %). So a large single-reduction context draws its CG
// fields (r, r2, the four p buffers, x) up to `draws` times, keeping every
// draw allocated until the end so that each lands on other pages, times a
// short fixed-iteration solve on each, keeps the fastest set and frees the
// others. Speed only: the fields are zeroed afterwards and the arithmetic is
// the same on any placement. The probes also try random assignments of the
// pool's buffers to the seven roles: what is slow is a PAIR of fields that
// meet (r06x: random assignments from 4 sets beat 8 sets as allocated).
// ---------------------------------------------------------------------------
static __global__ void k_probe_fill(double* f, long long n) {
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (long long)gridDim.x * blockDim.x) {
        const unsigned h = (unsigned)(e * 2654435761ll) >> 12;
        f[e] = (double)(h & 1023u) * (1.0 / 1024.0) - 0.5;
    }
}

static cfd_status_t placement_draws(hip_proj_ctx* c, int sets, int trials) {
    constexpr int NF = 7;
    constexpr int PROBE_IT = 16;  // probe solve: setup + 16 iterations (~20 ms at 512^3)
    double** slots[NF] = {&c->r, &c->r2, &c->pa, &c->pb, &c->pc4, &c->pd4, &c->pn};
    const size_t n = field_elems(c);
    const size_t fbytes = n * sizeof(double);
    if (!c->r2) ST_TRY(dalloc(c, &c->r2, n));
    // a short solve on a pseudo-random right-hand side (us, the predictor's
    // output buffer, free at creation), no early exit; device time by events
    hipEvent_t ea, eb;
    HIP_TRY(hipEventCreate(&ea));
    HIP_TRY(hipEventCreate(&eb));
    hipExtLaunchKernelGGL(k_probe_fill, dim3(4096), dim3(256), 0, c->stream, nullptr, nullptr, 0,
                          c->us, (long long)n);
    const double h = 1.0 / (double)(c->nx - 1);
    auto probe = [&](float* ms) -> cfd_status_t {
        double* keep_rhs = c->rhs;
        c->rhs = c->us;
        HIP_TRY(hipMemsetAsync(c->pn, 0, fbytes, c->stream));
        HIP_TRY(hipEventRecord(ea, c->stream));
        const cfd_status_t s = cg_solve(c, h, h, h, DivCoef{}, RHS_FROM_ARRAY, 0.0, 0.0, PROBE_IT, 1,
                                        false);
        c->rhs = keep_rhs;
        HIP_TRY(hipEventRecord(eb, c->stream));
        HIP_TRY(hipEventSynchronize(eb));
        HIP_TRY(hipEventElapsedTime(ms, ea, eb));
        return s == CFD_ERROR_MAX_ITER ? CFD_SUCCESS : s;
    };
    // the pool: the fields as created (set 0) and sets - 1 more allocations
    // of all seven, every one kept until the end so each lands on other pages
    std::vector<double*> pf;
    std::vector<void*> pb;
    // the allocation a field lives in: dalloc placed it allocs[i] + i x stagger
    auto base_of = [&](double* f) -> void* {
        for (size_t i = 0; i < c->allocs.size(); ++i)
            if ((char*)f - (char*)c->allocs[i] == (std::ptrdiff_t)(i * c->stagger_bytes))
                return c->allocs[i];
        return nullptr;
    };
    for (int q = 0; q < NF; ++q) {
        pf.push_back(*slots[q]);
        pb.push_back(base_of(*slots[q]));
    }
    for (int d = 1; d < sets; ++d) {
        size_t freeb = 0, total = 0;
        if (hipMemGetInfo(&freeb, &total) != hipSuccess || freeb < (size_t)(1.25 * NF * fbytes))
            break;
        // a set that cannot be allocated ends the pool (its allocated part
        // stays in it)
        bool ok = true;
        for (int q = 0; q < NF && ok; ++q) {
            double* f = nullptr;
            ok = dalloc(c, &f, n) == CFD_SUCCESS;
            if (ok) {
                pf.push_back(f);
                pb.push_back(c->allocs.back());
            }
        }
        if (!ok) {
            (void)hipGetLastError();
            break;
        }
    }
    // assignments of pool buffers to the seven roles: trial t < pool sets is
    // set t as allocated; the rest draw seven distinct buffers (a fixed LCG)
    const int npool = (int)pf.size();
    const int nsets = npool / NF;
    std::vector<std::array<int, NF>> asg;
    unsigned long long lcg = 0x9E3779B97F4A7C15ull;
    for (int t = 0; t < std::max(trials, 1); ++t) {
        std::array<int, NF> a{};
        if (t < nsets) {
            for (int q = 0; q < NF; ++q) a[q] = t * NF + q;
        } else {
            std::vector<int> idx(npool);
            for (int k = 0; k < npool; ++k) idx[k] = k;
            for (int q = 0; q < NF; ++q) {
                lcg = lcg * 6364136223846793005ull + 1442695040888963407ull;
                const int k = q + (int)((lcg >> 33) % (unsigned long long)(npool - q));
                std::swap(idx[q], idx[k]);
                a[q] = idx[q];
            }
        }
        asg.push_back(a);
    }
    cfd_status_t st = CFD_SUCCESS;
    std::vector<float> ms(asg.size(), 0.f);
    size_t done = 0;
    for (; done < asg.size() && st == CFD_SUCCESS; ++done) {
        for (int q = 0; q < NF; ++q) *slots[q] = pf[asg[done][q]];
        st = probe(&ms[done]);
    }
    hipEventDestroy(ea);
    hipEventDestroy(eb);
    if (st != CFD_SUCCESS) return st;
    size_t best = 0;
    for (size_t d = 1; d < done; ++d)
        if (ms[d] < ms[best]) best = d;
    for (int q = 0; q < NF; ++q) *slots[q] = pf[asg[best][q]];
    HIP_TRY(hipStreamSynchronize(c->stream));
    for (int k = 0; k < npool; ++k) {
        bool used = false;
        for (int q = 0; q < NF; ++q) used = used || asg[best][q] == k;
        if (used) continue;
        auto it = std::find(c->allocs.begin(), c->allocs.end(), pb[k]);
        if (pb[k] && it != c->allocs.end()) {
            c->allocs.erase(it);
            hipFree(pb[k]);
            c->bytes -= std::min(c->bytes, fbytes);
        }
    }
    c->placement_ms.clear();
    for (size_t d = 0; d < done; ++d) c->placement_ms.push_back(ms[d] / (float)PROBE_IT);
    c->placement_pick = (int)best;
    // a clean state: the probe's fields, its RHS buffer and the CG state
    for (int q = 0; q < NF; ++q) HIP_TRY(hipMemsetAsync(*slots[q], 0, fbytes, c->stream));
    HIP_TRY(hipMemsetAsync(c->us, 0, fbytes, c->stream));
    HIP_TRY(hipMemsetAsync(c->st, 0, sizeof(CgState), c->stream));
    c->pstats = poisson_solver_stats_t{};
    HIP_TRY(hipStreamSynchronize(c->stream));
    return CFD_SUCCESS;
}

static hip_proj_ctx* create_common(size_t nx, size_t ny, size_t nz_local, size_t nz_global,
                                   SlabComm* comm, size_t kofs, const hip_proj_config_t* cfg) {
    if (!hip_projection_available()) {
        set_err(CFD_ERROR_UNSUPPORTED, "projection_hip: no HIP device available");
        return nullptr;
    }
    hip_proj_ctx* c = new hip_proj_ctx();
    c->cfg = cfg ? *cfg : hip_proj_config_default();
    if (comm) {
        c->device = comm->device;
    } else if (c->cfg.device < 0) {
        int d = 0;
        hipGetDevice(&d);
        c->device = d;
    } else {
        c->device = c->cfg.device;
    }
    if (c->cfg.poll_interval <= 0) c->cfg.poll_interval = 64;
    c->comm = comm;
    c->rank = comm ? comm->rank : 0;
    c->nranks = comm ? comm->size : 1;
    c->nzg = nz_global;
    c->kofs = kofs;
    if (init_ctx(c, nx, ny, nz_local) != CFD_SUCCESS) {
        free_ctx(c);
        return nullptr;
    }
    // placement draws of the single-reduction CG's fields (3-D contexts of
    // >= 2^24 cells, one device or one Z-slab rank; see placement_draws)
    {
        // a pool of 6 allocated sets and 40 probes: the 6 sets as allocated,
        // then 34 random assignments of pool buffers to the seven roles.
        // r06x, 512^3, contexts of one process (ms per iteration): none
        // 1.109-1.201; 8 sets 1.037-1.126; 2 sets + 16 probes 1.033-1.047
        // with one 1.198 (a pool with no good pair); 4 sets + 16 probes
        // 1.030-1.044 (profiles/r06x_placement_strategies.jsonl). r06ar,
        // twelve contexts each: 4 sets + 24 probes 1.034-1.048 (mean
        // 1.0400), 6 + 40 1.032-1.042 (1.0372), 4 + 48 1.036-1.061
        // (profiles/r06ar_placement_draws.jsonl); ~0.3 s more per context.
        // CFD_HIP_PLACEMENT_DRAWS = sets (1: off), _TRIALS = probes
        const char* e = getenv("CFD_HIP_PLACEMENT_DRAWS");
        const int draws = e ? atoi(e) : 6;
        const char* et = getenv("CFD_HIP_PLACEMENT_TRIALS");
        const int trials = et ? std::max(1, atoi(et)) : 40;
        const long long cells = (long long)nx * (long long)ny * (long long)nz_local;
        if (c->cfg.cg_variant == 1 && nz_local >= 3 && cells >= (1LL << 24) && draws > 1 &&
            c->ccgeo.tiles_x > 0 && !c->env.ccf_off) {
            // a Z-slab rank probes its own fields as one device (no halo,
            // no all-reduce: nothing collective, so ranks may differ in how
            // many sets their memory allows), the march over its local planes
            const int nr = c->nranks;
            c->nranks = 1;
            const cfd_status_t ps = placement_draws(c, draws, trials);
            c->nranks = nr;
            if (ps != CFD_SUCCESS) {
                set_err(CFD_ERROR, "projection_hip: placement draws of the CG fields failed");
                free_ctx(c);
                return nullptr;
            }
        }
    }
    if (comm && c->cfg.poisson_method != HIP_POISSON_CG) {
        // Z-slab ranks of a relaxation solver: what the first solve would set
        // up lazily on a rank thread (the aux fields, the loop state, the
        // library's code object, which a kernel attribute query loads) is set
        // up here, at creation
        hipFuncAttributes fa;
        bool ok = hipFuncGetAttributes(&fa, (const void*)k_rx_init) == hipSuccess &&
                  ensure_aux(c, true, true) == CFD_SUCCESS;
        if (ok && !c->rxst) ok = hipMalloc((void**)&c->rxst, sizeof(RxState)) == hipSuccess;
        if (ok && !c->rxst2) ok = hipMalloc((void**)&c->rxst2, sizeof(RxState)) == hipSuccess;
        if (!ok) {
            set_err(CFD_ERROR_NOMEM, "projection_hip: slab relaxation setup failed");
            free_ctx(c);
            return nullptr;
        }
    }
    return c;
}

hip_proj_ctx_t* hip_proj_create(size_t nx, size_t ny, size_t nz, const hip_proj_config_t* cfg) {
    if (nx < 3 || ny < 3 || nz == 0 || (nz > 1 && nz < 3)) {
        set_err(CFD_ERROR_INVALID, "projection_hip: grid must be >= 3 points per active axis");
        return nullptr;
    }
    return create_common(nx, ny, nz, nz, nullptr, 0, cfg);
}

cfd_status_t hip_proj_slab_layout(size_t nz, int rank, int size, size_t* k_offset,
                                  size_t* nz_local) {
    if (nz < 3 || size < 1 || rank < 0 || rank >= size || (size_t)size > nz - 2)
        return CFD_ERROR_INVALID;
    // interior planes 1..nz-2 split as evenly as possible, lower ranks first
    const size_t nint = nz - 2, base = nint / (size_t)size, rem = nint % (size_t)size;
    const size_t r = (size_t)rank;
    const size_t first = 1 + r * base + std::min(r, rem);
    const size_t count = base + (r < rem ? 1 : 0);
    if (k_offset) *k_offset = first - 1;
    if (nz_local) *nz_local = count + 2;
    return CFD_SUCCESS;
}

hip_proj_ctx_t* hip_proj_create_slab(size_t nx, size_t ny, size_t nz, hip_proj_comm_t* comm,
                                     const hip_proj_config_t* cfg) {
    if (!comm || !comm->impl) {
        set_err(CFD_ERROR_INVALID, "hip_proj_create_slab: no communicator");
        return nullptr;
    }
    size_t kofs = 0, nzl = 0;
    if (nx < 3 || ny < 3 ||
        hip_proj_slab_layout(nz, comm->impl->rank, comm->impl->size, &kofs, &nzl) != CFD_SUCCESS) {
        set_err(CFD_ERROR_INVALID,
                "hip_proj_create_slab: 3-D grid with at least one interior plane per rank needed");
        return nullptr;
    }
    return create_common(nx, ny, nzl, nz, comm->impl, kofs, cfg);
}

cfd_status_t hip_proj_slab_info(const hip_proj_ctx_t* c, size_t* k_offset, size_t* nz_local,
                                int* rank, int* size) {
    if (!c) return CFD_ERROR_INVALID;
    if (k_offset) *k_offset = c->kofs;
    if (nz_local) *nz_local = c->nz;
    if (rank) *rank = c->rank;
    if (size) *size = c->nranks;
    return CFD_SUCCESS;
}

void hip_proj_destroy(hip_proj_ctx_t* ctx) {
    GroupHostLock hl_(ctx);  // holds the group, not the context: safe across the free
    free_ctx(ctx);
}

size_t hip_proj_device_bytes(const hip_proj_ctx_t* ctx) { return ctx ? ctx->bytes : 0; }
size_t hip_proj_row_pitch(const hip_proj_ctx_t* ctx) { return ctx ? (size_t)ctx->px : 0; }

cfd_status_t hip_proj_synchronize(hip_proj_ctx_t* c) {
    GroupHostLock hl_(c);
    if (!c) return CFD_ERROR_INVALID;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipStreamSynchronize(c->stream));
    flush_timing(c);
    return CFD_SUCCESS;
}

cfd_status_t hip_proj_set_field(hip_proj_ctx_t* c, int id, const double* host) {
    GroupHostLock hl_(c);
    if (!c || !host) return CFD_ERROR_INVALID;
    double* d = field_ptr(c, id);
    if ((id == HIP_FIELD_T || id == HIP_FIELD_RHO) && !d) {
        double** slot = (id == HIP_FIELD_T) ? &c->T : &c->rho;
        if (dalloc(c, slot, field_elems(c)) != CFD_SUCCESS) return CFD_ERROR_NOMEM;
        d = *slot;
    }
    if (!d) return CFD_ERROR_INVALID;
    c->resident = 0;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpy2DAsync(d, c->px * sizeof(double), host, c->nx * sizeof(double),
                             c->nx * sizeof(double), c->ny * c->nz, hipMemcpyHostToDevice,
                             c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (id == HIP_FIELD_T) c->have_T = c->T_dirty = 1;
    return CFD_SUCCESS;
}

cfd_status_t hip_proj_get_field(hip_proj_ctx_t* c, int id, double* host) {
    GroupHostLock hl_(c);
    if (!c || !host) return CFD_ERROR_INVALID;
    double* d = field_ptr(c, id);
    if (!d) return CFD_ERROR_INVALID;
    HIP_TRY(hipSetDevice(c->device));
    HIP_TRY(hipMemcpy2DAsync(host, c->nx * sizeof(double), d, c->px * sizeof(double),
                             c->nx * sizeof(double), c->ny * c->nz, hipMemcpyDeviceToHost,
                             c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return CFD_SUCCESS;
}

static __global__ void k_fill(double* f, long long n, double v) {
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (long long)gridDim.x * blockDim.x)
        f[e] = v;
}

cfd_status_t hip_proj_fill_field(hip_proj_ctx_t* c, int id, double value) {
    GroupHostLock hl_(c);
    if (!c) return CFD_ERROR_INVALID;
    double* d = field_ptr(c, id);
    if ((id == HIP_FIELD_T || id == HIP_FIELD_RHO) && !d) {
        double** slot = (id == HIP_FIELD_T) ? &c->T : &c->rho;
        if (dalloc(c, slot, field_elems(c)) != CFD_SUCCESS) return CFD_ERROR_NOMEM;
        d = *slot;
        if (id == HIP_FIELD_T) c->have_T = 1;
    }
    if (!d) return CFD_ERROR_INVALID;
    c->resident = 0;
    HIP_TRY(hipSetDevice(c->device));
    hipExtLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, c->stream, c->ta, c->tb, 0, d,
                       (long long)field_elems(c), value);
    HIP_TRY(hipGetLastError());
    if (id == HIP_FIELD_T) c->T_dirty = 1;
    return CFD_SUCCESS;
}

cfd_status_t hip_proj_set_density(hip_proj_ctx_t* c, double rho0) {
    GroupHostLock hl_(c);
    if (!c) return CFD_ERROR_INVALID;
    c->rho0 = rho0;
    // a per-cell density array (RK4, restart files) follows the uniform value
    if (c->rho) return hip_proj_fill_field(c, HIP_FIELD_RHO, rho0);
    return CFD_SUCCESS;
}

cfd_status_t hip_proj_upload(hip_proj_ctx_t* c, const flow_field* f) {
    GroupHostLock hl_(c);
    if (!c || !f) return CFD_ERROR_INVALID;
    if (f->nx != c->nx || f->ny != c->ny || f->nz != c->nz) return CFD_ERROR_INVALID;
    cfd_status_t s;
    if ((s = hip_proj_set_field(c, HIP_FIELD_U, f->u)) != CFD_SUCCESS) return s;
    if ((s = hip_proj_set_field(c, HIP_FIELD_V, f->v)) != CFD_SUCCESS) return s;
    if ((s = hip_proj_set_field(c, HIP_FIELD_W, f->w)) != CFD_SUCCESS) return s;
    if ((s = hip_proj_set_field(c, HIP_FIELD_P, f->p)) != CFD_SUCCESS) return s;
    if (f->T) {
        if ((s = hip_proj_set_field(c, HIP_FIELD_T, f->T)) != CFD_SUCCESS) return s;
    }
    c->rho0 = f->rho ? f->rho[0] : 1.0;
    if (c->rho) {  // keep an existing per-cell density in step with the field
        s = f->rho ? hip_proj_set_field(c, HIP_FIELD_RHO, f->rho)
                   : hip_proj_fill_field(c, HIP_FIELD_RHO, 1.0);
        if (s != CFD_SUCCESS) return s;
    }
    return CFD_SUCCESS;
}

cfd_status_t hip_proj_download(hip_proj_ctx_t* c, flow_field* f) {
    GroupHostLock hl_(c);
    if (!c || !f) return CFD_ERROR_INVALID;
    cfd_status_t s;
    if ((s = hip_proj_get_field(c, HIP_FIELD_U, f->u)) != CFD_SUCCESS) return s;
    if ((s = hip_proj_get_field(c, HIP_FIELD_V, f->v)) != CFD_SUCCESS) return s;
    if ((s = hip_proj_get_field(c, HIP_FIELD_W, f->w)) != CFD_SUCCESS) return s;
    if ((s = hip_proj_get_field(c, HIP_FIELD_P, f->p)) != CFD_SUCCESS) return s;
    return CFD_SUCCESS;
}

cfd_status_t hip_proj_apply_scalar_bc(hip_proj_ctx_t* c, int id, bc_type_t type) {
    GroupHostLock hl_(c);
    if (!c) return CFD_ERROR_INVALID;
    c->resident = 0;
    double* d = field_ptr(c, id);
    if (!d) return CFD_ERROR_INVALID;
    int mode;
    if (type == BC_TYPE_NEUMANN) mode = 0;
    else if (type == BC_TYPE_PERIODIC) mode = 1;
    else {
        set_err(CFD_ERROR_UNSUPPORTED, "hip_proj_apply_scalar_bc: only NEUMANN and PERIODIC");
        return CFD_ERROR_UNSUPPORTED;
    }
    HIP_TRY(hipSetDevice(c->device));
    if (mode == 1 && dist(c)) {
        // periodic z across slabs: x/y ring on every local plane, then the
        // z copy (plane 0 <- nz-2, nz-1 <- 1) as a wrap-around halo exchange
        Geo g = c->geo;
        g.lo_face = g.hi_face = 0;
        hipExtLaunchKernelGGL(k_bc_shell, dim3(shell_blocks(c)), dim3(256), 0, c->stream, c->ta, c->tb, 0, g, d, mode,
                           DirVals{});
        HIP_TRY(hipGetLastError());
        return halo(c, {d}, true);
    }
    launch_bc(c, d, mode, DirVals{});
    HIP_TRY(hipGetLastError());
    return CFD_SUCCESS;
}

cfd_status_t hip_proj_apply_dirichlet(hip_proj_ctx_t* c, int id, const bc_dirichlet_values_t* v) {
    GroupHostLock hl_(c);
    if (!c || !v) return CFD_ERROR_INVALID;
    c->resident = 0;
    double* d = field_ptr(c, id);
    if (!d) return CFD_ERROR_INVALID;
    DirVals dv{v->left, v->right, v->top, v->bottom, v->front, v->back};
    HIP_TRY(hipSetDevice(c->device));
    launch_bc(c, d, 2, dv);
    HIP_TRY(hipGetLastError());
    return CFD_SUCCESS;
}

cfd_status_t hip_proj_apply_thermal_bcs(hip_proj_ctx_t* c, const ns_solver_params_t* prm) {
    GroupHostLock hl_(c);
    if (!c || !prm) return CFD_ERROR_INVALID;
    c->resident = 0;
    if (!c->T) {
        set_err(CFD_ERROR_INVALID, "energy_apply_thermal_bcs: missing temperature field");
        return CFD_ERROR_INVALID;
    }
    if (prm->alpha <= 0.0) return CFD_SUCCESS;  // energy disabled: no-op (energy_solver.c:217)
    HIP_TRY(hipSetDevice(c->device));
    ST_TRY(ctx_apply_thermal_bcs(c, prm->thermal_bc, c->nzg > 1));
    c->T_dirty = 1;
    return CFD_SUCCESS;
}

cfd_status_t hip_proj_get_poisson_stats(hip_proj_ctx_t* c, poisson_solver_stats_t* s) {
    GroupHostLock hl_(c);
    if (!c || !s) return CFD_ERROR_INVALID;
    *s = c->pstats;
    return CFD_SUCCESS;
}

void hip_proj_enable_timing(hip_proj_ctx_t* c, int enable) {
    GroupHostLock hl_(c);
    if (c) c->timing = enable ? 1 : 0;
}

void hip_proj_reset_timing(hip_proj_ctx_t* c) {
    GroupHostLock hl_(c);
    if (!c) return;
    hipStreamSynchronize(c->stream);
    flush_timing(c);
    for (int k = 0; k < HIP_KT_COUNT; k++) {
        c->kt_ms[k] = 0;
        c->kt_n[k] = 0;
    }
    if (c->clk) {
        hipMemsetAsync(c->clk, 0, 4 * sizeof(unsigned long long), c->stream);
        hipStreamSynchronize(c->stream);
    }
}

int hip_proj_get_placement(hip_proj_ctx_t* c, double* ms_per_iter, int capacity, int* picked) {
    GroupHostLock hl_(c);
    if (picked) *picked = c ? c->placement_pick : -1;
    if (!c) return 0;
    const int n = (int)c->placement_ms.size();
    for (int i = 0; i < n && i < capacity && ms_per_iter; ++i) ms_per_iter[i] = c->placement_ms[i];
    return n;
}

cfd_status_t hip_proj_get_clock_sample(hip_proj_ctx_t* c, double* mhz, long long* workgroups) {
    GroupHostLock hl_(c);
    if (!c) return CFD_ERROR_INVALID;
    unsigned long long h[4] = {0, 0, 0, 0};
    if (c->clk) {
        HIP_TRY(hipSetDevice(c->device));
        HIP_TRY(hipStreamSynchronize(c->stream));
        HIP_TRY(hipMemcpy(h, c->clk, sizeof(h), hipMemcpyDeviceToHost));
    }
    if (mhz) *mhz = h[1] ? 100.0 * (double)h[0] / (double)h[1] : 0.0;
    if (workgroups) *workgroups = (long long)h[2];
    return CFD_SUCCESS;
}

int hip_proj_get_timing_n(hip_proj_ctx_t* c, double* total_ms, long long* launches,
                          int capacity) {
    GroupHostLock hl_(c);
    if (!c || capacity <= 0) return 0;
    hipStreamSynchronize(c->stream);
    flush_timing(c);
    const int n = std::min(capacity, (int)HIP_KT_COUNT);
    for (int k = 0; k < n; k++) {
        if (total_ms) total_ms[k] = c->kt_ms[k];
        if (launches) launches[k] = c->kt_n[k];
    }
    return n;
}

void hip_proj_get_timing(hip_proj_ctx_t* c, double* total_ms, long long* launches) {
    (void)hip_proj_get_timing_n(c, total_ms, launches, HIP_KT_COUNT_LEGACY);
}

int hip_proj_abi_version(void) { return HIP_PROJ_ABI_VERSION; }

}  // extern "C"

// energy_apply_thermal_bcs (energy_solver.c:204-334) on the device T:
// x faces, y faces, z faces (3-D), each a gather pass in the reference order.
cfd_status_t ctx_apply_thermal_bcs(hip_proj_ctx* c, const ns_thermal_bc_config_t& t, bool is3d) {
    ThermalFaces tf;
    const bc_type_t ty[6] = {t.left, t.right, t.bottom, t.top, t.back, t.front};
    const double v[6] = {t.dirichlet_values.left, t.dirichlet_values.right,
                         t.dirichlet_values.bottom, t.dirichlet_values.top,
                         t.dirichlet_values.back, t.dirichlet_values.front};
    for (int f = 0; f < 6; ++f) {
        tf.type[f] = (ty[f] == BC_TYPE_PERIODIC || ty[f] == BC_TYPE_NEUMANN ||
                      ty[f] == BC_TYPE_DIRICHLET) ? (int)ty[f] : -1;
        tf.val[f] = v[f];
    }
    auto blocks = [](long long n) {
        return (unsigned)std::max(1LL, std::min((n + 255) / 256, 65535LL));
    };
    hipExtLaunchKernelGGL(k_thermal_bc, dim3(blocks(2LL * c->ny * c->nz)), dim3(256), 0, c->stream, c->ta, c->tb, 0,
                       c->geo, c->T, tf, 0);
    hipExtLaunchKernelGGL(k_thermal_bc, dim3(blocks(2LL * c->nx * c->nz)), dim3(256), 0, c->stream, c->ta, c->tb, 0,
                       c->geo, c->T, tf, 1);
    if (is3d) {
        if (dist(c) && t.back == BC_TYPE_PERIODIC && t.front == BC_TYPE_PERIODIC) {
            ST_TRY(halo(c, {c->T}, true));  // z wrap across the slabs
        } else {
            hipExtLaunchKernelGGL(k_thermal_bc, dim3(blocks(2LL * c->nx * c->ny)), dim3(256), 0,
                               c->stream, c->ta, c->tb, 0, c->geo, c->T, tf, 2);
        }
    }
    HIP_TRY(hipGetLastError());
    return CFD_SUCCESS;
}

cfd_status_t ctx_energy_step(hip_proj_ctx* c, const grid* g, const ns_solver_params_t* prm,
                             bool apply_bcs) {
    // energy_step_explicit_with_workspace (energy_solver.c:21-176) on the
    // current velocity, then energy_apply_thermal_bcs (:204-334)
    const size_t nz = c->nzg;
    const double dx = g->dx[0], dy = g->dy[0];
    const double dz = (nz > 1 && g->dz) ? g->dz[0] : 0.0;
    if (!c->Tn) ST_TRY(dalloc(c, &c->Tn, field_elems(c)));
    EnergyCoef ec;
    ec.inv_2dx = 1.0 / (2.0 * dx);
    ec.inv_2dy = 1.0 / (2.0 * dy);
    ec.inv_2dz = (nz > 1 && g->dz) ? 1.0 / (2.0 * dz) : 0.0;
    ec.inv_dx2 = 1.0 / (dx * dx);
    ec.inv_dy2 = 1.0 / (dy * dy);
    ec.inv_dz2 = (nz > 1 && g->dz) ? 1.0 / (dz * dz) : 0.0;
    ec.alpha = prm->alpha;
    ec.dt = prm->dt;
    timed(c, HIP_KT_ENERGY, [&] {
        hipExtLaunchKernelGGL(k_energy, cell_grid(c), dim3(256), 0, c->stream, c->ta, c->tb, 0,
                              c->geo, ec, c->T, c->u, c->v, c->w, c->Tn, c->red);
    });
    std::swap(c->T, c->Tn);
    if (apply_bcs) ST_TRY(ctx_apply_thermal_bcs(c, prm->thermal_bc, nz > 1));
    c->T_dirty = 1;
    return CFD_SUCCESS;
}

void ctx_queue_max_T(hip_proj_ctx* c) {
    if (!c->have_T || !c->T_dirty) return;
    // compute_max_temperature (solver_registry.c:52-62), owned planes + faces
    const int ks = (c->nz > 1 && !c->geo.lo_face) ? 1 : 0;
    const int ke = (c->nz > 1 && !c->geo.hi_face) ? (int)c->nz - 1 : (int)c->nz;
    const dim3 cg = cell_grid(c);
    hipLaunchKernelGGL(k_field_max, dim3(cg.x, cg.y, (unsigned)(ke - ks)), dim3(256), 0,
                       c->stream, c->geo, c->T, c->red + 3, ks);
}

extern "C" {

static cfd_status_t step_device_impl(hip_proj_ctx_t* c, const grid* g,
                                     const ns_solver_params_t* prm, ns_solver_stats_t* stats,
                                     int iter) {
    if (!c) return CFD_ERROR_INVALID;
    cfd_status_t s = ctx_validate_params(c, g, prm);
    if (s != CFD_SUCCESS) return s;
    HIP_TRY(hipSetDevice(c->device));
    const size_t nz = c->nzg;
    const double dx = g->dx[0], dy = g->dy[0];
    const double dz = (nz > 1 && g->dz) ? g->dz[0] : 0.0;
    const double dt = prm->dt;
    const bool buoy = (prm->beta != 0.0);
    const bool energy = (prm->alpha > 0.0);
    if ((buoy || energy) && !c->have_T) {
        set_err(CFD_ERROR_INVALID, "projection_hip: buoyancy / energy equation need the T field");
        return CFD_ERROR_INVALID;
    }

    // source-term tables: compute_source_terms at iter = 0 (solver_explicit_euler.c:317-333)
    ST_TRY(upload_source_tables(c, g, prm, iter));

    PredCoef2 pc;
    pc.two_dx = 2.0 * dx;
    pc.two_dy = 2.0 * dy;
    pc.inv_2dz = (nz > 1 && g->dz) ? 1.0 / (2.0 * dz) : 0.0;
    pc.dx_sq = dx * dx;
    pc.dy_sq = dy * dy;
    pc.inv_dz2 = (nz > 1 && g->dz) ? 1.0 / (dz * dz) : 0.0;
    pc.r_two_dx = 1.0 / pc.two_dx;
    pc.r_two_dy = 1.0 / pc.two_dy;
    pc.r_dx_sq = 1.0 / pc.dx_sq;
    pc.r_dy_sq = 1.0 / pc.dy_sq;
    pc.dt = dt;
    pc.nu = prm->mu;
    pc.beta = prm->beta;
    pc.T_ref = prm->T_ref;
    pc.g0 = prm->gravity[0];
    pc.g1 = prm->gravity[1];
    pc.g2 = prm->gravity[2];
    const unsigned npg = (unsigned)(c->pgeo.tiles_x * c->pgeo.tiles_y * c->pgeo.tiles_z);
    // slabs: the neighbours' planes of everything the stencils read
    ST_TRY(halo(c, {c->u, c->v, c->w, c->p}));
    if (buoy || energy) ST_TRY(halo(c, {c->T}));
    const unsigned np3 =
        (unsigned)(c->pgeo16.tiles_x * c->pgeo16.tiles_y * c->pgeo16.tiles_z);
    timed(c, HIP_KT_PREDICTOR, [&] {
        // PF = 0: one plane's loads per step (the plane-ahead schedule
        // measured slower, profiles/r02_step_kernels.jsonl)
        auto p3 = [&](auto kern) {
            hipExtLaunchKernelGGL(kern, dim3(np3), dim3(64 * PC_TY), 0, c->stream, c->ta, c->tb, 0,
                                  c->pgeo16, pc, c->u, c->v, c->w, c->T, c->src_u_row,
                                  c->src_v_col, c->us, c->vs, c->ws);
        };
        if (c->pc3 == 1) {
            if (buoy) p3(k_pred3<true, 0>);
            else p3(k_pred3<false, 0>);
        } else if (c->pc3 == 2) {
            if (buoy) p3(k_pred3<true, SW_NT_STORE>);
            else p3(k_pred3<false, SW_NT_STORE>);
        } else if (c->pc3 == 4) {
            if (buoy) p3(k_pred3<true, SW_NT_STORE | SW_NT_LOAD>);
            else p3(k_pred3<false, SW_NT_STORE | SW_NT_LOAD>);
        } else if (buoy)
            hipExtLaunchKernelGGL((k_pred2<true, 0>), dim3(npg), dim3(64 * PR_TY), 0, c->stream,
                                  c->ta, c->tb, 0, c->pgeo, pc, c->u, c->v, c->w, c->T,
                                  c->src_u_row, c->src_v_col, c->us, c->vs, c->ws);
        else
            hipExtLaunchKernelGGL((k_pred2<false, 0>), dim3(npg), dim3(64 * PR_TY), 0, c->stream,
                                  c->ta, c->tb, 0, c->pgeo, pc, c->u, c->v, c->w, c->T,
                                  c->src_u_row, c->src_v_col, c->us, c->vs, c->ws);
    });
    hipExtLaunchKernelGGL(k_shell_copy, dim3(shell_blocks(c)), dim3(256), 0, c->stream, c->ta,
                          c->tb, 0, c->geo, c->u, c->v, c->w, c->us, c->vs, c->ws);
    HIP_TRY(hipGetLastError());
    ST_TRY(halo(c, {c->ws}));  // d(w*)/dz of the divergence

    // p_new = p (solver_projection.c:108)
    HIP_TRY(hipMemcpyAsync(c->pn, c->p, field_elems(c) * sizeof(double), hipMemcpyDeviceToDevice,
                           c->stream));

    double rho = c->rho0;
    if (rho < 1e-10) rho = 1.0;
    DivCoef dc;
    dc.two_dx = 2.0 * dx;
    dc.two_dy = 2.0 * dy;
    dc.inv_2dz = pc.inv_2dz;
    dc.rho_over_dt = c->cfg.rhs_density ? rho / dt : 1.0 / dt;

    const int method = c->cfg.poisson_method;
    cfd_status_t ps;
    if (method == HIP_POISSON_CG) {
        ps = cg_solve(c, dx, dy, dz, dc, RHS_FROM_VELOCITY, c->cfg.poisson_tolerance,
                      c->cfg.poisson_abs_tolerance, c->cfg.poisson_max_iter,
                      std::max(1, c->cfg.poisson_check_interval), true);
    } else {
        s = ensure_aux(c, true, method == HIP_POISSON_JACOBI);
        if (s != CFD_SUCCESS) return s;
        const Lap L = make_lap(dx, dy, dz);
        const int G = tile_grid(c);
        hipExtLaunchKernelGGL((k_cg_setup<true, true, false>), dim3(G), dim3(NT), 0, c->stream, c->ta, c->tb, 0,
                           c->geo, L, dc, c->us, c->vs, c->ws, c->rhs, c->pn, c->r, c->st,
                           c->partials, c->counter, 0.0, 0.0, 0, 1, c->dsum, (Mbox*)nullptr);
        if (method == HIP_POISSON_JACOBI)
            HIP_TRY(hipMemsetAsync(c->xt, 0, field_elems(c) * sizeof(double), c->stream));
        int maxit = c->cfg.poisson_max_iter;
        ps = relax_solve(c, method, dx, dy, dz, c->cfg.poisson_tolerance,
                         c->cfg.poisson_abs_tolerance, maxit,
                         std::max(1, c->cfg.poisson_check_interval), c->cfg.sor_omega);
    }
    if (ps == CFD_ERROR_MAX_ITER && !c->cfg.poisson_fail_fatal) ps = CFD_SUCCESS;
    if (ps != CFD_SUCCESS) {
        if (ps == CFD_ERROR_MAX_ITER) set_err(CFD_ERROR_MAX_ITER, "projection_hip: pressure solve did not converge");
        return ps;
    }

    CorrCoef2 cc;
    cc.two_dx = 2.0 * dx;
    cc.two_dy = 2.0 * dy;
    cc.inv_2dz = pc.inv_2dz;
    cc.r_two_dx = pc.r_two_dx;
    cc.r_two_dy = pc.r_two_dy;
    cc.dt_over_rho = dt / rho;
    hipExtLaunchKernelGGL(k_init_red, dim3(1), dim3(64), 0, c->stream, c->ta, c->tb, 0, c->red);
    timed(c, HIP_KT_CORRECTOR, [&] {
        auto c3 = [&](auto kern) {
            hipExtLaunchKernelGGL(kern, dim3(np3), dim3(64 * PC_TY), 0, c->stream, c->ta, c->tb, 0,
                                  c->pgeo16, cc, c->us, c->vs, c->ws, c->pn, c->u, c->v, c->w,
                                  c->red);
        };
        if (c->pc3 == 1) c3(k_corr3<0>);
        else if (c->pc3 == 2) c3(k_corr3<SW_NT_STORE>);
        else if (c->pc3 == 4) c3(k_corr3<SW_NT_STORE | SW_NT_LOAD>);
        else
            hipExtLaunchKernelGGL((k_corr2<0>), dim3(npg), dim3(64 * PR_TY), 0, c->stream, c->ta,
                                  c->tb, 0, c->pgeo, cc, c->us, c->vs, c->ws, c->pn, c->u, c->v,
                                  c->w, c->red);
    });
    hipExtLaunchKernelGGL(k_shell_stats, dim3(shell_blocks(c)), dim3(256), 0, c->stream, c->ta,
                          c->tb, 0, c->geo, c->u, c->v, c->w, c->pn, c->red);
    std::swap(c->p, c->pn);  // memcpy(field->p, p_new) (solver_projection.c:253)
    if (energy) ST_TRY(ctx_energy_step(c, g, prm, true));  // solver_projection.c:255-274
    ctx_queue_max_T(c);
    const unsigned long long* red = reduce_red(c, &s);
    if (s != CFD_SUCCESS) return s;
    HIP_TRY(hipMemcpyAsync(c->h_red, red, 8 * sizeof(unsigned long long), hipMemcpyDeviceToHost,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    flush_timing(c);
    if (c->h_red[5]) {
        set_err(CFD_ERROR_DIVERGED, "NaN/Inf detected in energy_step_explicit");
        return CFD_ERROR_DIVERGED;
    }
    if (c->h_red[2]) {
        set_err(CFD_ERROR_DIVERGED, "projection_hip: NaN/Inf in the flow field");
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
    return CFD_SUCCESS;
}

cfd_status_t hip_proj_mark_host_dirty(hip_proj_ctx_t* c) {
    GroupHostLock hl_(c);
    if (!c) return CFD_ERROR_INVALID;
    c->resident = 0;
    c->hash_ok = 0;
    return CFD_SUCCESS;
}

cfd_status_t hip_proj_step_device(hip_proj_ctx_t* c, const grid* g,
                                  const ns_solver_params_t* prm, ns_solver_stats_t* stats) {
    GroupHostLock hl_(c);
    if (c) c->resident = 0;
    return step_device_impl(c, g, prm, stats, 0);
}

}  // extern "C"

// Fields of the host-buffer step: u, v, w, p and, when present, T.
static int host_fields(hip_proj_ctx* c, flow_field* f, double** host, double** dev) {
    host[0] = f->u, host[1] = f->v, host[2] = f->w, host[3] = f->p;
    dev[0] = c->u, dev[1] = c->v, dev[2] = c->w, dev[3] = c->p;
    if (!f->T || !c->T) return 4;
    host[4] = f->T;
    dev[4] = c->T;
    return 5;
}

// Host-buffer path shared by hip_proj_step (one step, shell_ok = 1) and the
// plugin's solve (n steps, source-term iteration index 0..n-1 as in
// solver_projection.c:112). In the resident mode (cfg.dirty_faces, see
// shell_io.hip) a step on the same host arrays as the previous one uploads
// only the depth-1 boundary shell and downloads the depth-2 shell.
static cfd_status_t host_steps(hip_proj_ctx_t* c, flow_field* f, const grid* g,
                               const ns_solver_params_t* prm, ns_solver_stats_t* stats,
                               int n_steps, bool shell_ok) {
    if (!c || !f || !g || !prm) return CFD_ERROR_INVALID;
    if (f->nx < 3 || f->ny < 3 || (f->nz > 1 && f->nz < 3)) return CFD_ERROR_INVALID;
    cfd_status_t s = ctx_validate_params(c, g, prm);
    if (s != CFD_SUCCESS) return s;
    if (n_steps <= 0) return CFD_SUCCESS;
    const bool need_T = (prm->beta != 0.0) || (prm->alpha > 0.0);
    const bool shell = shell_ok && c->cfg.dirty_faces > 0 && ctx_shell_fits(c, 2);
    const bool same = c->resident && c->res_ptr[0] == f->u && c->res_ptr[1] == f->v &&
                      c->res_ptr[2] == f->w && c->res_ptr[3] == f->p &&
                      c->res_ptr[4] == f->T && (!f->T || c->T);
    const int verify = c->cfg.dirty_verify_interval;
    if (shell && same && verify > 0 && c->hash_ok && c->res_steps % verify == 0) {
        // the guard: the interior of the host arrays must be what the
        // resident steps left there (the device holds the current interior)
        double* host[5];
        double* dev[5];
        const int nf = host_fields(c, f, host, dev);
        unsigned long long h[5], h1[5];
        ctx_host_hash(c, host, nf, false, h);
        ctx_host_hash(c, host, nf, true, h1);
        for (int q = 0; q < nf && q < c->hash_nf; ++q)
            if (h[q] != c->host_hash[q] || h1[q] != c->host_hash1[q]) {
                set_err(CFD_ERROR_INVALID,
                        "projection_hip resident mode: the interior of a host field changed "
                        "since the last step (it is not uploaded); call hip_proj_sync_host, "
                        "write the cells, then hip_proj_mark_host_dirty");
                return CFD_ERROR_INVALID;
            }
    }
    const bool full_up = !(shell && same);
    if (shell && same) {
        double* host[5];
        double* dev[5];
        const int nf = host_fields(c, f, host, dev);
        ST_TRY(ctx_shell_put(c, host, dev, nf, 1));
        if (nf == 5) c->T_dirty = 1;
    } else {
        if ((s = hip_proj_set_field(c, HIP_FIELD_U, f->u)) != CFD_SUCCESS) return s;
        if ((s = hip_proj_set_field(c, HIP_FIELD_V, f->v)) != CFD_SUCCESS) return s;
        if ((s = hip_proj_set_field(c, HIP_FIELD_W, f->w)) != CFD_SUCCESS) return s;
        if ((s = hip_proj_set_field(c, HIP_FIELD_P, f->p)) != CFD_SUCCESS) return s;
        // resident mode: T travels too, so its maximum comes from the device
        if (f->T && (need_T || shell)) {
            if ((s = hip_proj_set_field(c, HIP_FIELD_T, f->T)) != CFD_SUCCESS) return s;
        }
        c->res_steps = 0;
    }
    c->resident = 0;
    c->rho0 = f->rho ? f->rho[0] : 1.0;
    int done = 0;  // steps completed: the reference leaves them applied to field
    for (int it = 0; it < n_steps; ++it) {
        s = step_device_impl(c, g, prm, stats, it);
        if (s != CFD_SUCCESS) break;
        ++done;
    }
    // a failed step (pressure solve unconverged, communication) leaves the
    // device u, v, w, p as the completed steps made them
    const bool energy_T = prm->alpha > 0.0 && f->T && c->T;
    if (s == CFD_SUCCESS || s == CFD_ERROR_DIVERGED || done > 0) {
        ++c->res_steps;
        const int every = c->cfg.dirty_sync_interval;
        const bool shell_down = shell && s == CFD_SUCCESS && !(every > 0 && c->res_steps % every == 0);
        if (!shell_down) c->hash_ok = 0;  // the whole host field changed
        if (shell_down) {
            double* host[5];
            double* dev[5];
            const int nall = host_fields(c, f, host, dev);
            ST_TRY(ctx_shell_get(c, host, dev, energy_T ? nall : 4, 2));
        } else {
            cfd_status_t d = hip_proj_download(c, f);
            if (d != CFD_SUCCESS) return d;
            if (energy_T) {
                d = hip_proj_get_field(c, HIP_FIELD_T, f->T);
                if (d != CFD_SUCCESS) return d;
            }
        }
    } else if (shell) {
        // nothing completed: the device holds the uploaded state; make the
        // whole host field current before handing the error back
        c->hash_ok = 0;
        cfd_status_t d = hip_proj_download(c, f);
        if (d != CFD_SUCCESS) return d;
    }
    if (shell) {
        c->resident = 1;
        c->res_ptr[0] = f->u, c->res_ptr[1] = f->v, c->res_ptr[2] = f->w, c->res_ptr[3] = f->p;
        c->res_ptr[4] = f->T;
        if (verify > 0) {
            // the guard's reference: layer 1 as this step's download left it;
            // the deep interior only after a full transfer (it is untouched
            // on the host otherwise)
            double* host[5];
            double* dev[5];
            const int nf = host_fields(c, f, host, dev);
            if (full_up || !c->hash_ok || c->hash_nf != nf) {
                ctx_host_hash(c, host, nf, false, c->host_hash);
                ctx_host_hash(c, host, nf, true, c->host_hash1);
            } else if (c->res_steps % verify == 0) {
                // layer 1 changes with every shell download: its reference is
                // retaken only before a step that checks (the next one)
                ctx_host_hash(c, host, nf, true, c->host_hash1);
            }
            c->hash_nf = nf;
            c->hash_ok = 1;
        }
    }
    if (s == CFD_SUCCESS && stats && f->T && !shell) {
        // compute_max_temperature (solver_registry.c:52-62) on the host copy,
        // threaded (r06: one core took ~0.1 s of a 512^3 host-buffer step)
        stats->max_temperature = ctx_host_max(f->T, c->nx * c->ny * c->nz);
    }
    return s;
}

extern "C" __attribute__((visibility("hidden"))) cfd_status_t hip_proj_step_iter_internal(
    hip_proj_ctx_t* c, flow_field* f, const grid* g, const ns_solver_params_t* prm,
    ns_solver_stats_t* stats, int n_steps) {
    return host_steps(c, f, g, prm, stats, n_steps, false);
}

extern "C" __attribute__((visibility("hidden"))) cfd_status_t hip_proj_step_host_internal(
    hip_proj_ctx_t* c, flow_field* f, const grid* g, const ns_solver_params_t* prm,
    ns_solver_stats_t* stats) {
    return host_steps(c, f, g, prm, stats, 1, true);
}

extern "C" __attribute__((visibility("hidden"))) int hip_proj_matches_internal(const hip_proj_ctx_t* c,
                                                                    size_t nx, size_t ny,
                                                                    size_t nz) {
    return c && c->nranks == 1 && c->nx == nx && c->ny == ny && c->nzg == nz;
}

extern "C" {

cfd_status_t hip_proj_step(hip_proj_ctx_t* c, flow_field* f, const grid* g,
                           const ns_solver_params_t* prm, ns_solver_stats_t* stats) {
    GroupHostLock hl_(c);
    return host_steps(c, f, g, prm, stats, 1, true);
}

cfd_status_t hip_proj_sync_host(hip_proj_ctx_t* c, flow_field* f) {
    GroupHostLock hl_(c);
    if (!c || !f) return CFD_ERROR_INVALID;
    if (f->nx != c->nx || f->ny != c->ny || f->nz != c->nz) return CFD_ERROR_INVALID;
    ST_TRY(hip_proj_download(c, f));
    if (c->resident && f->T && c->T) ST_TRY(hip_proj_get_field(c, HIP_FIELD_T, f->T));
    c->res_steps = 0;
    c->hash_ok = 0;
    if (c->resident && c->cfg.dirty_verify_interval > 0) {  // the guard's new reference
        double* host[5];
        double* dev[5];
        const int nf = host_fields(c, f, host, dev);
        ctx_host_hash(c, host, nf, false, c->host_hash);
        ctx_host_hash(c, host, nf, true, c->host_hash1);
        c->hash_nf = nf;
        c->hash_ok = 1;
    }
    return CFD_SUCCESS;
}

cfd_status_t hip_proj_poisson_solve(hip_proj_ctx_t* c, int method, double* x, const double* rhs,
                                    double dx, double dy, double dz,
                                    const poisson_solver_params_t* params,
                                    poisson_solver_stats_t* stats) {
    GroupHostLock hl_(c);
    return hip_proj_poisson_solve_ex(c, method, x, rhs, dx, dy, dz, params, stats,
                                     HIP_POISSON_BC_NEUMANN, nullptr);
}

static cfd_status_t poisson_solve_impl(hip_proj_ctx_t* c, int method, double* x,
                                       const double* rhs, double dx, double dy, double dz,
                                       const poisson_solver_params_t* params,
                                       poisson_solver_stats_t* stats);

cfd_status_t hip_proj_poisson_solve_ex(hip_proj_ctx_t* c, int method, double* x,
                                       const double* rhs, double dx, double dy, double dz,
                                       const poisson_solver_params_t* params,
                                       poisson_solver_stats_t* stats, int bc_mode,
                                       const double* bc_values) {
    GroupHostLock hl_(c);
    if (c) c->resident = 0;  // the solve reuses the step's pressure buffers
    if (!c || !x || !rhs) return CFD_ERROR_INVALID;
    if (bc_mode != HIP_POISSON_BC_NEUMANN && bc_mode != HIP_POISSON_BC_NONE &&
        bc_mode != HIP_POISSON_BC_FIXED)
        return CFD_ERROR_INVALID;
    if (bc_mode == HIP_POISSON_BC_FIXED && !bc_values) return CFD_ERROR_INVALID;
    if (bc_mode != HIP_POISSON_BC_NEUMANN && dist(c)) {
        set_err(CFD_ERROR_UNSUPPORTED, "hip_proj_poisson_solve_ex: caller BCs on Z-slabs");
        return CFD_ERROR_UNSUPPORTED;
    }
    HIP_TRY(hipSetDevice(c->device));
    if (bc_mode == HIP_POISSON_BC_FIXED) {
        if (!c->bcfix) ST_TRY(dalloc(c, &c->bcfix, field_elems(c)));
        HIP_TRY(hipMemcpy2DAsync(c->bcfix, c->px * sizeof(double), bc_values,
                                 c->nx * sizeof(double), c->nx * sizeof(double), c->ny * c->nz,
                                 hipMemcpyHostToDevice, c->stream));
    }
    c->poisson_bc = bc_mode;
    const cfd_status_t s = poisson_solve_impl(c, method, x, rhs, dx, dy, dz, params, stats);
    c->poisson_bc = HIP_POISSON_BC_NEUMANN;
    return s;
}

static cfd_status_t poisson_solve_impl(hip_proj_ctx_t* c, int method, double* x,
                                       const double* rhs, double dx, double dy, double dz,
                                       const poisson_solver_params_t* params,
                                       poisson_solver_stats_t* stats) {
    double rel = 1e-6, abs_tol = 1e-10, omega = 0.0;
    int maxit = (method == HIP_POISSON_JACOBI) ? 2000 : 5000, ci = 1;
    if (params) {
        rel = params->tolerance;
        abs_tol = params->absolute_tolerance;
        maxit = params->max_iterations;
        ci = std::max(1, params->check_interval);
        omega = params->omega;
        if (params->preconditioner != POISSON_PRECOND_NONE) {
            set_err(CFD_ERROR_UNSUPPORTED, "hip_proj_poisson_solve: preconditioner not supported");
            return CFD_ERROR_UNSUPPORTED;
        }
    }
    cfd_status_t s = ensure_aux(c, true, method == HIP_POISSON_JACOBI);
    if (s != CFD_SUCCESS) return s;
    HIP_TRY(hipMemcpy2DAsync(c->rhs, c->px * sizeof(double), rhs, c->nx * sizeof(double),
                             c->nx * sizeof(double), c->ny * c->nz, hipMemcpyHostToDevice,
                             c->stream));
    HIP_TRY(hipMemcpy2DAsync(c->pn, c->px * sizeof(double), x, c->nx * sizeof(double),
                             c->nx * sizeof(double), c->ny * c->nz, hipMemcpyHostToDevice,
                             c->stream));
    if (method == HIP_POISSON_JACOBI)
        HIP_TRY(hipMemcpyAsync(c->xt, c->pn, field_elems(c) * sizeof(double),
                               hipMemcpyDeviceToDevice, c->stream));
    if (method == HIP_POISSON_CG) {
        DivCoef dc{};
        s = cg_solve(c, dx, dy, dz, dc, RHS_FROM_ARRAY, rel, abs_tol, maxit, ci, true);
    } else {
        s = relax_solve(c, method, dx, dy, dz, rel, abs_tol, maxit, ci, omega);
    }
    HIP_TRY(hipMemcpy2DAsync(x, c->nx * sizeof(double), c->pn, c->px * sizeof(double),
                             c->nx * sizeof(double), c->ny * c->nz, hipMemcpyDeviceToHost,
                             c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (stats) {
        *stats = c->pstats;
        stats->elapsed_time_ms = 0.0;
    }
    return s;
}

double hip_proj_cg_fixed_iters(hip_proj_ctx_t* c, const double* rhs_host, double dx, double dy,
                               double dz, int iters) {
    if (!rhs_host) return -1.0;
    return hip_proj_cg_fixed_iters_ex(c, rhs_host, dx, dy, dz, iters, 0.0);
}

double hip_proj_cg_fixed_iters_ex(hip_proj_ctx_t* c, const double* rhs_host, double dx,
                                  double dy, double dz, int iters, double rho_over_dt) {
    GroupHostLock hl_(c);
    if (!c || iters <= 0) return -1.0;
    if (hipSetDevice(c->device) != hipSuccess) return -1.0;
    if (!rhs_host && (!c->us || !c->vs || !c->ws)) return -1.0;
    if (rhs_host) {
        if (ensure_aux(c, true, false) != CFD_SUCCESS) return -1.0;
        if (hipMemcpy2DAsync(c->rhs, c->px * sizeof(double), rhs_host, c->nx * sizeof(double),
                             c->nx * sizeof(double), c->ny * c->nz, hipMemcpyHostToDevice,
                             c->stream) != hipSuccess)
            return -1.0;
    }
    hipMemsetAsync(c->pn, 0, field_elems(c) * sizeof(double), c->stream);
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    // rhs_host == NULL: the step's own right-hand side, (rho/dt) div u* of the
    // context's u*, v*, w* (the last step's predictor output), fused into the
    // CG setup exactly as the step forms it
    DivCoef dc{};
    dc.two_dx = 2.0 * dx;
    dc.two_dy = 2.0 * dy;
    dc.inv_2dz = (c->nzg > 1 && dz > 0.0) ? 1.0 / (2.0 * dz) : 0.0;
    dc.rho_over_dt = rho_over_dt;
    hipEventRecord(a, c->stream);
    // zero tolerances: no early exit, exactly `iters` iterations
    cfd_status_t s = cg_solve(c, dx, dy, dz, dc, rhs_host ? RHS_FROM_ARRAY : RHS_FROM_VELOCITY,
                              0.0, 0.0, iters, 1, false);
    (void)s;
    hipEventRecord(b, c->stream);
    hipEventSynchronize(b);
    float ms = 0.f;
    hipEventElapsedTime(&ms, a, b);
    hipEventDestroy(a);
    hipEventDestroy(b);
    return (double)ms;
}

}  // extern "C"
