// ccf.hpp -- one z-march per Chronopoulos-Gear CG iteration (k_ccf): one
// device, 3-D, cg_variant 1 (the single-reduction CG of kernels.hpp k_cc1 /
// k_cc2).
//
// Iteration it, from r_it (buffer R0), p_{it-1}, alpha_it and beta_it:
//   p_it     = r_it + beta_it p_{it-1}              (FIRST: p_0 = r_0)
//   s_it     = A p_it                               (the stencil, not the
//                                                    recurrence w + beta s)
//   r_{it+1} = r_it - alpha_it s_it                 (into buffer R1)
//   w_{it+1} = A r_{it+1};  gamma = (r, r), delta = (w, r) at it + 1
// and every CG_XFOLD-th iteration x += the four pending alpha_j p_j, in
// k_cc1's order. Only r, p (and x on fold iterations) touch HBM: read r_it
// and p_{it-1}, write p_it and r_{it+1}, 32 B per cell (k_cc1 + k_cc2: 72),
// plus the fold's 40 B every fourth iteration. s and w are formed in
// registers from p and r one and two cells out, so a tile carries a two-cell
// halo and computes s and w on the fly instead of storing and re-reading
// them; A = -lap7 with zero walls, as k_cc2.
//
// The iterates equal k_cc1 / k_cc2's up to rounding (s is A p_it itself, not
// its recurrence; the dot products are summed per tile), which is what the
// single-reduction tests gate against textbook CG (iterations +-2).
//
// Pipeline. Step q of the z march, per lane (an x pair of one row):
//   a: p_it at plane q + 2 from the loaded r_it, p_{it-1}  (published in LDS)
//   b: s_it and r_{it+1} at plane q + 1: in-plane p from LDS, z from the
//      lane's ring; p_it and r_{it+1} stored there (published in LDS)
//   c: w_{it+1} at plane q and the two dot products
// one barrier per step; LDS holds p_it and r_{it+1} planes by parity.
//
// Tiles: 32 x pairs (64 columns) x 32 rows, 1024 threads, lane l of wave w
// owns pair l % 32 of rows w and w + 16; 60 x 28 cells written per tile.
#pragma once

#include "kernels.hpp"

namespace cfdhip {

// planes of r_it, p_{it-1} in flight ahead of their use (1 or 2; the
// build's -DCFD_CCF_AHEAD selects it for A/B runs)
#ifndef CFD_CCF_AHEAD
#define CFD_CCF_AHEAD 2
#endif
constexpr int CCF_AHEAD = CFD_CCF_AHEAD;
static_assert(CCF_AHEAD == 1 || CCF_AHEAD == 2, "k_ccf prefetch depth");
// 1: stage c's LDS reads issued right after the barrier, ahead of stages a
// and b (-DCFD_CCF_CFIRST=1); 0: after stage b. Measured equal at 512^3
// (1.2616 vs 1.2610 ms per iteration, profiles/r05f_ccf_cfirst_ab.jsonl),
// so the default keeps the 10 VGPRs the early reads hold (the fold form
// would sit at 126 of 128)
#ifndef CFD_CCF_CFIRST
#define CFD_CCF_CFIRST 0
#endif
constexpr bool CCF_CFIRST = CFD_CCF_CFIRST != 0;
// Diagnostic builds only (wrong results; never the product): -DCFD_CCF_DIAG=1
// every load reads plane 0 (cache-resident) and no store reaches memory;
// 2: no in-plane stencil (no LDS reads, no stencil arithmetic). Both ignore
// the done flag so that every launch runs its whole march. They split the
// iteration's time into its memory and its synchronised-compute parts.
#ifndef CFD_CCF_DIAG
#define CFD_CCF_DIAG 0
#endif
constexpr int CCF_DIAG = CFD_CCF_DIAG;
// non-temporal stores of p_it, r_{it+1} and x (-DCFD_CCF_NTST=1, A/B builds)
// (r05: 1.132 -> 1.085 ms per iteration at 512^3, profiles/r05l_ccf_ntst_ab.jsonl:
// p, r and x are next read a whole iteration later, far beyond the caches,
// and written through they no longer displace the halo lines the
// neighbouring tiles re-read). -DCFD_CCF_NTST=0: plain stores
#ifndef CFD_CCF_NTST
#define CFD_CCF_NTST 1
#endif
constexpr bool CCF_NTST = CFD_CCF_NTST != 0;
// the stores' full cache-policy bits (A/B builds: -DCFD_CCF_STAUX=N)
#ifndef CFD_CCF_STAUX
#define CFD_CCF_STAUX (CFD_CCF_NTST ? 2 : 0)
#endif
constexpr int CCF_STAUX = CFD_CCF_STAUX;
// the march's r_it / p_{it-1} loads' cache-policy bits (A/B: -DCFD_CCF_LDAUX=N)
#ifndef CFD_CCF_LDAUX
#define CFD_CCF_LDAUX 0
#endif
constexpr int CCF_LDAUX = CFD_CCF_LDAUX;
// non-temporal loads of the fold operands (x, p_{it-3..it-1}: read once, by
// the storing lanes only) with -DCFD_CCF_NTFOLD=1: measured slower (1.188 vs
// 1.156 ms per iteration, profiles/r05m_ccf_ntfold_ab.jsonl), so plain loads
#ifndef CFD_CCF_NTFOLD
#define CFD_CCF_NTFOLD 0
#endif
constexpr bool CCF_NTFOLD = CFD_CCF_NTFOLD != 0;
constexpr int CCF_TC = 32;  // x pairs per tile row
constexpr int CCF_TR = 32;  // tile rows
constexpr int CCF_OX = 60;  // columns written per tile
constexpr int CCF_OY = 28;  // rows written per tile
// LDS plane: rows of 2 padded halves (.x cells, then .y cells) so that an x
// neighbour (one double of the adjacent lane) is a conflict-free 8-B read
constexpr int CCF_LP = CCF_TC + 2;
constexpr int CCF_LR = 2 * CCF_LP;
constexpr int CCF_LS = (CCF_TR + 2) * CCF_LR;
struct CcfLds {
    double pl[4][CCF_LS];  // 0-1: p_it by plane parity, 2-3: r_{it+1} by parity
    double sh[32];
    int flag;
};

// NOC (Z-slabs): no stage c; p_it is also stored on the slab's halo planes
// (the next iteration forms p there from the exchanged r), and the r halo +
// k_cc2<..., WST = false> complete the iteration with its one reduction.
// That is the march of a slab's two edge planes (kmode 1), and of a whole
// slab of < 3 planes. The interior planes of a slab (kmode 2) run the full
// march (!NOC): stage c covers planes k0 + 1 .. k1 - 2, whose r_{it+1}
// neighbours the march forms itself (the edge planes' r_{it+1} from the same
// operands as the edge launch), and its partial dot products join the edge
// planes' k_cc2 launch (g.part_ofs / part_total, dist = 1).
template <bool FIRST, bool FOLD, bool NOC = false>
static __global__ __launch_bounds__(1024, 4) void k_ccf(
    SGeo g, Lap Lp, const double* __restrict__ R0, double* __restrict__ R1,
    const double* __restrict__ Po, double* __restrict__ Pn, PPrev pv, double* __restrict__ x,
    CgState* st, double* partials, unsigned* counter, int it, int xmap, int dist, double* dsum,
    Mbox* mb, unsigned long long* clk) {
    // (a fold step reads p_{it-1} from the po ring, which FIRST never loads)
    static_assert(!(FIRST && FOLD), "k_ccf: no fold in the first iteration");
    __shared__ CcfLds L;
    if (CCF_DIAG == 0 && st->done) return;
    // clock sample (clk != nullptr on one launch in eight while the context
    // times its kernels, hip_proj_get_clock_sample): wave 0 stamps the shader
    // clock (s_memtime) and the 100 MHz constant clock (s_memrealtime) at the
    // workgroup's start and end; uniform branch, no stamp in other launches
    unsigned long long clk_t0 = 0, clk_r0 = 0;
    if (clk != nullptr && threadIdx.x < 64) {
        clk_t0 = __builtin_amdgcn_s_memtime();
        clk_r0 = __builtin_amdgcn_s_memrealtime();
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the stamps are back
    }
    const double a = st->alpha[it % CG_XFOLD];
    const double ma = -a;
    const double beta = FIRST ? 0.0 : st->beta;
    double aq[CG_XFOLD - 1];
#pragma unroll
    for (int q = 0; q < CG_XFOLD - 1; ++q)
        aq[q] = FOLD ? st->alpha[(it + 1 + q) % CG_XFOLD] : 0.0;  // alpha_{it-3+q}
    const int t = xmap ? xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int tx = t % g.tiles_x;
    const int rest = t / g.tiles_x;
    const int ty = rest % g.tiles_y;
    const int tz = rest / g.tiles_y;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int c = lane & 31;
    const int r = w + 16 * (lane >> 5);
    const int i0 = tx * CCF_OX - 2 + 2 * c;  // even; the pair is (i0, i0 + 1)
    const int j = ty * CCF_OY - 2 + r;
    // kmode 1 (Z-slabs, NOC): the slab's two edge planes (tz 0 -> k0, tz 1 ->
    // k1 - 1); kmode 2: the planes [kt0, kt1) between them
    int kb, ke;
    if (g.kmode == 1) {
        kb = (tz == 0) ? g.k0 : g.k1 - 1;
        ke = kb + 1;
    } else {
        const int kt0 = (g.kmode == 2) ? g.kt0 : g.k0;
        const int kt1 = (g.kmode == 2) ? g.kt1 : g.k1;
        if (tz < g.nz1) {
            kb = kt0 + tz * g.kc;
            ke = min(kb + g.kc, kt1);
        } else {  // tail layers: shorter runs (dispatched last)
            kb = min(kt0 + g.nz1 * g.kc + (tz - g.nz1) * g.kc2, kt1);
            ke = min(kb + g.kc2, kt1);
        }
    }
    const bool jin = j >= 1 && j <= g.ny - 2;
    const bool in0 = jin && i0 >= 1 && i0 <= g.nx - 2;
    const bool in1 = jin && i0 + 1 >= 1 && i0 + 1 <= g.nx - 2;
    // written / reduced: pairs 1..30 of rows 2..29 that hold a grid pair
    const bool own = c >= 1 && c <= CCF_TC - 2 && r >= 2 && r <= CCF_TR - 3;
    const bool wr = own && jin && i0 >= 0 && i0 < g.nx;
    // loads from always-valid addresses: outside the grid they hold other
    // cells' values, which only feed cells outside the interior (masked)
    const int ic = i0 < 0 ? 0 : (i0 < g.nx ? i0 : g.nx - 2 - ((g.nx - 2) & 1));
    const int col = max(min(j, g.ny - 1), 0) * (int)g.px + ic;
    auto plane = [&](int k) -> long long {
        return CCF_DIAG == 1 ? 0LL : (long long)min(max(k, 0), g.nz - 1) * g.ps;
    };
    // LDS: one base at the lane's cell minus one row and one column of the
    // padded plane, so every operand is a non-negative immediate offset
    double* const Lb = &L.pl[0][r * CCF_LR + c];
    constexpr int OWX = CCF_LR + 1, OWY = CCF_LR + 1 + CCF_LP;
    constexpr int LFo = CCF_LR + CCF_LP, RTo = CCF_LR + 2;  // pair c-1 .y, pair c+1 .x
    constexpr int DNX = 1, DNY = 1 + CCF_LP, UPX = 2 * CCF_LR + 1, UPY = 2 * CCF_LR + 1 + CCF_LP;
    auto lrd = [&](int pl, int d) __attribute__((always_inline)) -> double {
        // keeps each read a ds_read_b64 (see rb2.hpp)
        __builtin_amdgcn_sched_barrier(0x7ff);
        return Lb[pl * CCF_LS + d];
    };
    auto lput = [&](int pl, double2 v) __attribute__((always_inline)) {
        Lb[pl * CCF_LS + OWX] = v.x;
        Lb[pl * CCF_LS + OWY] = v.y;
    };
    // zero the pads (never written; halo lanes read them)
    for (int e = threadIdx.x; e < 4 * CCF_LS; e += 1024) {
        const int q = e % CCF_LS;
        const int row = q / CCF_LR, cc = q % CCF_LP;
        if (row == 0 || row == CCF_TR + 1 || cc == 0 || cc == CCF_LP - 1) L.pl[e / CCF_LS][q] = 0.0;
    }
    // the six in-plane neighbours of the pair in LDS plane pl
    struct Nb {
        double lf, rt, dx, dy, ux, uy;
    };
    auto nbrs = [&](int pl) __attribute__((always_inline)) -> Nb {
        Nb n;
        n.lf = lrd(pl, LFo);
        n.rt = lrd(pl, RTo);
        n.dx = lrd(pl, DNX);
        n.dy = lrd(pl, DNY);
        n.ux = lrd(pl, UPX);
        n.uy = lrd(pl, UPY);
        return n;
    };
    // -A v at the pair from its own pair (v), its z neighbours and the in-plane ones
    auto stencil_n = [&](const Nb& n, double2 v, double2 zm, double2 zp, double2& out)
                         __attribute__((always_inline)) {
        out.x = -lap7(Lp, v.x, n.lf, v.y, n.dx, n.ux, zm.x, zp.x);
        out.y = -lap7(Lp, v.y, v.x, n.rt, n.dy, n.uy, zm.y, zp.y);
    };
    auto stencil = [&](int pl, double2 v, double2 zm, double2 zp, double2& out)
                       __attribute__((always_inline)) {
        if constexpr (CCF_DIAG == 2) {
            out.x = v.x + zm.x + zp.x;
            out.y = v.y + zm.y + zp.y;
        } else {
            stencil_n(nbrs(pl), v, zm, zp, out);
        }
    };
    const int q0 = kb - 4;  // steps q0 .. ke - 1 (see the header)
    const int nsteps = ke - kb + 4;
    // rings (slot of plane p at step q: (p - q0) & 3): r_it, p_{it-1} (loaded
    // one step ahead), p_it, r_{it+1}; fold operands (x, p_{it-3..it-1}) by parity
    double2 rr[4], po[4], pn[4], rn[4];
    double2 fx[2], f0[2], f1[2];
    const double2 zero = make_double2(0.0, 0.0);
#pragma unroll
    for (int s = 0; s < 4; ++s) pn[s] = rn[s] = po[s] = rr[s] = zero;
    fx[0] = fx[1] = f0[0] = f0[1] = f1[0] = f1[1] = zero;
    // (r_it of plane q0 + 1 = kb - 3 only feeds r_{it+1} there, never used)
    // (the fold operands of plane q0 + 1 = kb - 3 are never stored: no load)
    // Each prologue load is followed by dropped stores in the place of a
    // step's stores, so that the first steps' waits for these loads count the
    // same ops as every later step's (the loop header joins both paths).
    auto pro = [&](int k) __attribute__((always_inline)) {
        const int s = (k - q0) & 3;
        rr[s] = ld2ba<CCF_LDAUX>(R0 + plane(k), g.ps, col * 8);
        if (!FIRST) po[s] = ld2ba<CCF_LDAUX>(Po + plane(k), g.ps, col * 8);
        st2b<false>(Pn, g.ps, ST_NOSTORE, zero);
        st2b<false>(R1, g.ps, ST_NOSTORE, zero);
        if (FOLD) st2b<false>(x, g.ps, ST_NOSTORE, zero);
        __builtin_amdgcn_sched_barrier(0);
    };
    // AHEAD 1: plane q0 + 2 here, step q loads q + 3; AHEAD 2: planes q0 + 2
    // and q0 + 3 here, step q loads q + 4 (into the slot of plane q, which no
    // step from q on reads: stage a reads q + 2, stage b q + 1)
    rr[2] = po[2] = zero;
    pro(q0 + 2);
    if (CCF_AHEAD == 2) pro(q0 + 3);
    double accg = 0.0, accd = 0.0;
    auto step = [&](auto Pc, int q) __attribute__((always_inline)) {
        constexpr int P = decltype(Pc)::value;
        constexpr int S0 = P & 3, S1 = (P + 1) & 3, S2 = (P + 2) & 3, S3 = (P + 3) & 3;
        constexpr int SM = (P + 3) & 3;  // plane q - 1 (r_{it+1})
        constexpr int F1 = (P + 1) & 1, F2 = P & 1;  // fold slots of planes q + 1, q + 2
        constexpr int LPR = (P + 1) & 1, LPW = P & 1;        // p_it planes q + 1 (read), q + 2
        constexpr int LRR = 2 + (P & 1), LRW = 2 + ((P + 1) & 1);  // r_{it+1} q (read), q + 1
        // prefetch plane q + 2 + AHEAD (r_it, p_{it-1}) and the fold operands
        // of q + 2 (r04, with the branch-conservative waits below: two steps
        // ahead measured slower, 1.32 vs 1.27 ms per iteration at 512^3,
        // profiles/r04_ccf_prefetch2_cg_variant.jsonl)
        // Memory ops of a step in a fixed order with no branch around any of
        // them: the loads of plane q + 2 + AHEAD (r_it, p_{it-1}) and the fold
        // operands of plane q + 2 first, then (end of the step) the stores of
        // plane q + 1. With every step issuing the same ops the compiler's
        // vmcnt count is exact, and the wait before the next barrier (for
        // these loads) leaves the stores issued after them in flight; a load
        // or store under a branch makes the count at the join conservative,
        // and that wait then also waits for the stores just issued.
        __builtin_amdgcn_sched_barrier(0);
        {
            // plane q + AHEAD + 2; the planes past ke + 1 (the last steps')
            // no step reads: those loads are dropped (offset past the plane:
            // no memory access; the unused edge-plane reads cost 1.157 vs 1.119
            // ms per iteration at 512^3, profiles/r04_ccf_edge_plane_loads_ab.jsonl)
            constexpr int SL = (CCF_AHEAD == 2) ? S0 : S3;
            const int ql = q + CCF_AHEAD + 2;
            const long long pbl = plane(ql);
            const int ol = (ql <= ke + 1) ? col * 8 : ST_NOSTORE;
            rr[SL] = ld2ba<CCF_LDAUX>(R0 + pbl, g.ps, ol);
            if (!FIRST) po[SL] = ld2ba<CCF_LDAUX>(Po + pbl, g.ps, ol);
        }
        if (FOLD) {
            // only the lanes and planes that store x read its operands (the
            // halo lanes' and planes' loads would be re-fetched lines): 1.123
            // vs 1.159 ms per iteration at 512^3, profiles/r04_ccf_fold_owned_loads_ab.jsonl
            const long long pb2 = plane(q + 2);
            const int o2 = (wr && q + 2 >= kb && q + 2 < ke) ? col * 8 : ST_NOSTORE;
            // (p_{it-1}, the fold's third pending direction, is the march's
            // own p_{it-1} ring (po), still holding plane q + 1 when step q
            // folds it: no load of its own, r05)
            fx[F2] = ld2b<CCF_NTFOLD>(x + pb2, g.ps, o2);
            f0[F2] = ld2b<CCF_NTFOLD>(pv.q[0] + pb2, g.ps, o2);
            f1[F2] = ld2b<CCF_NTFOLD>(pv.q[1] + pb2, g.ps, o2);
        }
        __builtin_amdgcn_sched_barrier(0);
        __syncthreads();
        // stage c's in-plane operands (r_{it+1} of plane q, published last
        // step) first: their LDS latency then overlaps stages a and b
        Nb nc{};
        if constexpr (!NOC && CCF_CFIRST) nc = nbrs(LRR);
        // ---- a: p_it at q + 2 ----
        const double2 p2 = FIRST ? rr[S2] : fma2p(rr[S2], beta, po[S2]);
        pn[S2] = p2;
        // ---- b: s_it, r_{it+1} at q + 1 ----
        double2 s;
        stencil(LPR, pn[S1], pn[S0], p2, s);
        const int qb = q + 1;
        const bool kbin = qb >= 1 && qb <= g.nz - 2;
        const double2 rv = rr[S1];
        const double2 r1 = make_double2((kbin && in0) ? rv.x + ma * s.x : 0.0,
                                        (kbin && in1) ? rv.y + ma * s.y : 0.0);
        rn[S1] = r1;
        if constexpr (!CCF_CFIRST) __builtin_amdgcn_sched_barrier(0);
        // ---- c: w_{it+1} at q, the dot products ----
        if constexpr (!NOC) {
            double2 wv;
            if constexpr (CCF_CFIRST) stencil_n(nc, rn[S0], rn[SM], r1, wv);
            else stencil(LRR, rn[S0], rn[SM], r1, wv);
            if (q >= kb && own) {
                const double2 rc = rn[S0];
                if (in0) {
                    accg += rc.x * rc.x;
                    accd += wv.x * rc.x;
                }
                if (in1) {
                    accg += rc.y * rc.y;
                    accd += wv.y * rc.y;
                }
            }
        }
        // ---- publish p_it (q + 2), r_{it+1} (q + 1); stores at q + 1 ----
        lput(LPW, p2);
        if constexpr (!NOC) lput(LRW, r1);
        {
            const bool qown = qb >= kb && qb < ke;
            const int bo = (qown && wr && CCF_DIAG != 1) ? col * 8 : ST_NOSTORE;
            // NOC: p also on the halo plane below / above the slab's owned planes
            const bool qhalo = NOC && ((qb == kb - 1 && kb == g.k0) || (qb == ke && ke == g.k1));
            const int bp = ((qown || qhalo) && wr && CCF_DIAG != 1) ? col * 8 : ST_NOSTORE;
            const long long pb = plane(qb);
            const double2 p1 = pn[S1];
            st2ba<CCF_STAUX>(Pn + pb, g.ps, bp, make_double2(in0 ? p1.x : 0.0, in1 ? p1.y : 0.0));
            st2ba<CCF_STAUX>(R1 + pb, g.ps, bo, r1);
            if (FOLD) {
                const double2 xo = fx[F1], qa = f0[F1], qq = f1[F1], qc = po[S1];
                double2 xw;
                xw.x = in0 ? (((xo.x + aq[0] * qa.x) + aq[1] * qq.x) + aq[2] * qc.x) + a * p1.x
                           : xo.x;
                xw.y = in1 ? (((xo.y + aq[0] * qa.y) + aq[1] * qq.y) + aq[2] * qc.y) + a * p1.y
                           : xo.y;
                st2ba<CCF_STAUX>(x + pb, g.ps, bo, xw);
            }
        }
        __builtin_amdgcn_sched_barrier(0);
    };
    int n = 0;
    for (; n + 3 < nsteps; n += 4) {
        step(IntC<0>{}, q0 + n);
        step(IntC<1>{}, q0 + n + 1);
        step(IntC<2>{}, q0 + n + 2);
        step(IntC<3>{}, q0 + n + 3);
    }
    if (n < nsteps) step(IntC<0>{}, q0 + n);
    if (n + 1 < nsteps) step(IntC<1>{}, q0 + n + 1);
    if (n + 2 < nsteps) step(IntC<2>{}, q0 + n + 2);
    if (clk != nullptr && threadIdx.x < 64) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime();
        const unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
        __builtin_amdgcn_s_waitcnt(0xC07F);
        if (threadIdx.x == 0) {  // vector atomics (no-return adds)
            atomicAdd(&clk[0], t1 - clk_t0);
            atomicAdd(&clk[1], r1 - clk_r0);
            atomicAdd(&clk[2], 1ull);
        }
    }
    if constexpr (NOC) return;  // k_cc2 reduces
    // ---- one reduction: (gamma, delta) of iteration it + 1 ----
    accg = wave_sum(accg);
    accd = wave_sum(accd);
    __syncthreads();
    if (lane == 0) {
        L.sh[w] = accg;
        L.sh[16 + w] = accd;
    }
    __syncthreads();
    double bg = 0.0, bd = 0.0;
    if (threadIdx.x == 0)
        for (int v = 0; v < 16; ++v) {
            bg += L.sh[v];
            bd += L.sh[16 + v];
        }
    double tg, td;
    double* shs = &L.pl[0][0];
    // g.part_total > 0: the interior planes of a Z-slab, whose reduction the
    // edge planes' k_cc2 launch after the r halo completes (kernels.hpp)
    if (grid_sum2_last<1024>(bg, bd, partials, counter, shs, &L.flag, tg, td,
                             (unsigned)g.part_ofs, (unsigned)g.part_total) &&
        threadIdx.x == 0)
        cc_reduce_finish(st, tg, td, it, false, dist != 0, mb, dsum);
}

}  // namespace cfdhip
