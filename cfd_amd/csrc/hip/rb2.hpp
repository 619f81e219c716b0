// rb2.hpp -- two Red-Black SOR iterations per z-march (k_rb2): one device,
// 3-D, Neumann BC folded into the stores (linear_solver_redblack.c:80-147
// twice, with the BC of :139 between and after the iterations), driven by the
// common loop's L-inf test (linear_solver.c:397-485) on both iterates.
//
// Why: one RB-SOR iteration per sweep (k_rb1) moves 24 B/cell and runs at
// about the HBM rate its traffic allows; two iterations per sweep read X and
// rhs and write the iterate once per two iterations (12 B/cell/iteration).
//
// Pipeline. Step q of the march forms, for the tile's columns,
//   S1  R1_{q+1}: the first colour ("red", (i+j+k) odd) of X updated
//   S2  Y1_q    : the second colour from R1          (iteration s+1 done)
//   S3  R2_{q-1}: the first colour of Y1' (Y1 after its Neumann BC)
//   S4  Y2_{q-2}: the second colour from R2          (iteration s+2 done)
// with the L-inf residual of X (at plane q+1, beside S1) and of Y1' (at
// plane q-1, beside S3). Every in-plane operand of a stage comes from the
// plane the previous step published in LDS, every z operand from the lane's
// own registers, so one barrier per step suffices. In step q all four
// updates touch the same component of the lane's x pair (the colour pattern
// is wave-uniform, as in k_rb1), and each stage's plane is stored in LDS as
// ONE colour: R1 and R2 keep their first-colour cells, Y1 its second-colour
// cells; the other colour of those planes is the previous stage's.
//
// Tiles: 32 x pairs (64 columns) x 32 rows, 1024 threads; lane l of wave w
// owns pair l % 32 of rows w and w + 16 (same parity). Validity shrinks by
// one cell per stage, so 56 x 24 cells are written per 64 x 32 loaded (1.52x,
// against k_rb1's 1.38x for ONE iteration).
//
// Neumann BC between the iterations: the reference sets every boundary cell
// of Y1 to its inward neighbour, and for the cells next to a face that
// neighbour IS the cell whose stencil is evaluated; S3, S4 and the residual
// of Y1' therefore read the centre value in place of a face cell (x / y
// faces per lane, z faces per plane). Edge and corner cells are no interior
// cell's neighbours. Y2 is stored with its boundary shell folded in as k_rb1
// does. Y1 is not stored: when the loop stops on it, the host recomputes it
// with one k_rb1 sweep from X (which this kernel leaves intact).
//
// APX (the product form): the SOR divisions by dx^2 / dy^2 take divc's fast
// path without its per-division range test, and the residuals are evaluated
// as sx/dx^2 + sy/dy^2 + sz/dz^2 - 2c(...) - b with FMAs and the SOR's own
// neighbour sums, a few operations instead of the reference's division form.
// Both are certified per sweep, so every decision and every stored value is
// the reference's bit for bit:
//  - range: the fast quotient is the correctly rounded a/d whenever |a/d| is
//    in [2^-900, 2^900] or a = +-0 (divc / divz, tools/divc_check.c). The
//    sweep certifies M = max |v| <= 2^800 over every value it reads or
//    writes (so every neighbour sum is at most 2^801; 1 <= 1/d <= 2^60 is
//    checked on the host); a sweep that fails it stops the loop
//    (ST_RB2_UNCERT) and the host reruns its iterations with k_rb1. The
//    lower end is tested per update (rb2_sorc): a wave holding a nonzero
//    neighbour sum below 2^-900 recomputes that update with divc.
//  - residuals: both the reference's value and the approximation are within
//    8u (4 M K + B) of the exact residual (u = 2^-53, M = max |v| over the
//    sweep's values, K = 1/dx^2 + 1/dy^2 + 1/dz^2, B = max |rhs|); the loop
//    decides only when the approximate maximum is more than E = 32u (4 M K +
//    B) from the threshold, and otherwise stops (ST_RB2_AMBIG) for the host
//    to compute that iterate's exact residual and resume with it. The final
//    iterate's reported residual is always recomputed exactly by the host.
// APX = false evaluates everything in the reference's form (divc with its
// range test, res1) and decides exactly: the bitwise baseline of the APX form.
#pragma once

#include "kernels.hpp"

namespace cfdhip {

#ifndef CFD_RB2_DIAG
#define CFD_RB2_DIAG 0
#endif
constexpr bool RB2_DIAG = CFD_RB2_DIAG != 0;
constexpr int RB2_TC = 32;   // x pairs per tile row
constexpr int RB2_TR = 32;   // tile rows (two per wave)
constexpr int RB2_OX = 56;   // columns written per tile
constexpr int RB2_OY = 24;   // rows written per tile
constexpr int ST_RB2_AMBIG = 10;   // a decision within the approximation bound (host resolves)
constexpr int ST_RB2_UNCERT = 11;  // a value outside the certified range (host reruns exactly)

struct Rb2Coef {
    RelaxCoef rc;
    double k2;   // 2 (RN(1/dx2) + RN(1/dy2) + inv_dz2): the centre weight of the approximation
    // slow: a wave recomputes an SOR update in the reference's arithmetic
    // when the smaller |neighbour sum| of one of its lanes is below it
    // (2^-900; test knob CFD_HIP_RB2_TEST=3: 1e300, every update)
    double slow;
    double nif;  // -inv_factor: pn = t * nif is RN(-t * inv_factor) bit for bit (RN is odd)
};

// The sweep's decision constants, read by the last workgroup only. They sit
// in device memory (k_rb2_dec_init, once per solve) rather than in the
// kernel's arguments: an argument stays in a scalar register across the
// whole march, and the march's scalar registers are full (the compiler then
// spills loop operands and reloads them with v_readlane every step).
struct Rb2Dec {
    double kb;      // 1/dx2 + 1/dy2 + inv_dz2 (error bound)
    // test knobs (CFD_HIP_RB2_TEST): escale multiplies the residual bound
    // (1e300: every decision ambiguous); mlim is the largest certified
    // |value| (2^800; 0: every sweep uncertified)
    double escale, mlim;
};

// LDS of one k_rb2 workgroup (148 KB): X by plane parity, and the one-colour
// planes of R1, Y1, R2 by plane mod 4 -- the in-plane operands of every
// stage and the lane's own z ring (kept here rather than in registers: the
// 16-wave workgroup caps a wave at 128 VGPRs). Every plane has a one-cell
// pad around the tile (never written: it feeds halo lanes only), so a lane
// reaches its four neighbours at fixed offsets from ONE address, which
// keeps the address registers to a couple instead of one per neighbour.
constexpr int RB2_LP = RB2_TC + 2;             // padded row (doubles)
constexpr int RB2_LS = (RB2_TR + 2) * RB2_LP;  // padded one-colour plane
// planes: 0-3 X (slot * 2 + component), 4-7 R1, 8-11 Y1, 12-15 R2 (by slot)
constexpr int RB2_PX = 0, RB2_PR1 = 4, RB2_PY1 = 8, RB2_PR2 = 12;
struct Rb2Lds {
    double pl[16][RB2_LS];
    double sh[4][16];
    int flag;
};

// a / d for the constant divisors, fast path only (APX: certified per sweep)
// or divc with its range test
template <bool APX>
__device__ __forceinline__ double rb2_div(double a, double d, double r) {
    if constexpr (APX) {
        const double q = a * r;
        return fma(-fma(q, d, -a), r, q);  // divz's form: keeps the sign of a zero a
    } else {
        return divc(a, d, r);
    }
}

// One SOR update from the neighbour sums sx = right + left, sy = up + down,
// sz = above + below (linear_solver_redblack.c:103-112 order, as sor1)
// (pn = -t / factor as t times the negated reciprocal: the same rounding, one
// instruction fewer than a negation and a product)
template <bool APX>
__device__ __forceinline__ double rb2_sor(const RelaxCoef& rc, double nif, double vc, double sx,
                                          double sy, double sz, double vb,
                                          double* tout = nullptr) {
    const double t = vb - rb2_div<APX>(sx, rc.dx2, rc.rdx2) - rb2_div<APX>(sy, rc.dy2, rc.rdy2) -
                     sz * rc.inv_dz2;
    if (tout) *tout = t;
    const double pn = t * nif;
    return vc + rc.omega * (pn - vc);
}

// the approximate residual of the cell an update just touched, from the
// update's own t = b - sx/dx^2 - sy/dy^2 - sz/dz^2 (lap - b = -t - k2 c):
// one FMA, within the same bound as rb2_res_apx. Signed (its negation, as
// fma rounds oddly): the running maximum takes |.| in its own instruction
__device__ __forceinline__ double rb2_res_from_t(const Rb2Coef& cf, double c, double t) {
    return fma(c, cf.k2, t);
}

// approximate lap(x) - rhs from the neighbour sums (see the header), signed
__device__ __forceinline__ double rb2_res_apx(const Rb2Coef& cf, double c, double sx, double sy,
                                              double sz, double b) {
    return fma(sx, cf.rc.rdx2, fma(sy, cf.rc.rdy2, fma(sz, cf.rc.inv_dz2, fma(c, -cf.k2, -b))));
}

// the binary exponent of v as frexp gives it (0 for zero)
__device__ __forceinline__ int rb2_exp(double v) { return __builtin_amdgcn_frexp_exp(v); }

// running maxima in one instruction: max(m, a) and max(m, |a|) (a quiet NaN
// operand is dropped, as the compare-and-select form drops it); written out
// because fmax on a loop-carried value costs a canonicalize per use
__device__ __forceinline__ double rb2_vmax(double m, double a) {
    double r;
    asm("v_max_f64 %0, %1, %2" : "=v"(r) : "v"(m), "v"(a));
    return r;
}
__device__ __forceinline__ double rb2_vmax_abs(double m, double a) {
    double r;
    asm("v_max_f64 %0, %1, |%2|" : "=v"(r) : "v"(m), "v"(a));
    return r;
}
__device__ __forceinline__ double rb2_max_abs2(double a, double b) {
    double r;
    asm("v_max_f64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

__device__ __forceinline__ double rb2_min_abs2(double a, double b) {
    double r;
    asm("v_min_f64 %0, |%1|, |%2|" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

// One SOR update, APX: the fast divisions, with their range test folded into
// ONE wave-uniform branch per update. The fast quotient is correctly rounded
// for |a r| in [2^-900, 2^900] or a = 0 (divz); the sweep certifies |v| <=
// 2^800 for every value (so |sx|, |sy| <= 2^801, and 1 <= 1/d^2 <= 2^60 is
// checked on the host), and here a wave in which some neighbour sum has
// |sum| < 2^-900 (the zero-valued front of a solve from a zero guess leaves
// such values) recomputes the update with divc. The test is min(|sx|, |sy|)
// < 2^-900: two instructions (r05; the binary-exponent form, two frexp + min
// + compare, also let exact zeros take the fast path, which is exact for
// them, and costs two more per update). Either way the value is the
// reference's.
template <bool APX>
__device__ __forceinline__ double rb2_sorc(const Rb2Coef& cf, double vc, double sx, double sy,
                                           double sz, double vb, double* tout = nullptr) {
    if constexpr (!APX) {
        return rb2_sor<false>(cf.rc, cf.nif, vc, sx, sy, sz, vb, tout);
    } else {
        double v = rb2_sor<true>(cf.rc, cf.nif, vc, sx, sy, sz, vb, tout);
        if (__builtin_amdgcn_ballot_w64(rb2_min_abs2(sx, sy) < cf.slow) != 0)
            v = rb2_sor<false>(cf.rc, cf.nif, vc, sx, sy, sz, vb, tout);
        return v;
    }
}

// The decision of the common loop for iterate `it` >= 1 (check_interval 1)
// from an approximate residual maximum m with bound E; false = ambiguous.
__device__ __forceinline__ bool rb2_decide(RxState* st, double m, double E, int it) {
    const double thr = fmax(st->tol, st->abs_tol);  // m < tol || m < abs_tol
    bool conv;
    if (st->ovr_it == it) {
        m = st->ovr_m;
        conv = m < thr;
        st->res_exact = 1;
    } else if (m + E < thr) {
        conv = true;
        st->res_exact = 0;
    } else if (m - E >= thr) {
        conv = false;
        st->res_exact = 0;
    } else {
        st->done = 1;
        st->status = ST_RB2_AMBIG;
        st->res_it = it;
        return false;
    }
    st->res = m;
    if (conv) {
        st->done = 1;
        st->status = ST_CONVERGED;
        st->iterations = it;
        st->res_it = it;
    } else if (it >= st->max_iter) {
        st->done = 1;
        st->status = ST_MAX_ITER;
        st->iterations = st->max_iter + 1;
        st->res_it = it;
    }
    return true;
}

// X = iterate s (s >= 1, its boundary shell Neumann), Y <- iterate s + 2.
// X's own values are certified by k_rb2_xmax before the sweeps that need it
// (certx: the first sweep after a k_rb1 sweep), not in the march.
// The march of one k_rb2 tile (see the header); BND: the tile touches the
// faces (per-lane face, range and shell logic), else all of it folds away.
template <bool APX, int FL, bool BND>
__device__ __forceinline__ void rb2_march(Rb2Lds& L, const SGeo& g, const Rb2Coef& cf,
                                          const double* __restrict__ X, double* __restrict__ Y,
                                          const double* __restrict__ rhs, int c, int r, int i0,
                                          int j, int kb, int ke, double& mX,
                                          double& mY, double& M) {
    const RelaxCoef& rc = cf.rc;
    // LDS addressing: two per-lane bases (planes 0-7 and 8-15), each at the
    // lane's cell minus one row and one column, so every operand is a
    // non-negative immediate offset below 64 KB (a negative or larger offset
    // makes the compiler keep one address register per access)
    double* const Lb0 = &L.pl[0][r * RB2_LP + c];
    double* const Lb1 = &L.pl[8][r * RB2_LP + c];
    constexpr int OWN = RB2_LP + 1, LF = RB2_LP, RT = RB2_LP + 2, DNo = 1, UPo = 2 * RB2_LP + 1;
    // every read stays a ds_read_b64 (2 LDS cycles per wave): the compiler
    // would pair same-plane reads into ds_read2_b64, which takes 8. A
    // scheduling barrier that lets every instruction class cross it still
    // ends the pairing pass's search window.
    auto ld = [&](int plane, int d) __attribute__((always_inline)) -> double {
        __builtin_amdgcn_sched_barrier(0x7ff);
        return plane < 8 ? Lb0[plane * RB2_LS + d] : Lb1[(plane - 8) * RB2_LS + d];
    };
    auto st = [&](int plane, double v) __attribute__((always_inline)) {
        if (plane < 8) Lb0[plane * RB2_LS + OWN] = v;
        else Lb1[(plane - 8) * RB2_LS + OWN] = v;
    };
    // BND = false: the tile's loaded cells are all interior and none is next
    // to an x / y face, so every per-lane face and range test folds away
    const bool jin = !BND || (j >= 1 && j <= g.ny - 2);
    const bool in0 = !BND || (jin && i0 >= 1 && i0 <= g.nx - 2);
    const bool in1 = !BND || (jin && i0 + 1 <= g.nx - 2);
    const bool own = (c >= 2 && c <= RB2_TC - 3) && (r >= 4 && r <= RB2_TR - 5);
    const bool own0 = own && in0, own1 = own && in1;
    // the folded Neumann shell of Y2 (as k_rb1's nrole): 1 = pair (0, 1),
    // 2 = pair (nx-2, nx-1), 4 = nx odd and .y is cell nx-2, 8 = store
    const int nrole = BND ? ((i0 == 0 ? 1 : 0) | (i0 + 1 == g.nx - 1 ? 2 : 0) |
                             (i0 + 1 == g.nx - 2 ? 4 : 0) |
                             ((own && jin && i0 <= g.nx - 2) ? 8 : 0))
                          : (own ? 8 : 0);
    // face neighbours of iteration 2 (read as the centre): per component,
    // the x- / x+ neighbour is a face cell; y- / y+ per row
    const bool f0r = BND && (i0 + 1 == g.nx - 1);  // .x's right neighbour (own .y)
    const bool f1l = BND && (i0 == 0);              // .y's left neighbour (own .x)
    const bool f1r = BND && (i0 + 2 == g.nx - 1);   // .y's right neighbour (pair c+1 .x)
    const bool fdn = BND && (j == 1), fup = BND && (j == g.ny - 2);
    // loads from clamped, always valid addresses (see k_rb1): values outside
    // the grid only feed boundary cells and halo lanes
    const int ic = (i0 < g.nx) ? max(i0, 0) : g.nx - 2 - ((g.nx - 2) & 1);
    // 32-bit offsets within a plane from a wave-uniform plane base
    const int colx = max(min(j, g.ny - 1), 0) * (int)g.px + ic;
    const int col = max(min(j, g.ny - 1), 0) * (int)g.px + max(i0, 0);
    const int px = (int)g.px;
    // RB2_DIAG (diagnostic builds only, wrong results): every load reads
    // plane 0 (cache-resident) and the steady steps' stores are dropped,
    // which splits a sweep's time into its memory and its on-chip part
    auto ldx = [&](int k) -> double2 {
        if constexpr (RB2_DIAG) return ld2(X, colx);
        return ld2(X + (long long)min(max(k, 0), g.nz - 1) * g.ps, colx);
    };
    // rhs enters S1 first, whose values are valid one row inside the loaded
    // tile: the tile's outer rows (0, TR - 1) never load it and keep the
    // ring's zeros (the halo lanes' values stay ordinary); 2 of the 32 rows'
    // rhs lines. A masked load into the ring slot, no select.
    const bool rrow = r >= 1 && r <= RB2_TR - 2;
    auto ldr = [&](double2& dst, int k) __attribute__((always_inline)) {
        if constexpr (RB2_DIAG) {
            dst = ld2(rhs, colx);
        } else {
            if (rrow) dst = ld2(rhs + (long long)min(max(k, 0), g.nz - 1) * g.ps, colx);
        }
    };
    auto comp = [](const double2& v, int e) __attribute__((always_inline)) {
        return e == 0 ? v.x : v.y;
    };
    const int q0 = kb - 4;
    double2 xr[4], br[4];
    xr[0] = ldx(q0);
    xr[1] = ldx(q0 + 1);
    xr[2] = ldx(q0 + 2);
    xr[3] = make_double2(0.0, 0.0);
    br[0] = br[1] = br[2] = br[3] = make_double2(0.0, 0.0);
    ldr(br[2], q0 + 1);
    // X_{q0+1} into the X slot step q0 reads: LDS slots count planes from q0
    st(RB2_PX + 2, xr[1].x);
    st(RB2_PX + 3, xr[1].y);
    // the one-cell pad of every plane is never written by a step; zero it, so
    // that what halo lanes compute from it stays ordinary values (a stale
    // denormal there would send waves to rb2_sorc's recompute for nothing)
    for (int e = threadIdx.x; e < 16 * 2 * (RB2_LP + RB2_TR); e += 1024) {
        const int pl = e / (2 * (RB2_LP + RB2_TR)), q = e % (2 * (RB2_LP + RB2_TR));
        const int idx = q < 2 * RB2_LP ? (q < RB2_LP ? q : (RB2_TR + 1) * RB2_LP + q - RB2_LP)
                                       : ((q - 2 * RB2_LP) / 2 + 1) * RB2_LP +
                                             ((q & 1) ? RB2_LP - 1 : 0);
        L.pl[pl][idx] = 0.0;
    }
    // certification of one value (APX): branch-free, so the step stays one
    // basic block and its LDS reads can be scheduled ahead of the arithmetic
    auto cert = [&](bool ok, double v) __attribute__((always_inline)) {
        if constexpr (APX) {
            const double av = fabs(v);
            M = (ok && av > M) ? av : M;
        }
    };
    auto umax = [](bool ok, double a, double m) __attribute__((always_inline)) {
        return (ok && a > m) ? a : m;
    };
    // pin the running maxima at the end of their stage: left alone, the
    // compiler sinks every residual and range update of the unrolled steps
    // to the loop's back edge, where their operands no longer fit in VGPRs
    auto pin = [&]() __attribute__((always_inline)) {
        asm volatile("" : "+v"(mX), "+v"(mY));
        if constexpr (APX) asm volatile("" : "+v"(M));
    };
    const int nzi = g.nz - 2;  // last interior plane
    // ZB: a step at the ends of the march or next to a z face (range and
    // face tests per plane); the steady steps between take every stage in
    // range and no z face, so those tests fold away, and in an interior tile
    // (!BND) the maxima run over every lane unmasked: the owned-lane mask of
    // the residuals is applied once after the march, and the certification
    // bound may include halo lanes' values (finite: computed from the
    // planes this march wrote, the zeroed pads and clamped loads)
    auto step = [&](auto Ec, auto Pc, auto Zc, int q) __attribute__((always_inline)) {
        constexpr bool E = decltype(Ec)::value;
        constexpr int P = decltype(Pc)::value;
        constexpr bool ZB = decltype(Zc)::value;
        // a: a signed residual (APX) or its magnitude (res1); |a| enters the max
        auto rmax = [&](double& m, bool ok, bool ow, double a) __attribute__((always_inline)) {
            if constexpr (!ZB && !BND) m = rb2_vmax_abs(m, a);
            else m = umax(ok && ow, fabs(a), m);
        };
        auto certv = [&](bool ok, bool ow, double v) __attribute__((always_inline)) {
            if constexpr (!ZB) {
                if constexpr (APX) M = rb2_vmax_abs(M, v);
            } else {
                cert(ok && ow, v);
            }
        };
        constexpr int e = E ? 0 : 1;  // the component every update of this step touches
        // register rings (X, rhs): slot of plane p = (P + p - q + off) & 3
        constexpr int X0 = P & 3, X1 = (P + 1) & 3, X2 = (P + 2) & 3, X3 = (P + 3) & 3;
        constexpr int Bm1 = P & 3, B0 = (P + 1) & 3, B1 = (P + 2) & 3, B2 = (P + 3) & 3;
        // LDS slots of plane p: (P + p - q) & 1 (X) or & 3 (R1, Y1, R2)
        constexpr int LX1 = (P + 1) & 1, LX2 = P & 1;  // X_{q+1} read, X_{q+2} written
        constexpr int A1n = (P + 1) & 3, A1c = P & 3, A1m = (P + 3) & 3, A1mm = (P + 2) & 3;
        constexpr int AYn = P & 3, AYm = (P + 3) & 3, AYmm = (P + 2) & 3;
        constexpr int A2n = (P + 3) & 3, A2m = (P + 2) & 3, A2mm = (P + 1) & 3;
        // the one-colour neighbour of the updated component e on its x side
        // (pair c-1 for .x, pair c+1 for .y), and the other side's
        constexpr int SD = (e == 0) ? LF : RT, SDo = (e == 0) ? RT : LF;
        // rhs_{q-2} leaves its slot to rhs_{q+2}
        const double bq2 = comp(br[B2], e);
        xr[X3] = ldx(q + 3);
        ldr(br[B2], q + 2);
        __syncthreads();
        const int qa = q + 1, qc = q - 1, qd = q - 2;
        const bool pin1 = !ZB || (qa >= 1 && qa <= nzi), pin0 = !ZB || (q >= 1 && q <= nzi);
        const bool pinm = !ZB || (qc >= 1 && qc <= nzi), pind = !ZB || (qd >= 1 && qd <= nzi);
        const bool oka = !ZB || (qa >= kb && qa < ke), ok0 = !ZB || (q >= kb && q < ke);
        const bool okc = !ZB || (qc >= kb && qc < ke), okd = !ZB || (qd >= kb && qd < ke);
        // z faces next to the stages of iteration 2 (their Neumann copies)
        const bool zc1 = ZB && qc == 1, zcn = ZB && qc == nzi;
        const bool zd1 = ZB && qd == 1, zdn = ZB && qd == nzi;
        const bool ine = (e == 0) ? in0 : in1;
        const bool owe = (e == 0) ? own0 : own1, owb = (e == 0) ? own1 : own0;
        // ---- LDS operands of S1 and S2 ----
        constexpr int PX0 = RB2_PX + 2 * LX1, PX1 = PX0 + 1;
        const double2 xlo = make_double2(ld(PX0, DNo), ld(PX1, DNo));
        const double2 xhi = make_double2(ld(PX0, UPo), ld(PX1, UPo));
        const double xlp = ld(PX1, LF);  // pair c-1 .y
        const double xrp = ld(PX0, RT);  // pair c+1 .x
        const double r1c = ld(RB2_PR1 + A1c, OWN);  // the pair's first-colour cell of R1_q
        const double r1m = ld(RB2_PR1 + A1m, OWN);  // ... of R1_{q-1} (= Y1' there)
        const double r1dn = ld(RB2_PR1 + A1c, DNo), r1up = ld(RB2_PR1 + A1c, UPo);
        const double r1sd = ld(RB2_PR1 + A1c, SD);
        const double2 Xm = xr[X0], Xc = xr[X1], Xp = xr[X2];
        const double2 b1 = br[B1];
        // scheduling fences: each group of LDS reads is issued ahead of the
        // stage before the one that consumes it (its latency hides behind
        // that stage's arithmetic), and no group is hoisted further (the
        // operands of all four stages at once do not fit in 128 VGPRs)
        __builtin_amdgcn_sched_barrier(0);
        // ---- S1: R1_{q+1} (+ L-inf residual of X at plane q+1) ----
        // neighbour sums (right + left, up + down, above + below) of both cells
        const double sx0 = Xc.y + xlp, sy0 = xhi.x + xlo.x, sz0 = Xp.x + Xm.x;
        const double sx1 = xrp + Xc.x, sy1 = xhi.y + xlo.y, sz1 = Xp.y + Xm.y;
        double r1v, t1;
        if (e == 0) {
            const double v = rb2_sorc<APX>(cf, Xc.x, sx0, sy0, sz0, b1.x, &t1);
            r1v = (pin1 && in0) ? v : Xc.x;
        } else {
            const double v = rb2_sorc<APX>(cf, Xc.y, sx1, sy1, sz1, b1.y, &t1);
            r1v = (pin1 && in1) ? v : Xc.y;
        }
        {
            double a0, a1;
            if constexpr (APX) {
                a0 = (e == 0) ? rb2_res_from_t(cf, Xc.x, t1)
                              : rb2_res_apx(cf, Xc.x, sx0, sy0, sz0, b1.x);
                a1 = (e == 1) ? rb2_res_from_t(cf, Xc.y, t1)
                              : rb2_res_apx(cf, Xc.y, sx1, sy1, sz1, b1.y);
            } else {
                a0 = res1(rc, DivC{}, Xc.x, xlp, Xc.y, xlo.x, xhi.x, Xm.x, Xp.x, b1.x);
                a1 = res1(rc, DivC{}, Xc.y, Xc.x, xrp, xlo.y, xhi.y, Xm.y, Xp.y, b1.y);
            }
            rmax(mX, oka, own0, a0);
            rmax(mX, oka, own1, a1);
            certv(oka, owe, r1v);
            pin();
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- LDS operands of S3, the residual of Y1' and S4 ----
        const double y1mm = ld(RB2_PY1 + AYmm, OWN);  // Y1' second-colour cell at q-2 (= R2)
        const double ob = ld(RB2_PY1 + AYm, OWN);     // the pair's second-colour cell at q-1
        double ydn = ld(RB2_PY1 + AYm, DNo), yup = ld(RB2_PY1 + AYm, UPo);
        const double ysd = ld(RB2_PY1 + AYm, SD);
        double qdn = ld(RB2_PR1 + A1m, DNo), qup = ld(RB2_PR1 + A1m, UPo);
        const double qsd = ld(RB2_PR1 + A1m, SDo);
        double wm1 = ld(RB2_PR1 + A1mm, OWN);
        const double ow = ld(RB2_PR2 + A2m, OWN);     // the pair's first-colour cell of R2 at q-2
        double wdn = ld(RB2_PR2 + A2m, DNo), wup = ld(RB2_PR2 + A2m, UPo);
        const double wsd = ld(RB2_PR2 + A2m, SD);
        double zm2 = ld(RB2_PR2 + A2mm, OWN);
        __builtin_amdgcn_sched_barrier(0);
        // ---- S2: Y1_q, second colour (component e) from R1 ----
        double y1v;
        {
            const double sx = (e == 0) ? r1c + r1sd : r1sd + r1c;
            const double v = rb2_sorc<APX>(cf, comp(Xm, e), sx, r1up + r1dn, r1v + r1m,
                                          comp(br[B0], e));
            y1v = (pin0 && ine) ? v : comp(Xm, e);
            certv(ok0, owe, y1v);
            pin();
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- S3: R2_{q-1} from Y1' (+ L-inf residual of Y1' at plane q-1) ----
        double r2v;
        {
            const double cen = r1m;  // Y1' first-colour cell at q-1
            const double zm = zc1 ? cen : y1mm;
            const double zp = zcn ? cen : y1v;
            ydn = fdn ? cen : ydn;
            yup = fup ? cen : yup;
            double lf, rt;
            if (e == 0) {
                lf = ysd;
                rt = f0r ? cen : ob;
            } else {
                lf = f1l ? cen : ob;
                rt = f1r ? cen : ysd;
            }
            const double sx = rt + lf, sy = yup + ydn, sz = zp + zm;
            const double2 bm = br[Bm1];
            double t3;
            const double v = rb2_sorc<APX>(cf, cen, sx, sy, sz, comp(bm, e), &t3);
            r2v = (pinm && ine) ? v : cen;
            // the residual of Y1' at plane q-1: cell e (first colour) shares the
            // update's sums; cell 1-e (second colour, value ob) reads the
            // first-colour cells of Y1' = R1 at q-1
            const double cb = ob;
            const double wm = zc1 ? cb : wm1;
            const double wp = zcn ? cb : r1c;
            qdn = fdn ? cb : qdn;
            qup = fup ? cb : qup;
            double lf2, rt2;
            if (e == 0) {  // cell 1 (.y): left own .x (first colour), right pair c+1 .x
                lf2 = f1l ? cb : cen;
                rt2 = f1r ? cb : qsd;
            } else {       // cell 0 (.x): left pair c-1 .y, right own .y
                lf2 = qsd;
                rt2 = f0r ? cb : cen;
            }
            double ae, ab;
            if constexpr (APX) {
                ae = rb2_res_from_t(cf, cen, t3);
                ab = rb2_res_apx(cf, cb, rt2 + lf2, qup + qdn, wp + wm, comp(bm, 1 - e));
            } else {
                ae = res1(rc, DivC{}, cen, lf, rt, ydn, yup, zm, zp, comp(bm, e));
                ab = res1(rc, DivC{}, cb, lf2, rt2, qdn, qup, wm, wp, comp(bm, 1 - e));
            }
            rmax(mY, okc, owe, ae);
            rmax(mY, okc, owb, ab);
            certv(okc, owe, r2v);
            pin();
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- S4: Y2_{q-2}, second colour from R2 -> stored ----
        double2 out;
        {
            const double cen = y1mm;  // Y1' second-colour cell at q-2
            const double zm = zd1 ? cen : zm2;
            const double zp = zdn ? cen : r2v;
            wdn = fdn ? cen : wdn;
            wup = fup ? cen : wup;
            double lf, rt;
            if (e == 0) {
                lf = wsd;
                rt = f0r ? cen : ow;
            } else {
                lf = f1l ? cen : ow;
                rt = f1r ? cen : wsd;
            }
            const double v = rb2_sorc<APX>(cf, cen, rt + lf, wup + wdn, zp + zm, bq2);
            const double y2v = (pind && ine) ? v : cen;
            certv(okd, owe, y2v);
            pin();
            out = (e == 0) ? make_double2(y2v, ow) : make_double2(ow, y2v);
        }
        __builtin_amdgcn_sched_barrier(0);
        // ---- publish for step q + 1, then store Y2 ----
        st(RB2_PX + 2 * LX2, Xp.x);
        st(RB2_PX + 2 * LX2 + 1, Xp.y);
        st(RB2_PR1 + A1n, r1v);
        st(RB2_PY1 + AYn, y1v);
        st(RB2_PR2 + A2n, r2v);
        if constexpr (!ZB && !BND) {
            // steady step of an interior tile: one store, never branched
            // around (st2b), so the loads' vmcnt waits exclude it
            st2b<(FL & SW_NT_STORE) != 0>(Y + (long long)qd * g.ps, g.ps,
                                          (own && !RB2_DIAG) ? col * 8 : ST_NOSTORE, out);
        } else if (okd) {
            // the Neumann shell folded into the stores (as k_rb1)
            if (nrole & 1) out.x = out.y;
            if (nrole & 2) out.y = out.x;
            if (nrole & 8) {
                auto put = [&](double* yp) __attribute__((always_inline)) {
                    st2v<FL>(yp, col, out);
                    if (nrole & 4) yp[col + 2] = out.y;
                    if (BND && (j == 1 || j == g.ny - 2)) {
                        const int c2 = col + (j == 1 ? -px : px);
                        st2v<FL>(yp, c2, out);
                        if (nrole & 4) yp[c2 + 2] = out.y;
                    }
                };
                double* yq = Y + (long long)qd * g.ps;
                put(yq);
                if (zd1) put(yq - g.ps);
                if (zdn) put(yq + g.ps);
            }
        }
    };
    // E(q) = ((j + q + kofs) & 1) == 0, wave-uniform (rows r and r + 16 share it)
    const bool E0 = __builtin_amdgcn_readfirstlane(((j + q0 + g.kofs) & 1) == 0 ? 1 : 0) != 0;
    const int nsteps = ke - kb + 6;  // q0 .. ke + 1
    // the steady steps: q in [max(kb + 2, 4), ke - 2] (every stage's plane in
    // [kb, ke), none a z face or next to one, every operand from a plane the
    // march wrote), entered at a multiple of 4 steps to keep the ring phases
    const int n_s = min((max(kb + 2, 4) - q0 + 3) & ~3, nsteps);
    const int n_e = ke - 2 - q0 + 1;
    int n = 0;
    auto march = [&](auto E0c) __attribute__((always_inline)) {
        constexpr bool A = decltype(E0c)::value;
        using TA = BoolC<A>;
        using TB = BoolC<!A>;
        auto four = [&](auto Zc) __attribute__((always_inline)) {
            step(TA{}, IntC<0>{}, Zc, q0 + n);
            step(TB{}, IntC<1>{}, Zc, q0 + n + 1);
            step(TA{}, IntC<2>{}, Zc, q0 + n + 2);
            step(TB{}, IntC<3>{}, Zc, q0 + n + 3);
        };
        for (; n + 3 < n_s; n += 4) four(BoolC<true>{});
        for (; n + 3 < n_e; n += 4) four(BoolC<false>{});
        for (; n + 3 < nsteps; n += 4) four(BoolC<true>{});
        if (n < nsteps) step(TA{}, IntC<0>{}, BoolC<true>{}, q0 + n);
        if (n + 1 < nsteps) step(TB{}, IntC<1>{}, BoolC<true>{}, q0 + n + 1);
        if (n + 2 < nsteps) step(TA{}, IntC<2>{}, BoolC<true>{}, q0 + n + 2);
    };
    if (E0) march(BoolC<true>{});
    else march(BoolC<false>{});
    // the steady steps of an interior tile took every lane's residuals
    if constexpr (!BND) {
        mX = own ? mX : 0.0;
        mY = own ? mY : 0.0;
    }
}

template <bool APX, int FL>
static __global__ __launch_bounds__(1024, 4) void k_rb2(SGeo g, Rb2Coef cf,
                                                       const double* __restrict__ X,
                                                       double* __restrict__ Y,
                                                       const double* __restrict__ rhs,
                                                       RxState* st, double* partials,
                                                       unsigned* counter, int s, int certx,
                                                       int xmap, const Rb2Dec* __restrict__ dec) {
    __shared__ Rb2Lds L;
    if (st->done) return;
    // tile order: xmap = 1 gives each XCD a contiguous range of tiles
    // (xcd_tile), so the halo rows and columns a tile shares with its x / y
    // neighbours are fetched once into that XCD's L2 by whichever of the
    // concurrently running neighbours gets there first
    const int t = xmap ? xcd_tile(blockIdx.x, gridDim.x) : (int)blockIdx.x;
    const int tx = t % g.tiles_x;
    const int rest = t / g.tiles_x;
    const int ty = rest % g.tiles_y;
    const int tz = rest / g.tiles_y;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int c = lane & 31;
    const int r = w + 16 * (lane >> 5);
    const int i0 = tx * RB2_OX - 4 + 2 * c;  // even; the pair is (i0, i0 + 1)
    const int j = ty * RB2_OY - 4 + r;
    const int kb = g.k0 + tz * g.kc;
    const int ke = min(kb + g.kc, g.k1);
    // does the tile touch the faces (its loaded cells reach i < 1,
    // i > nx - 3, j < 2 or j > ny - 3)?
    const int ilo = tx * RB2_OX - 4, jlo = ty * RB2_OY - 4;
    const bool bnd = !(ilo >= 1 && ilo + 2 * RB2_TC - 1 <= g.nx - 3 && jlo >= 2 &&
                       jlo + RB2_TR - 1 <= g.ny - 3);
    double mX = 0.0, mY = 0.0, M = 0.0;
    if (bnd)
        rb2_march<APX, FL, true>(L, g, cf, X, Y, rhs, c, r, i0, j, kb, ke, mX, mY, M);
    else
        rb2_march<APX, FL, false>(L, g, cf, X, Y, rhs, c, r, i0, j, kb, ke, mX, mY, M);
    // ---- the sweep's maxima: partials[4 b + 0..2]; the last workgroup decides ----
    mX = wave_max(mX);
    mY = wave_max(mY);
    if constexpr (APX) M = wave_max(M);
    if (lane == 0) {
        L.sh[0][w] = mX;
        L.sh[1][w] = mY;
        L.sh[2][w] = M;
        L.sh[3][w] = 0.0;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0.0, b = 0.0, mm = 0.0, em = 0.0;
        for (int v = 0; v < 16; ++v) {
            a = fmax(a, L.sh[0][v]);
            b = fmax(b, L.sh[1][v]);
            mm = fmax(mm, L.sh[2][v]);
            em = fmin(em, L.sh[3][v]);
        }
        store_sc1(&partials[4 * blockIdx.x + 0], a);
        store_sc1(&partials[4 * blockIdx.x + 1], b);
        store_sc1(&partials[4 * blockIdx.x + 2], mm);
        store_sc1(&partials[4 * blockIdx.x + 3], em);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned tk = __hip_atomic_fetch_add((gu32*)counter, 1u, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        L.flag = (tk == gridDim.x - 1) ? 1 : 0;
    }
    __syncthreads();
    if (L.flag == 0) return;
    double a = 0.0, b = 0.0, mm = 0.0, em = 0.0;
    for (unsigned blk = threadIdx.x; blk < gridDim.x; blk += 1024) {
        a = fmax(a, load_sc1(&partials[4 * blk + 0]));
        b = fmax(b, load_sc1(&partials[4 * blk + 1]));
        mm = fmax(mm, load_sc1(&partials[4 * blk + 2]));
        em = fmin(em, load_sc1(&partials[4 * blk + 3]));
    }
    a = wave_max(a);
    b = wave_max(b);
    mm = wave_max(mm);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) em = fmin(em, __shfl_down(em, off, 64));
    __syncthreads();
    if (lane == 0) {
        L.sh[0][w] = a;
        L.sh[1][w] = b;
        L.sh[2][w] = mm;
        L.sh[3][w] = em;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double tX = 0.0, tY = 0.0, tM = 0.0, tE = 0.0;
        for (int v = 0; v < 16; ++v) {
            tX = fmax(tX, L.sh[0][v]);
            tY = fmax(tY, L.sh[1][v]);
            tM = fmax(tM, L.sh[2][v]);
            tE = fmin(tE, L.sh[3][v]);
        }
        __hip_atomic_store((gu32*)counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if constexpr (APX) {
            // X's own values (k_rb2_xmax; a NaN there fails the test too)
            if (certx && !(st->xmax <= tM)) tM = st->xmax;
            if (!(tM <= dec->mlim)) {
                st->done = 1;
                st->status = ST_RB2_UNCERT;
                st->res_it = s;
                return;
            }
            const double E = 32.0 * 0x1p-53 * (4.0 * tM * dec->kb + st->bmax) * dec->escale;
            if (rb2_decide(st, tX, E, s) && !st->done) rb2_decide(st, tY, E, s + 1);
        } else {
            rx_finish(st, tX, s);
            if (!st->done) rx_finish(st, tY, s + 1);
        }
    }
}

// max |rhs| over the interior (the residual bound's B), into st->bmax; one
// workgroup per block of planes, atomic max on the bit pattern (|v| >= 0
// orders as its bits)
static __global__ __launch_bounds__(256) void k_rb2_bmax(Geo g, const double* __restrict__ rhs,
                                                         RxState* st) {
    double m = 0.0;
    const long long plane = (long long)g.nx * g.ny;
    const long long total = plane * g.nz;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {
        const int k = (int)(e / plane);
        const long long q = e % plane;
        const int jj = (int)(q / g.nx), ii = (int)(q % g.nx);
        m = fmax(m, fabs(rhs[(long long)k * g.ps + (long long)jj * g.px + ii]));
    }
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0 && m > 0.0)
        __hip_atomic_fetch_max((gu64*)&st->bmax, (unsigned long long)__double_as_longlong(m),
                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// max |X| over the interior into st->xmax (zeroed by the host first): the
// certification of X's own values for a sweep whose input did not come
// from a k_rb2 sweep (certx); a NaN's bits order above every finite value,
// so a NaN fails the sweep's range test as before
static __global__ __launch_bounds__(256) void k_rb2_xmax(Geo g, const double* __restrict__ X,
                                                         RxState* st) {
    double m = 0.0;
    const int ni = g.nx - 2, nj = g.ny - 2;
    const long long plane = (long long)ni * nj;
    const long long total = plane * (g.nz - 2);
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {
        const int k = 1 + (int)(e / plane);
        const long long q = e % plane;
        const int jj = 1 + (int)(q / ni), ii = 1 + (int)(q % ni);
        const double v = fabs(X[(long long)k * g.ps + (long long)jj * g.px + ii]);
        m = (v > m || v != v) ? v : m;
    }
    // the bit patterns of non-negative values (and NaN above them) order as
    // unsigned integers
    unsigned long long b = (unsigned long long)__double_as_longlong(m);
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        const unsigned long long o = __shfl_down(b, off, 64);
        b = o > b ? o : b;
    }
    if ((threadIdx.x & 63) == 0 && b != 0)
        __hip_atomic_fetch_max((gu64*)&st->xmax, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

static __global__ void k_rb2_dec_init(Rb2Dec* d, double kb, double escale, double mlim) {
    if (threadIdx.x == 0) {
        d->kb = kb;
        d->escale = escale;
        d->mlim = mlim;
    }
}

// resume the loop after the host resolved a stop: clear the decision, and
// with ovr_it >= 0 give the loop that iterate's exact residual
static __global__ void k_rb2_resume(RxState* st, int ovr_it, double ovr_m) {
    if (threadIdx.x == 0) {
        st->done = 0;
        st->status = ST_MAX_ITER;
        st->ovr_it = ovr_it;
        st->ovr_m = ovr_m;
    }
}

}  // namespace cfdhip
