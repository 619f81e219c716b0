// kernels.hpp -- gfx950 device code for the Chorin projection step.
//
// Layout in HBM: every field is an SoA fp64 array with a padded row pitch
// `px` (multiple of 8 doubles = 64 B) and plane pitch `ps` = px*ny, x fastest.
// The reference layout idx = k*nx*ny + j*nx + i (lib/include/cfd/core/indexing.h)
// is recovered with px = nx; uploads/downloads convert with 2-D copies.
//
// Stencil sweeps use 2.5-D tiles: a 256-thread workgroup owns a 64 (x) by 4 (y)
// column tile and marches a chunk of `kc` planes in z, keeping the k-1/k/k+1
// values of its own column in registers so each plane is read once from HBM;
// x/y neighbours come from the L1/L2 lines the neighbouring lanes and waves
// of the same tile just loaded. One wavefront = one 64-wide x row, so every
// load is a fully coalesced 512-B row segment.
//
// Reductions are deterministic: per-thread sums in a fixed k order, a fixed
// 64-lane shuffle tree, a fixed cross-wave order, one partial per workgroup,
// and the last-arriving workgroup (agent-scope ticket) sums the partials in
// index order. The partial hand-off follows the sc1 write-through protocol
// (MI355X_MICROARCH.md "Valid forms", first table row): one lane stores the
// partial with an agent-scope relaxed store, waits vmcnt(0), then takes the
// ticket; the last workgroup reads every partial with agent-scope loads.
//
// All arithmetic is written in the reference's operation order and the file
// is compiled with -ffp-contract=off, so every per-cell value is bitwise the
// reference's; only the summation order of the CG dot products differs.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "mbox.hpp"

namespace cfdhip {

constexpr int TX = 64;       // x extent of a tile = one wavefront
constexpr int TY = 4;        // y rows per tile
constexpr int NT = TX * TY;  // threads per workgroup
constexpr int NWAVE = NT / 64;

// Poisson status codes (poisson_solver.h:83-89)
constexpr int ST_CONVERGED = 0;
constexpr int ST_MAX_ITER = 1;
constexpr int ST_STAGNATED = 3;

struct Geo {
    int nx, ny, nz;        // points of the local array, boundary included
    long long px;          // row pitch (doubles)
    long long ps;          // plane pitch (doubles)
    long long sz;          // z stencil offset: ps in 3-D, 0 in 2-D (reference stride_z)
    int k0, k1;            // interior planes [k0, k1)
    int kc;                // planes per tile
    int tiles_x, tiles_y, tiles_z;
    int lo_face, hi_face;  // local plane 0 / nz-1 is a global z face (Z-slabs: edge ranks)
    int kofs;              // global index of local plane 0 (Z-slabs)
};

struct Lap {
    double dx2_inv, dy2_inv, inv_dz2;  // linear_solver_cg.c:103-110
};

// x is updated every CG_XFOLD iterations: sweep A of iteration it with
// it % CG_XFOLD == 0, it > 0, folds the CG_XFOLD pending alpha_j p_j
// (j = it - 4 .. it - 1) into x before p_it overwrites slot it % CG_XFOLD;
// the search directions live in a ring of CG_XFOLD buffers (p_j in [j % CG_XFOLD]).
// A solve that stops after iteration it therefore leaves it % CG_XFOLD + 1
// (1 .. CG_XFOLD) updates pending, in distinct ring slots, for k_cg_finalize.
constexpr int CG_XFOLD = 4;

// Device-resident CG state; written only by the finishing (last) workgroup.
struct CgState {
    double rho;     // (r, r) of the current residual
    double alpha[CG_XFOLD];  // alpha_j of iteration j at [j % CG_XFOLD]
    double beta;    // beta for the next sweep A
    double pAp;
    double res;     // current residual 2-norm
    double res0;    // initial residual
    double tol;     // max(rel_tol * res0, abs_tol)
    double abs_tol;
    int iterations; // completed iterations (reference stats->iterations)
    int done;       // no further iteration may run
    int status;     // poisson_solver_status_t
    int nalpha;     // iterations whose alpha is valid (x must hold alpha_j p_j, j < nalpha)
    int xdone;      // x holds alpha_j p_j for j < xdone (folded by sweep B)
    int max_iter;
    int check_interval;
    int pad0;
};

typedef __attribute__((address_space(1))) unsigned long long gu64;
typedef __attribute__((address_space(1))) unsigned int gu32;

__device__ __forceinline__ void store_sc1(double* p, double v) {
    __hip_atomic_store((gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double load_sc1(const double* p) {
    unsigned long long b =
        __hip_atomic_load((gu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return __longlong_as_double((long long)b);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = fmax(v, __shfl_down(v, off, 64));
    return v;
}

// Sum over the workgroup; result valid in thread 0. `sh` holds NWAVE doubles.
__device__ __forceinline__ double block_sum(double v, double* sh) {
    v = wave_sum(v);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
    __syncthreads();
    double s = 0.0;
    if (threadIdx.x == 0) {
#pragma unroll
        for (int w = 0; w < NWAVE; ++w) s += sh[w];
    }
    __syncthreads();
    return s;
}

// Grid-wide deterministic sum. Returns true (in every thread) for the
// last-arriving workgroup; its thread 0 then holds the grid total.
__device__ __forceinline__ bool grid_sum_last(double block_total, double* partials,
                                              unsigned* counter, double* sh, int* flag,
                                              double& total) {
    if (threadIdx.x == 0) {
        store_sc1(&partials[blockIdx.x], block_total);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned t = __hip_atomic_fetch_add((gu32*)counter, 1u, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
        *flag = (t == gridDim.x - 1) ? 1 : 0;
    }
    __syncthreads();
    if (*flag == 0) return false;
    double s = 0.0;
    for (unsigned b = threadIdx.x; b < gridDim.x; b += NT) s += load_sc1(&partials[b]);
    total = block_sum(s, sh);
    if (threadIdx.x == 0)
        __hip_atomic_store((gu32*)counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
}

// Same protocol for NTH-thread workgroups; `sh` needs NTH/64 doubles of LDS
// that no wave still reads (callers pass their stencil row buffer after the
// workgroup barrier that ends the sweep).
template <int NTH>
__device__ __forceinline__ bool grid_sum_last_n(double block_total, double* partials,
                                                unsigned* counter, double* sh, int* flag,
                                                double& total, unsigned pofs = 0,
                                                unsigned ptot = 0) {
    if (ptot == 0) ptot = gridDim.x;
    if (threadIdx.x == 0) {
        store_sc1(&partials[pofs + blockIdx.x], block_total);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned t = __hip_atomic_fetch_add((gu32*)counter, 1u, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
        *flag = (t == ptot - 1) ? 1 : 0;
    }
    __syncthreads();
    if (*flag == 0) return false;
    double s = 0.0;
    for (unsigned b = threadIdx.x; b < ptot; b += NTH) s += load_sc1(&partials[b]);
    s = wave_sum(s);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = 0.0;
#pragma unroll
        for (int w = 0; w < NTH / 64; ++w) a += sh[w];
        total = a;
        __hip_atomic_store((gu32*)counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return true;
}

// Order-preserving encoding of doubles into uint64 for atomicMax.
__device__ __forceinline__ unsigned long long ord_enc(double d) {
    unsigned long long b = (unsigned long long)__double_as_longlong(d);
    return (b & 0x8000000000000000ull) ? ~b : (b | 0x8000000000000000ull);
}

struct TileCoord {
    int i, j, kb, ke;
    bool active;
};

__device__ __forceinline__ TileCoord tile_coord(const Geo& g, int t) {
    TileCoord c;
    const int tx = t % g.tiles_x;
    const int rest = t / g.tiles_x;
    const int ty = rest % g.tiles_y;
    const int tz = rest / g.tiles_y;
    c.i = tx * TX + (threadIdx.x & 63);
    c.j = ty * TY + (threadIdx.x >> 6);
    c.kb = g.k0 + tz * g.kc;
    c.ke = min(c.kb + g.kc, g.k1);
    c.active = (c.i >= 1) && (c.i <= g.nx - 2) && (c.j >= 1) && (c.j <= g.ny - 2);
    return c;
}

__device__ __forceinline__ long long cidx(const Geo& g, int i, int j, int k) {
    return (long long)k * g.ps + (long long)j * g.px + i;
}

// Laplacian exactly as linear_solver_cg.c:113-116 groups it.
__device__ __forceinline__ double lap7(const Lap& L, double c, double xm, double xp, double ym,
                                       double yp, double zm, double zp) {
    return ((xp - (2.0 * c) + xm) * L.dx2_inv) + ((yp - (2.0 * c) + ym) * L.dy2_inv) +
           ((zp + zm - (2.0 * c)) * L.inv_dz2);
}

// ---------------------------------------------------------------------------
// CG state transitions, run by one thread once a dot product's global total is
// known: inline in the last workgroup on one device, or in a 1-thread k_finish_*
// kernel after the cross-rank all-reduce of the per-rank totals (Z-slabs).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void fin_setup(CgState* st, double tot, double rel_tol, double abs_tol,
                                          int max_iter, int check_interval) {
    double res0 = sqrt(tot);                   // linear_solver_cg.c:345
    double tol = rel_tol * res0;               // :352-355
    if (tol < abs_tol) tol = abs_tol;
    st->rho = tot;
    st->res0 = res0;
    st->res = res0;
    st->tol = tol;
    st->abs_tol = abs_tol;
    for (int q = 0; q < CG_XFOLD; ++q) st->alpha[q] = 0.0;
    st->beta = 0.0;
    st->pAp = 0.0;
    st->iterations = 0;
    st->nalpha = 0;
    st->xdone = 0;
    st->max_iter = max_iter;
    st->check_interval = check_interval;
    if (res0 < abs_tol || max_iter <= 0) {     // :357-365
        st->done = 1;
        st->status = (res0 < abs_tol) ? ST_CONVERGED : ST_MAX_ITER;
    } else {
        st->done = 0;
        st->status = ST_MAX_ITER;
    }
}

// after (p, Ap): alpha or pAp breakdown (linear_solver_cg.c:395-407)
__device__ __forceinline__ void fin_A(CgState* st, double tot, int it, bool fold = false) {
    if (fold) st->xdone = it;  // this sweep A folded alpha_j p_j, j < it, into x
    st->pAp = tot;
    if (fabs(tot) < 1e-30) {
        st->done = 1;
        st->status = ST_STAGNATED;
        st->iterations = it + 1;
    } else {
        st->alpha[it % CG_XFOLD] = st->rho / tot;
        st->nalpha = it + 1;
    }
}

// after (r, r): convergence test, rho breakdown, beta (linear_solver_cg.c:416-445)
__device__ __forceinline__ void fin_B(CgState* st, double tot, int it) {
    double res = sqrt(tot);
    st->res = res;
    st->iterations = it + 1;
    const bool check = (it % st->check_interval) == 0;
    const bool conv = (res < st->tol) || (res < st->abs_tol);
    if (check && conv) {
        st->done = 1;
        st->status = ST_CONVERGED;
    } else if (fabs(st->rho) < 1e-30) {
        st->done = 1;
        st->status = ST_STAGNATED;
    } else {
        st->beta = tot / st->rho;
        st->rho = tot;
        if (it + 1 >= st->max_iter) {
            st->done = 1;
            st->status = conv ? ST_CONVERGED : ST_MAX_ITER;
        }
    }
}

constexpr int ST_COMM_TIMEOUT = 9;

__device__ __forceinline__ void comm_fail(CgState* st) {
    st->done = 1;
    st->status = ST_COMM_TIMEOUT;
}

static __global__ void k_finish_setup(CgState* st, const double* tot, double rel_tol, double abs_tol,
                               int max_iter, int check_interval) {
    if (threadIdx.x == 0) fin_setup(st, tot[0], rel_tol, abs_tol, max_iter, check_interval);
}
static __global__ void k_finish_A(CgState* st, const double* tot, int it, int fold) {
    if (threadIdx.x == 0 && !st->done) fin_A(st, tot[0], it, fold != 0);
}
static __global__ void k_finish_B(CgState* st, const double* tot, int it) {
    if (threadIdx.x == 0 && !st->done) fin_B(st, tot[0], it);
}

// ---------------------------------------------------------------------------
// CG setup: r = -rhs + lap(x) (linear_solver_cg.c:134-158) and rho = (r, r).
// FROM_VEL: rhs = (rho/dt) * div(u*) computed on the fly exactly as
// solver_projection.c:195-214 (the rhs array is never materialised for CG);
// otherwise rhs is read from memory. WRITE_RHS stores the rhs for the
// relaxation solvers, which re-read it every sweep.
// ---------------------------------------------------------------------------
struct DivCoef {
    double two_dx, two_dy;   // 2.0*dx, 2.0*dy (divided by, as the reference does)
    double inv_2dz;          // 1/(2dz), 0 in 2-D
    double rho_over_dt;
};

template <bool FROM_VEL, bool WRITE_RHS, bool WITH_RR, bool DIST = false>
static __global__ __launch_bounds__(NT) void k_cg_setup(Geo g, Lap L, DivCoef dc,
                                                 const double* __restrict__ us,
                                                 const double* __restrict__ vs,
                                                 const double* __restrict__ ws,
                                                 double* __restrict__ rhs,
                                                 const double* __restrict__ x,
                                                 double* __restrict__ r, CgState* st,
                                                 double* partials, unsigned* counter,
                                                 double rel_tol, double abs_tol, int max_iter,
                                                 int check_interval, double* dsum,
                                                 Mbox* mb) {
    __shared__ double sh[NWAVE];
    __shared__ int flag;
    double acc = 0.0;
    const int ntiles = g.tiles_x * g.tiles_y * g.tiles_z;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        TileCoord c = tile_coord(g, t);
        if (!c.active) continue;
        long long idx = cidx(g, c.i, c.j, c.kb);
        double xm = x[idx - g.sz], xc = x[idx];
        for (int k = c.kb; k < c.ke; ++k, idx += g.ps) {
            double xp = x[idx + g.sz];
            double b;
            if (FROM_VEL) {
                double dus = (us[idx + 1] - us[idx - 1]) / dc.two_dx;
                double dvs = (vs[idx + g.px] - vs[idx - g.px]) / dc.two_dy;
                double dws = (ws[idx + g.sz] - ws[idx - g.sz]) * dc.inv_2dz;
                double div = dus + dvs + dws;
                b = dc.rho_over_dt * div;
                if (WRITE_RHS) rhs[idx] = b;
            } else {
                b = rhs[idx];
            }
            double lap = lap7(L, xc, x[idx - 1], x[idx + 1], x[idx - g.px], x[idx + g.px], xm, xp);
            double rv = -b + lap;
            if (WITH_RR) {
                r[idx] = rv;
                acc += rv * rv;
            }
            xm = xc;
            xc = xp;
        }
    }
    if (!WITH_RR) return;
    double bt = block_sum(acc, sh);
    double tot;
    if (grid_sum_last(bt, partials, counter, sh, &flag, tot) && threadIdx.x == 0) {
        if (DIST && mb) {
            double g;
            if (mbox_allreduce(mb, tot, &g)) fin_setup(st, g, rel_tol, abs_tol, max_iter, check_interval);
            else comm_fail(st);
        } else if (DIST) {
            dsum[0] = tot;
        } else {
            fin_setup(st, tot, rel_tol, abs_tol, max_iter, check_interval);
        }
    }
}

// ===========================================================================
// Production CG sweeps ("row-pair" kernels).
//
// Tile = 128 (x) x TY (y) x kc (z); one wavefront per y row, each lane owns
// the x pair (i0, i0+1) and moves it with 16-B loads/stores (the streaming
// width MI355X's memory path prefers). x neighbours come from the adjacent
// lanes (__shfl), y neighbours from the TY+2 rows the workgroup's waves
// publish in LDS each plane (double-buffered, one barrier per plane), z
// neighbours from registers. Workgroups are mapped to tiles XCD-aware: the 8
// XCDs each get a contiguous band of tiles, so the y halo rows a workgroup
// reads were just streamed into the same XCD's L2 by its neighbour.
// Measured at 512^3 (tools/mb/stencil_mb6.hip): 5.2 TB/s for sweep A versus
// 4.3-4.5 TB/s for one-cell-per-lane designs.
// ===========================================================================
struct SGeo {
    int nx, ny, nz;
    long long px, ps, sz;
    int k0, k1, kc;
    int tiles_x, tiles_y, tiles_z;  // tiles of 128 x TY x kc
    // kmode 1: the two slab-edge planes only (tz 0 -> plane k0, tz 1 -> k1-1),
    // one plane per tile; the launch covering the remaining planes uses
    // k0+1 .. k1-1. A sweep split over several launches shares one partials
    // array: this launch's workgroups own partials [part_ofs, part_ofs +
    // gridDim.x) of part_total, and the last of all part_total workgroups
    // (same stream, so the later launch) finishes the reduction.
    int kmode;
    int part_ofs, part_total;
    int kofs;  // global index of local plane 0 (Z-slabs; colour parity)
    // kmode 2 (k_rb1 on slabs): tiles cover planes [kt0, kt1) only, while
    // k0 / k1 still bound the planes that are updated
    int kt0, kt1;
    // k_rb1: x of the first tile's first output column (the narrow
    // remainder strip starts where the full-width tiles end)
    int xofs;
    // k_ccf (kmode 0 / 2): z layers tz < nz1 run kc planes from the range's
    // start; layers tz >= nz1 ("tail") run kc2 planes from plane start +
    // nz1 kc, so the last-dispatched workgroups are short (nz1 = tiles_z:
    // every layer kc planes)
    int kc2, nz1;
};

__device__ __forceinline__ int xcd_tile(int b, int nt) {
    // bijective remap: block b runs on XCD b % 8 (round-robin dispatch);
    // give each XCD a contiguous range of tiles (speed only, never correctness)
    const int q = nt / 8, rem = nt % 8;
    const int x = b % 8, l = b / 8;
    const int start = x < rem ? x * (q + 1) : rem * (q + 1) + (x - rem) * q;
    return start + l;
}

__device__ __forceinline__ double2 ld2(const double* p, long long i) {
    return *reinterpret_cast<const double2*>(p + i);
}
__device__ __forceinline__ void st2(double* p, long long i, double2 v) {
    *reinterpret_cast<double2*>(p + i) = v;
}

// Sweep variants (template FL): bit 0 = non-temporal stores of the streamed
// outputs, bit 1 = non-temporal loads of inputs no other tile reads.
constexpr int SW_NT_STORE = 1;
constexpr int SW_NT_LOAD = 2;
typedef double d2x __attribute__((ext_vector_type(2)));
template <int FL>
__device__ __forceinline__ void st2v(double* p, long long i, double2 v) {
    if (FL & SW_NT_STORE) {
        d2x w = {v.x, v.y};
        __builtin_nontemporal_store(w, reinterpret_cast<d2x*>(p + i));
    } else {
        *reinterpret_cast<double2*>(p + i) = v;
    }
}
// A 16-B store into one plane through a buffer resource: an offset past the
// plane's bytes is dropped by the hardware, so a lane (or a step) that must
// not store passes ST_NOSTORE instead of branching around the store. Every
// step of a march then issues the same stores, and the compiler's vmcnt
// counting stays exact (a store under a branch counts as possibly absent, so
// the wait for a later plane's loads would also wait for that store).
constexpr int ST_NOSTORE = 0x7ffffff0;
// AUX: the store's cache-policy bits (2: nt, 16: sc1 write-through)
template <int AUX>
__device__ __forceinline__ void st2ba(double* plane_base, long long plane_elems, int boff,
                                      double2 v) {
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(plane_base, 0, (int)(plane_elems * 8), 0x00020000);
    const unsigned long long bx = (unsigned long long)__double_as_longlong(v.x);
    const unsigned long long by = (unsigned long long)__double_as_longlong(v.y);
    const u4 d = {(unsigned)bx, (unsigned)(bx >> 32), (unsigned)by, (unsigned)(by >> 32)};
    __builtin_amdgcn_raw_buffer_store_b128(d, rs, boff, 0, AUX);
}
template <bool NT>
__device__ __forceinline__ void st2b(double* plane_base, long long plane_elems, int boff,
                                     double2 v) {
    st2ba<NT ? 2 : 0>(plane_base, plane_elems, boff, v);  // aux 2: nt
}

// The load counterpart of st2b: a 16-B load from one plane through a buffer
// resource; an offset past the plane (ST_NOSTORE) returns zeros without a
// memory access, so a lane or step that needs no data issues the same load
// instead of branching around it (no branch: exact vmcnt counting).
// AUX: the load's cache-policy bits (2: nt, 16: sc1, which bypasses the L1)
template <int AUX>
__device__ __forceinline__ double2 ld2ba(const double* plane_base, long long plane_elems,
                                         int boff) {
    typedef unsigned int u4 __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<double*>(plane_base), 0, (int)(plane_elems * 8), 0x00020000);
    const u4 d = __builtin_amdgcn_raw_buffer_load_b128(rs, boff, 0, AUX);
    const unsigned long long bx = (unsigned long long)d.x | ((unsigned long long)d.y << 32);
    const unsigned long long by = (unsigned long long)d.z | ((unsigned long long)d.w << 32);
    return make_double2(__longlong_as_double((long long)bx), __longlong_as_double((long long)by));
}
template <bool NT = false>
__device__ __forceinline__ double2 ld2b(const double* plane_base, long long plane_elems, int boff) {
    return ld2ba<NT ? 2 : 0>(plane_base, plane_elems, boff);  // aux 2: nt
}

template <int FL>
__device__ __forceinline__ double2 ld2v(const double* p, long long i) {
    if (FL & SW_NT_LOAD) {
        d2x w = __builtin_nontemporal_load(reinterpret_cast<const d2x*>(p + i));
        return make_double2(w.x, w.y);
    }
    return *reinterpret_cast<const double2*>(p + i);
}

struct RowPair {
    int i0, j, kb, ke, lane, w;
    bool act, in0, in1;
    long long idx;   // cell (i0, clamp(j), kb)
};

template <int TY>
__device__ __forceinline__ RowPair row_pair(const SGeo& g) {
    RowPair c;
    const int nt = g.tiles_x * g.tiles_y * g.tiles_z;
    const int t = xcd_tile(blockIdx.x, nt);
    const int tx = t % g.tiles_x;
    const int rest = t / g.tiles_x;
    const int ty = rest % g.tiles_y;
    const int tz = rest / g.tiles_y;
    c.lane = threadIdx.x & 63;
    c.w = threadIdx.x >> 6;
    c.i0 = tx * 128 + 2 * c.lane;
    c.j = ty * TY + c.w;
    if (g.kmode == 1) {
        c.kb = (tz == 0) ? g.k0 : g.k1 - 1;
        c.ke = c.kb + 1;
    } else {
        c.kb = g.k0 + tz * g.kc;
        c.ke = min(c.kb + g.kc, g.k1);
    }
    c.act = (c.j >= 1) && (c.j <= g.ny - 2) && (c.i0 < g.nx);
    c.in0 = c.act && (c.i0 >= 1) && (c.i0 <= g.nx - 2);
    c.in1 = c.act && (c.i0 + 1 <= g.nx - 2);
    const int ic = min(c.i0, g.nx - 2 - ((g.nx - 2) & 1));  // even, in-row, 16-B aligned
    const int jc = min(c.j, g.ny - 1);
    c.idx = (long long)c.kb * g.ps + (long long)jc * g.px + (c.i0 < g.nx ? c.i0 : ic);
    return c;
}

// Loads of one plane step are issued through a small "bundle": without
// SW_PREFETCH the bundle of plane k is loaded at the top of iteration k (and
// its centre loads are consumed in the same iteration); with SW_PREFETCH the
// bundle of plane k+1 is issued before plane k is processed, so one plane of
// loads stays in flight across the LDS barrier and the arithmetic.
constexpr int SW_PREFETCH = 4;
// bit 3: the two x-edge cells of a row (lane 0's left, lane 63's right
// neighbour) are fetched by ONE load instruction with per-lane addresses;
// bit 4: the centre rows of the inner waves of a stencil field (rows no
// neighbouring tile re-reads as its y halo) are loaded non-temporally.
constexpr int SW_EDGE1 = 8;
constexpr int SW_NT_INNER = 16;
// (r01e: asking for 8 waves per SIMD, i.e. <= 64 VGPRs and two 1024-thread
// workgroups per CU, spills and is slower; profiles/r01e_sweep_variants.jsonl)
template <int FL>
constexpr int sweep_min_waves() {
    return (FL & SW_PREFETCH) ? 4 : 1;
}

template <bool NT>
__device__ __forceinline__ double2 ld2n(const double* p, long long i) {
    if (NT) {
        d2x w = __builtin_nontemporal_load(reinterpret_cast<const d2x*>(p + i));
        return make_double2(w.x, w.y);
    }
    return *reinterpret_cast<const double2*>(p + i);
}

__device__ __forceinline__ double2 fma2p(double2 a, double beta, double2 b) {
    return make_double2(a.x + beta * b.x, a.y + beta * b.y);
}

// Sweep A (iteration it):  p_it = r + beta p_{it-1} (FIRST: p = r), written
// to pnew; (p, A p) with A p in registers.
// FOLD (it % CG_XFOLD == 0, it > 0): x = (((x + a_{it-4} p_{it-4}) +
// a_{it-3} p_{it-3}) + a_{it-2} p_{it-2}) + a_{it-1} p_{it-1}, the
// reference's per-iteration updates x += alpha p (linear_solver_cg.c:379-380,
// axpy :85-96) in their order with the partial sums in registers, so x is
// bitwise the reference's while it is read and written every fourth
// iteration only. p_{it-1} = p_old is already streamed by this sweep and
// p_{it-4} is the ring slot p_it is written to (read before the write, same
// lane), so the fold costs x, p_{it-3}, p_{it-2} and the x store.
struct PFold {
    const double* q3;  // p_{it-3}
    const double* q2;  // p_{it-2}
    double* x;
};

template <int TY, bool FIRST, bool DIST, int FL = 0, bool FOLD = false>
static __global__ __launch_bounds__(64 * TY, sweep_min_waves<FL>()) void k_cgA(
    SGeo g, Lap L, const double* __restrict__ r, const double* __restrict__ po,
    double* __restrict__ pn, CgState* st, double* partials, unsigned* counter, int it,
    double* dsum, Mbox* mb, PFold fd) {
    constexpr bool PF = (FL & SW_PREFETCH) != 0;
    __shared__ double2 rows[2][TY + 2][64];
    __shared__ double sh[TY];
    __shared__ int flag;
    if (st->done) return;
    const double beta = FIRST ? 0.0 : st->beta;
    double fa[CG_XFOLD];  // alpha_{it-4} .. alpha_{it-1}
#pragma unroll
    for (int q = 0; q < CG_XFOLD; ++q) fa[q] = FOLD ? st->alpha[(it + q) % CG_XFOLD] : 0.0;
    const double* __restrict__ fq3 = fd.q3;
    const double* __restrict__ fq2 = fd.q2;
    double* __restrict__ fx = fd.x;
    RowPair c = row_pair<TY>(g);
    const bool halo = (c.w == 0) || (c.w == TY - 1);
    const int jh = (c.w == 0) ? max(c.j - 1, 0) : min(c.j + 1, g.ny - 1);
    const int hslot = (c.w == 0) ? 0 : TY + 1;
    const long long hoff = (long long)(jh - min(c.j, g.ny - 1)) * g.px;
    const bool xok = c.i0 < g.nx;
    const bool eok_l = c.lane == 0 && c.i0 >= 1 && xok;
    const bool eok_r = c.lane == 63 && c.i0 + 2 < g.nx;
    constexpr bool E1 = (FL & SW_EDGE1) != 0;
    const bool eok = eok_l || eok_r;
    const long long eoff = (c.lane == 0) ? -1 : 2;
    const bool inner = (FL & SW_NT_INNER) && !halo;
    const double2 zero = make_double2(0.0, 0.0);
    // raw r / p_old of: the centre of plane k+1, the y-halo row of plane k+1,
    // the x-edge cells of plane k (p is formed from them when used; with
    // SW_EDGE1 lane 0's left and lane 63's right cell share lr / lo)
    struct Bundle {
        double2 cr, co, hr, ho;
        double lr, lo, rr, ro;
        double2 fxo, f4, f3, f2;  // FOLD: x, p_{it-4}, p_{it-3}, p_{it-2} of plane k
    };
    auto issue = [&](int k, long long ix) __attribute__((always_inline)) {
        const double2 zero = make_double2(0.0, 0.0);  // a value, not the captured object
        Bundle b;
        const long long ip = ix + g.sz;
        if (inner) {
            b.cr = xok ? ld2n<true>(r, ip) : zero;
            b.co = (xok && !FIRST) ? ld2n<true>(po, ip) : zero;
        } else {
            b.cr = xok ? ld2(r, ip) : zero;
            b.co = (xok && !FIRST) ? ld2(po, ip) : zero;
        }
        const bool h = xok && halo && k + 1 < c.ke;
        b.hr = h ? ld2(r, ip + hoff) : zero;
        b.ho = (h && !FIRST) ? ld2(po, ip + hoff) : zero;
        if (E1) {
            b.lr = eok ? r[ix + eoff] : 0.0;
            b.lo = (eok && !FIRST) ? po[ix + eoff] : 0.0;
            b.rr = b.ro = 0.0;
        } else {
            b.lr = eok_l ? r[ix - 1] : 0.0;
            b.lo = (eok_l && !FIRST) ? po[ix - 1] : 0.0;
            b.rr = eok_r ? r[ix + 2] : 0.0;
            b.ro = (eok_r && !FIRST) ? po[ix + 2] : 0.0;
        }
        const bool fl = FOLD && xok && c.act;
        b.fxo = fl ? ld2v<FL>(fx, ix) : zero;
        b.f4 = fl ? ld2v<FL>(pn, ix) : zero;
        b.f3 = fl ? ld2v<FL>(fq3, ix) : zero;
        b.f2 = fl ? ld2v<FL>(fq2, ix) : zero;
        return b;
    };
    auto form2 = [&](double2 a, double2 b) { return FIRST ? a : fma2p(a, beta, b); };
    auto form1 = [&](double a, double b) { return FIRST ? a : a + beta * b; };
    double acc = 0.0;
    long long idx = c.idx;
    double2 pm = xok ? form2(ld2(r, idx - g.sz), FIRST ? zero : ld2(po, idx - g.sz)) : zero;
    // raw p_{it-1} of the current plane (the fold's last term)
    double2 praw = (FOLD && xok) ? ld2(po, idx) : zero;
    double2 pc = xok ? form2(ld2(r, idx), FIRST ? zero : (FOLD ? praw : ld2(po, idx))) : zero;
    double2 hc = (xok && halo) ? form2(ld2(r, idx + hoff), FIRST ? zero : ld2(po, idx + hoff))
                               : zero;
    // Z-slabs: p is pointwise in r and p_old, so the tiles at the slab ends
    // also write the new p on the halo planes (r's halo is exchanged after
    // sweep B); sweep B then needs no halo exchange of p.
    if (DIST && c.act && c.kb == g.k0) {
        double2 pw;
        pw.x = c.in0 ? pm.x : 0.0;
        pw.y = c.in1 ? pm.y : 0.0;
        st2(pn, idx - g.sz, pw);
    }
    Bundle cur;
    if (PF) cur = issue(c.kb, idx);
    int buf = 0;
    for (int k = c.kb; k < c.ke; ++k, idx += g.ps) {
        Bundle nxt;
        if (PF) {
            if (k + 1 < c.ke) nxt = issue(k + 1, idx + g.ps);
        } else {
            cur = issue(k, idx);
        }
        rows[buf][c.w + 1][c.lane] = pc;
        if (halo) rows[buf][hslot][c.lane] = hc;
        __syncthreads();
        const double2 ys = rows[buf][c.w][c.lane];
        const double2 yn = rows[buf][c.w + 2][c.lane];
        const double2 pp = form2(cur.cr, cur.co);
        double left = __shfl_up(pc.y, 1, 64);
        double right = __shfl_down(pc.x, 1, 64);
        if (c.lane == 0) left = form1(cur.lr, cur.lo);
        if (c.lane == 63) right = E1 ? form1(cur.lr, cur.lo) : form1(cur.rr, cur.ro);
        const double Ap0 = -lap7(L, pc.x, left, pc.y, ys.x, yn.x, pm.x, pp.x);
        const double Ap1 = -lap7(L, pc.y, pc.x, right, ys.y, yn.y, pm.y, pp.y);
        if (FOLD && c.act) {
            double2 xw;
            xw.x = c.in0 ? (((cur.fxo.x + fa[0] * cur.f4.x) + fa[1] * cur.f3.x) + fa[2] * cur.f2.x) +
                               fa[3] * praw.x
                         : cur.fxo.x;
            xw.y = c.in1 ? (((cur.fxo.y + fa[0] * cur.f4.y) + fa[1] * cur.f3.y) + fa[2] * cur.f2.y) +
                               fa[3] * praw.y
                         : cur.fxo.y;
            st2v<FL>(fx, idx, xw);
        }
        if (c.act) {
            double2 pw;
            pw.x = c.in0 ? pc.x : 0.0;
            pw.y = c.in1 ? pc.y : 0.0;
            st2v<FL>(pn, idx, pw);
        }
        if (c.in0) acc += pc.x * Ap0;
        if (c.in1) acc += pc.y * Ap1;
        pm = pc;
        pc = pp;
        if (FOLD) praw = cur.co;
        hc = form2(cur.hr, cur.ho);
        if (PF) cur = nxt;
        buf ^= 1;
    }
    if (DIST && c.act && c.ke == g.k1) {  // pc = p on plane k1 (upper halo)
        double2 pw;
        pw.x = c.in0 ? pc.x : 0.0;
        pw.y = c.in1 ? pc.y : 0.0;
        st2(pn, idx, pw);
    }
    // deterministic workgroup sum: wave tree, then waves in order
    acc = wave_sum(acc);
    if (c.lane == 0) sh[c.w] = acc;
    __syncthreads();
    double bt = 0.0;
    if (threadIdx.x == 0)
        for (int q = 0; q < TY; ++q) bt += sh[q];
    double tot;
    double* shs = (double*)&rows[0][0][0];
    if (grid_sum_last_n<64 * TY>(bt, partials, counter, shs, &flag, tot) && threadIdx.x == 0) {
        if (DIST && mb) {
            double g;
            if (mbox_allreduce(mb, tot, &g)) fin_A(st, g, it, FOLD);
            else comm_fail(st);
        } else if (DIST) {
            dsum[0] = tot;
        } else {
            fin_A(st, tot, it, FOLD);
        }
    }
}

// Sweep B (iteration it): r -= alpha A p (A p recomputed from p, bitwise equal
// to sweep A's), rho_new = (r, r), convergence test and beta. (x is folded by
// sweep A every CG_XFOLD iterations, k_cgA<FOLD>.)
struct PRing {
    const double* p[CG_XFOLD];  // p_j at [j % CG_XFOLD]
};
struct PPrev {
    const double* q[CG_XFOLD - 1];  // p_{it-3}, p_{it-2}, p_{it-1}
};

// REV (r03, one device, 3-D): the tile marches z downwards. Sweep A marches
// upwards, so each sweep starts on the planes the previous one touched last,
// which the 256 MB Infinity Cache still holds (p just written by sweep A,
// r just read by it; then r just written by sweep B for the next sweep A).
// The z neighbours keep their roles in lap7, so A p is bitwise sweep A's; only
// the order of the (r, r) partial sums within a tile changes.
template <int TY, bool DIST, int FL = 0, bool REV = false>
static __global__ __launch_bounds__(64 * TY, sweep_min_waves<FL>()) void k_cgB(
    SGeo g, Lap L, const double* __restrict__ p, double* __restrict__ r, CgState* st,
    double* partials, unsigned* counter, int it, double* dsum, Mbox* mb) {
    constexpr bool PF = (FL & SW_PREFETCH) != 0;
    __shared__ double2 rows[2][TY + 2][64];
    __shared__ double sh[TY];
    __shared__ int flag;
    if (st->done) return;
    const double malpha = -st->alpha[it % CG_XFOLD];
    RowPair c = row_pair<TY>(g);
    const bool halo = (c.w == 0) || (c.w == TY - 1);
    const int jh = (c.w == 0) ? max(c.j - 1, 0) : min(c.j + 1, g.ny - 1);
    const int hslot = (c.w == 0) ? 0 : TY + 1;
    const long long hoff = (long long)(jh - min(c.j, g.ny - 1)) * g.px;
    const bool xok = c.i0 < g.nx;
    const bool eok_l = c.lane == 0 && c.i0 >= 1 && xok;
    const bool eok_r = c.lane == 63 && c.i0 + 2 < g.nx;
    constexpr bool E1 = (FL & SW_EDGE1) != 0;
    const bool eok = eok_l || eok_r;
    const long long eoff = (c.lane == 0) ? -1 : 2;
    const bool inner = (FL & SW_NT_INNER) && !halo;
    const double2 zero = make_double2(0.0, 0.0);
    // p of the centre and y-halo row of plane k+1; r and the x-edge p of
    // plane k (SW_EDGE1: both edge cells in el)
    struct Bundle {
        double2 pp, hp, rr;
        double el, er;
    };
    // sd: the z stride towards the next plane of the march
    const long long sd = REV ? -g.sz : g.sz;
    const long long pstep = REV ? -g.ps : g.ps;
    auto issue = [&](int k, long long ix) __attribute__((always_inline)) {
        const double2 zero = make_double2(0.0, 0.0);  // a value, not the captured object
        Bundle b;
        const long long ip = ix + sd;
        const bool more = REV ? (k - 1 >= c.kb) : (k + 1 < c.ke);
        if (inner) b.pp = xok ? ld2n<true>(p, ip) : zero;
        else b.pp = xok ? ld2(p, ip) : zero;
        b.hp = (xok && halo && more) ? ld2(p, ip + hoff) : zero;
        b.rr = xok ? ld2v<FL>(r, ix) : zero;
        if (E1) {
            b.el = eok ? p[ix + eoff] : 0.0;
            b.er = 0.0;
        } else {
            b.el = eok_l ? p[ix - 1] : 0.0;
            b.er = eok_r ? p[ix + 2] : 0.0;
        }
        return b;
    };
    double acc = 0.0;
    const int k_first = REV ? c.ke - 1 : c.kb;
    long long idx = c.idx + (REV ? (long long)(c.ke - 1 - c.kb) * g.ps : 0LL);
    // pm: the plane the march left (z- forwards, z+ in REV), pp: the next one
    double2 pm = xok ? ld2(p, idx - sd) : zero;
    double2 pc = xok ? ld2(p, idx) : zero;
    double2 hc = (xok && halo) ? ld2(p, idx + hoff) : zero;
    Bundle cur;
    if (PF) cur = issue(k_first, idx);
    int buf = 0;
    for (int n = 0, k = k_first; n < c.ke - c.kb; ++n, k += REV ? -1 : 1, idx += pstep) {
        Bundle nxt;
        if (PF) {
            if (n + 1 < c.ke - c.kb) nxt = issue(REV ? k - 1 : k + 1, idx + pstep);
        } else {
            cur = issue(k, idx);
        }
        rows[buf][c.w + 1][c.lane] = pc;
        if (halo) rows[buf][hslot][c.lane] = hc;
        __syncthreads();
        const double2 ys = rows[buf][c.w][c.lane];
        const double2 yn = rows[buf][c.w + 2][c.lane];
        const double2 pp = cur.pp;
        double left = __shfl_up(pc.y, 1, 64);
        double right = __shfl_down(pc.x, 1, 64);
        if (c.lane == 0) left = cur.el;
        if (c.lane == 63) right = E1 ? cur.el : cur.er;
        const double2 zm = REV ? pp : pm, zp = REV ? pm : pp;
        const double Ap0 = -lap7(L, pc.x, left, pc.y, ys.x, yn.x, zm.x, zp.x);
        const double Ap1 = -lap7(L, pc.y, pc.x, right, ys.y, yn.y, zm.y, zp.y);
        double2 rn;
        rn.x = c.in0 ? cur.rr.x + malpha * Ap0 : cur.rr.x;
        rn.y = c.in1 ? cur.rr.y + malpha * Ap1 : cur.rr.y;
        if (c.act) st2v<FL>(r, idx, rn);
        if (c.in0) acc += rn.x * rn.x;
        if (c.in1) acc += rn.y * rn.y;
        pm = pc;
        pc = pp;
        hc = cur.hp;
        if (PF) cur = nxt;
        buf ^= 1;
    }
    acc = wave_sum(acc);
    if (c.lane == 0) sh[c.w] = acc;
    __syncthreads();
    double bt = 0.0;
    if (threadIdx.x == 0)
        for (int q = 0; q < TY; ++q) bt += sh[q];
    double tot;
    double* shs = (double*)&rows[0][0][0];
    if (grid_sum_last_n<64 * TY>(bt, partials, counter, shs, &flag, tot, g.part_ofs,
                                 g.part_total) &&
        threadIdx.x == 0) {
        if (DIST && mb) {
            double g2;
            if (mbox_allreduce(mb, tot, &g2)) fin_B(st, g2, it);
            else comm_fail(st);
        } else if (DIST) {
            dsum[0] = tot;
        } else {
            fin_B(st, tot, it);
        }
    }
}

// ---------------------------------------------------------------------------
// Whole CG solve in ONE persistent launch for small grids (r02b). On a
// 128 x 128 grid a CG iteration's two sweeps cost ~15 us, nearly all kernel
// dispatch and completion. Here one cooperative launch runs
// every iteration: phase A (p = r + beta p_old, A p, (p, Ap)), a grid barrier,
// phase B (x += alpha p, r -= alpha A p, (r, r)), a grid barrier (up to 256
// workgroups, one per 256 interior cells). Every
// workgroup sums the per-workgroup partials in the same order and applies
// the state transition (fin_A / fin_B) to its own LDS copy of the CG state,
// so all leave the loop at the same iteration with no extra barrier. r and
// the two p buffers are shared between workgroups inside the launch, so they
// move through agent-scope atomic loads / stores (coherent across the XCDs'
// L2s); x is only touched by its own cell. Per-cell arithmetic is the
// sweeps' (same lap7 operands, p = r + beta p_old, r + (-alpha) A p,
// x + alpha p per iteration, which is bitwise the sweeps' x fold); only the
// dot-product summation order differs, as between the sweep kernels and the
// reference. The barrier wait is bounded (a timeout ends the solve with
// ST_COMM_TIMEOUT instead of hanging the GPU).
// ---------------------------------------------------------------------------
constexpr int CGS_THREADS = 256;
constexpr int CGS_MAX_WG = 256;
constexpr long long CG_SMALL_CELLS = 300000;  // default ceiling (interior cells): 64^3 yes, 96^3 no

static __global__ __launch_bounds__(CGS_THREADS) void k_cg_small(Geo g, Lap L,
                                                                 double* __restrict__ x, double* r,
                                                                 double* pa, double* pb,
                                                                 CgState* st, double* partials,
                                                                 unsigned* bar,
                                                                 long long timeout_ticks) {
    __shared__ CgState ls;
    __shared__ double sh[CGS_THREADS / 64];
    __shared__ int bad;
    const unsigned nb = gridDim.x;
    const long long nxi = g.nx - 2, nyi = g.ny - 2;
    const long long ncell = nxi * nyi * (long long)(g.k1 - g.k0);
    if (threadIdx.x == 0) {
        ls = *st;
        bad = 0;
    }
    __syncthreads();
    unsigned target = 0;
    auto barrier = [&]() __attribute__((always_inline)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's stores landed
        __syncthreads();
        target += nb;
        if (threadIdx.x == 0) {
            __hip_atomic_fetch_add((gu32*)bar, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const long long t0 = wall_clock64();
            while (__hip_atomic_load((gu32*)bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) <
                   target) {
                __builtin_amdgcn_s_sleep(1);
                if (wall_clock64() - t0 > timeout_ticks) {
                    bad = 1;
                    break;
                }
            }
        }
        __syncthreads();
    };
    // block partial -> partials[slot][block] -> barrier (gsum_begin); every
    // workgroup then sums the partials in the same fixed tree (gsum_end,
    // total in thread 0). The next phase's loads of each thread's first cell
    // are issued between the two, so they overlap the partials' round trip.
    auto gsum_begin = [&](int slot, double v) __attribute__((always_inline)) {
        v = wave_sum(v);
        if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = v;
        __syncthreads();
        if (threadIdx.x == 0) {
            double b = 0.0;
#pragma unroll
            for (int w = 0; w < CGS_THREADS / 64; ++w) b += sh[w];
            store_sc1(&partials[slot * CGS_MAX_WG + blockIdx.x], b);
        }
        barrier();
    };
    auto gsum_end = [&](int slot) __attribute__((always_inline)) {
        double t = (threadIdx.x < nb) ? load_sc1(&partials[slot * CGS_MAX_WG + threadIdx.x]) : 0.0;
        t = wave_sum(t);
        if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = t;
        __syncthreads();
        double tot = 0.0;
        if (threadIdx.x == 0) {
#pragma unroll
            for (int w = 0; w < CGS_THREADS / 64; ++w) tot += sh[w];
        }
        __syncthreads();  // sh is reused by the next reduction
        return tot;
    };
    auto cell = [&](long long e) __attribute__((always_inline)) {
        const long long i = 1 + e % nxi;
        const long long q = e / nxi;
        const long long j = 1 + q % nyi;
        const long long k = g.k0 + q / nyi;
        return k * g.ps + j * g.px + i;
    };
    const long long stride = (long long)nb * CGS_THREADS;
    const long long e0 = (long long)blockIdx.x * CGS_THREADS + threadIdx.x;
    const bool has0 = e0 < ncell;
    const long long c0 = cell(has0 ? e0 : 0);  // a valid address either way
    // the 7 stencil points of a cell: centre, x-, x+, y-, y+, z-, z+
    auto pts = [&](long long c, long long (&q)[7]) __attribute__((always_inline)) {
        q[0] = c; q[1] = c - 1; q[2] = c + 1; q[3] = c - g.px; q[4] = c + g.px;
        q[5] = c - g.sz; q[6] = c + g.sz;
    };
    long long q0s[7];
    pts(c0, q0s);
    // phase A operands of cell c0: r and p_old at its stencil points
    double ar[7], ap[7];
    auto loadA = [&](const double* po_, bool first_) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < 7; ++t) {
            ar[t] = load_sc1(&r[q0s[t]]);
            ap[t] = first_ ? 0.0 : load_sc1(&po_[q0s[t]]);
        }
    };
    // phase A of one cell from its operands: p = r + beta p_old, A p
    auto cellA = [&](long long c, const double (&rv)[7], const double (&pv)[7], bool first_,
                     double beta, double* pn_, double& acc) __attribute__((always_inline)) {
        double pp[7];
#pragma unroll
        for (int t = 0; t < 7; ++t) pp[t] = first_ ? rv[t] : rv[t] + beta * pv[t];
        const double Ap = -lap7(L, pp[0], pp[1], pp[2], pp[3], pp[4], pp[5], pp[6]);
        store_sc1(&pn_[c], pp[0]);
        acc += pp[0] * Ap;
    };
    // phase B operands of cell c0: p_it at its stencil points, r, x
    double bp[7], brr, bx;
    auto loadB = [&](const double* pn_) __attribute__((always_inline)) {
#pragma unroll
        for (int t = 0; t < 7; ++t) bp[t] = load_sc1(&pn_[q0s[t]]);
        brr = load_sc1(&r[c0]);
        bx = x[c0];
    };
    auto cellB = [&](long long c, const double (&pv)[7], double rv, double xv, double al,
                     double ma, double& acc) __attribute__((always_inline)) {
        const double Ap = -lap7(L, pv[0], pv[1], pv[2], pv[3], pv[4], pv[5], pv[6]);
        x[c] = xv + al * pv[0];
        const double rn = rv + ma * Ap;
        store_sc1(&r[c], rn);
        acc += rn * rn;
    };
    loadA(pb, true);  // iteration 0: p = r
    for (int it = 0;; ++it) {
        if (ls.done) break;
        double* pn = (it & 1) ? pb : pa;
        const double* po = (it & 1) ? pa : pb;
        const bool first = (it == 0);
        const double beta = first ? 0.0 : ls.beta;
        // phase A: p_it = r + beta p_{it-1} (formed at the neighbours too), (p, A p)
        double acc = 0.0;
        if (has0) cellA(c0, ar, ap, first, beta, pn, acc);
        for (long long e = e0 + stride; e < ncell; e += stride) {
            const long long c = cell(e);
            long long q[7];
            pts(c, q);
            double rv[7], pv[7];
#pragma unroll
            for (int t = 0; t < 7; ++t) {
                rv[t] = load_sc1(&r[q[t]]);
                pv[t] = first ? 0.0 : load_sc1(&po[q[t]]);
            }
            cellA(c, rv, pv, first, beta, pn, acc);
        }
        gsum_begin(0, acc);
        if (bad) break;
        loadB(pn);
        const double tA = gsum_end(0);
        if (threadIdx.x == 0) fin_A(&ls, tA, it);
        __syncthreads();
        if (ls.done) break;
        // phase B: x += alpha p, r -= alpha A p (A p recomputed), (r, r)
        const double al = ls.alpha[it % CG_XFOLD];
        const double ma = -al;
        acc = 0.0;
        if (has0) cellB(c0, bp, brr, bx, al, ma, acc);
        for (long long e = e0 + stride; e < ncell; e += stride) {
            const long long c = cell(e);
            long long q[7];
            pts(c, q);
            double pv[7];
#pragma unroll
            for (int t = 0; t < 7; ++t) pv[t] = load_sc1(&pn[q[t]]);
            cellB(c, pv, load_sc1(&r[c]), x[c], al, ma, acc);
        }
        gsum_begin(1, acc);
        if (bad) break;
        loadA(pn, false);  // iteration it + 1: p_old = p_it
        const double tB = gsum_end(1);
        if (threadIdx.x == 0) fin_B(&ls, tB, it);
        __syncthreads();
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        if (bad) {
            ls.done = 1;
            ls.status = ST_COMM_TIMEOUT;
        }
        ls.xdone = ls.nalpha;  // x holds every alpha_j p_j: nothing for k_cg_finalize
        *st = ls;
    }
}

// Apply the x += alpha_j p_j the sweeps have not folded yet (j in [xdone,
// nalpha), at most CG_XFOLD of them: a stop after iteration it = 4m + 3
// leaves alpha_{4m} .. alpha_{4m+3}, whose p_j still sit in the four ring
// slots), in order, partial sums in a register (bitwise the reference's
// sequential updates).
static __global__ __launch_bounds__(NT) void k_cg_finalize(Geo g, PRing pr,
                                                    double* __restrict__ x, const CgState* st) {
    const int j0 = st->xdone, j1 = st->nalpha;  // at most CG_XFOLD pending
    if (j0 >= j1) return;
    const int ntiles = g.tiles_x * g.tiles_y * g.tiles_z;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        TileCoord c = tile_coord(g, t);
        if (!c.active) continue;
        long long idx = cidx(g, c.i, c.j, c.kb);
        for (int k = c.kb; k < c.ke; ++k, idx += g.ps) {
            double v = x[idx];
            for (int jj = j0; jj < j1; ++jj)
                v += st->alpha[jj % CG_XFOLD] * pr.p[jj % CG_XFOLD][idx];
            x[idx] = v;
        }
    }
}

// ===========================================================================
// Chronopoulos-Gear CG (opt-in, hip_proj_config_t.cg_variant = 1): the two
// dot products of an iteration come out of ONE reduction, so a Z-slab run
// needs one all-reduce per iteration instead of two. With
// w = A r and s = A p kept as vectors (Chronopoulos & Gear 1989):
//   p_i = r_i + beta_i p_{i-1},  s_i = w_i + beta_i s_{i-1}      (k_cc1)
//   x_{i+1} = x_i + alpha_i p_i, r_{i+1} = r_i - alpha_i s_i      (k_cc1)
//   w_{i+1} = A r_{i+1}; gamma = (r, r), delta = (w, r)          (k_cc2)
//   beta_{i+1} = gamma_{i+1} / gamma_i,
//   alpha_{i+1} = gamma_{i+1} / (delta_{i+1} - beta_{i+1} gamma_{i+1} / alpha_i)
// Same operator, boundary semantics (zero walls in r, lagged Neumann x),
// stopping rule and statistics as the textbook loop; the iterates differ by
// rounding, so it is gated against textbook CG (iterations +-2, residual),
// not bitwise. x += alpha p is folded every CG_XFOLD iterations as in k_cgB.
// ===========================================================================
// after the first w = A r_0: alpha_0 = (r,r) / (w,r) (the textbook's first
// (p, Ap) with p_0 = r_0), breakdown as fin_A
__device__ __forceinline__ void fin_cc0(CgState* st, double delta) {
    st->pAp = delta;
    if (fabs(delta) < 1e-30) {
        st->done = 1;
        st->status = ST_STAGNATED;
        st->iterations = 1;
    } else {
        st->alpha[0] = st->rho / delta;
        st->beta = 0.0;
    }
}

// after iteration it's reduction: convergence test as fin_B, then beta and
// the next alpha (its denominator standing in for the textbook's (p, Ap))
__device__ __forceinline__ void fin_cc(CgState* st, double gamma, double delta, int it,
                                       bool fold) {
    if (fold) st->xdone = it + 1;
    st->nalpha = it + 1;
    const double res = sqrt(gamma);
    st->res = res;
    st->iterations = it + 1;
    const bool check = (it % st->check_interval) == 0;
    const bool conv = (res < st->tol) || (res < st->abs_tol);
    if (check && conv) {
        st->done = 1;
        st->status = ST_CONVERGED;
    } else if (fabs(st->rho) < 1e-30) {
        st->done = 1;
        st->status = ST_STAGNATED;
    } else {
        const double beta = gamma / st->rho;
        const double den = delta - beta * gamma / st->alpha[it % CG_XFOLD];
        st->beta = beta;
        st->rho = gamma;
        st->pAp = den;
        if (it + 1 >= st->max_iter) {
            st->done = 1;
            st->status = conv ? ST_CONVERGED : ST_MAX_ITER;
        } else if (fabs(den) < 1e-30) {
            st->done = 1;
            st->status = ST_STAGNATED;
            st->iterations = it + 2;
        } else {
            st->alpha[(it + 1) % CG_XFOLD] = gamma / den;
        }
    }
}

static __global__ void k_finish_cc(CgState* st, const double* tot, int it, int fold, int init) {
    if (threadIdx.x != 0 || st->done) return;
    if (init) fin_cc0(st, tot[1]);
    else fin_cc(st, tot[0], tot[1], it, fold != 0);
}

// Pointwise part of iteration it over the interior cells, 16-B pairs:
// p_it into the ring slot pn, s in place, r in place; FOLD (it % 4 == 3)
// also x += the four pending alpha_j p_j in the reference's order.
template <bool FIRST, bool FOLD>
static __global__ __launch_bounds__(256) void k_cc1(SGeo g, double* __restrict__ r,
                                                    const double* __restrict__ w,
                                                    double* __restrict__ s,
                                                    const double* __restrict__ po,
                                                    double* __restrict__ pn, PPrev pv,
                                                    double* __restrict__ x, const CgState* st,
                                                    int it) {
    if (st->done) return;
    const double a = st->alpha[it % CG_XFOLD];
    const double ma = -a;
    const double beta = FIRST ? 0.0 : st->beta;
    double aq[CG_XFOLD - 1];
#pragma unroll
    for (int q = 0; q < CG_XFOLD - 1; ++q)
        aq[q] = FOLD ? st->alpha[(it + 1 + q) % CG_XFOLD] : 0.0;  // alpha_{it-3+q}
    const unsigned pairs = (unsigned)(g.px / 2);
    const unsigned nyi = (unsigned)(g.ny - 2);
    const unsigned n = pairs * nyi * (unsigned)(g.k1 - g.k0);
    for (unsigned e = blockIdx.x * blockDim.x + threadIdx.x; e < n; e += gridDim.x * blockDim.x) {
        const unsigned row = e / pairs;
        const int i0 = 2 * (int)(e - row * pairs);
        if (i0 >= g.nx) continue;
        const int j = 1 + (int)(row % nyi);
        const int k = g.k0 + (int)(row / nyi);
        const bool in0 = i0 >= 1 && i0 <= g.nx - 2;
        const bool in1 = i0 + 1 <= g.nx - 2;
        const long long idx = (long long)k * g.ps + (long long)j * g.px + i0;
        const double2 rv = ld2(r, idx);
        const double2 wv = ld2(w, idx);
        const double2 pf = FIRST ? rv : fma2p(rv, beta, ld2(po, idx));
        const double2 sf = FIRST ? wv : fma2p(wv, beta, ld2(s, idx));
        const double2 pw = make_double2(in0 ? pf.x : 0.0, in1 ? pf.y : 0.0);
        const double2 sw = make_double2(in0 ? sf.x : 0.0, in1 ? sf.y : 0.0);
        st2(pn, idx, pw);
        st2(s, idx, sw);
        st2(r, idx, make_double2(in0 ? rv.x + ma * sf.x : rv.x, in1 ? rv.y + ma * sf.y : rv.y));
        if (FOLD) {
            const double2 xo = ld2(x, idx);
            const double2 qa = ld2(pv.q[0], idx), qb = ld2(pv.q[1], idx), qc = ld2(pv.q[2], idx);
            double2 xw;
            xw.x = in0 ? (((xo.x + aq[0] * qa.x) + aq[1] * qb.x) + aq[2] * qc.x) + a * pf.x : xo.x;
            xw.y = in1 ? (((xo.y + aq[0] * qa.y) + aq[1] * qb.y) + aq[2] * qc.y) + a * pf.y : xo.y;
            st2(x, idx, xw);
        }
    }
}

// Two-value form of grid_sum_last_n (partials[pofs + b] and partials[nb +
// pofs + b], nb = ptot, or gridDim.x when ptot is 0). With ptot > 0 several
// launches on one stream share the reduction: this launch owns slots [pofs,
// pofs + gridDim.x) of ptot, and the last of all ptot workgroups finishes.
template <int NTH>
__device__ __forceinline__ bool grid_sum2_last(double b0, double b1, double* partials,
                                               unsigned* counter, double* sh, int* flag,
                                               double& t0, double& t1, unsigned pofs = 0,
                                               unsigned ptot = 0) {
    const unsigned nb = ptot ? ptot : gridDim.x;
    if (threadIdx.x == 0) {
        store_sc1(&partials[pofs + blockIdx.x], b0);
        store_sc1(&partials[nb + pofs + blockIdx.x], b1);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned t = __hip_atomic_fetch_add((gu32*)counter, 1u, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
        *flag = (t == nb - 1) ? 1 : 0;
    }
    __syncthreads();
    if (*flag == 0) return false;
    double s0 = 0.0, s1 = 0.0;
    for (unsigned b = threadIdx.x; b < nb; b += NTH) {
        s0 += load_sc1(&partials[b]);
        s1 += load_sc1(&partials[nb + b]);
    }
    s0 = wave_sum(s0);
    s1 = wave_sum(s1);
    if ((threadIdx.x & 63) == 0) {
        sh[threadIdx.x >> 6] = s0;
        sh[NTH / 64 + (threadIdx.x >> 6)] = s1;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double a0 = 0.0, a1 = 0.0;
#pragma unroll
        for (int q = 0; q < NTH / 64; ++q) {
            a0 += sh[q];
            a1 += sh[NTH / 64 + q];
        }
        t0 = a0;
        t1 = a1;
        __hip_atomic_store((gu32*)counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return true;
}

// The end of the single-reduction iteration's one reduction (the finishing
// workgroup, thread 0): on Z-slabs the all-ranks sum through the device
// mailbox, or left in dsum for an RCCL all-reduce + k_finish_cc; on one
// device fin_cc0 / fin_cc directly.
__device__ __forceinline__ void cc_reduce_finish(CgState* st, double tg, double td, int it,
                                                 bool init, bool dist, Mbox* mb, double* dsum) {
    if (dist && mb) {
        double gg, gd;
        if (mbox_allreduce2(mb, tg, td, &gg, &gd)) {
            if (init) fin_cc0(st, gd);
            else fin_cc(st, gg, gd, it, (it % CG_XFOLD) == CG_XFOLD - 1);
        } else {
            comm_fail(st);
        }
    } else if (dist) {
        dsum[0] = tg;
        dsum[1] = td;
    } else if (init) {
        fin_cc0(st, td);
    } else {
        fin_cc(st, tg, td, it, (it % CG_XFOLD) == CG_XFOLD - 1);
    }
}

// w = A r on the row-pair tiling (k_cgA's stencil with p = r), written to w,
// and the one reduction of iteration it: gamma = (r, r), delta = (w, r).
// g.part_total > 0 (Z-slabs, the fused iteration): the launch covers the two
// edge planes (kmode 1) and shares the reduction with the k_ccf launch of the
// interior planes before it (its partials first).
// INIT: the w = A r_0 before iteration 0 (fin_cc0; gamma_0 comes from setup).
// WST = false (the fused iteration on Z-slabs, ccf.hpp): w stays in registers
template <int TY, bool DIST, bool INIT, bool WST = true>
static __global__ __launch_bounds__(64 * TY) void k_cc2(SGeo g, Lap L,
                                                        const double* __restrict__ r,
                                                        double* __restrict__ w, CgState* st,
                                                        double* partials, unsigned* counter,
                                                        int it, double* dsum, Mbox* mb) {
    __shared__ double2 rows[2][TY + 2][64];
    __shared__ double sh[2 * TY];
    __shared__ int flag;
    if (st->done) return;
    RowPair c = row_pair<TY>(g);
    const bool halo = (c.w == 0) || (c.w == TY - 1);
    const int jh = (c.w == 0) ? max(c.j - 1, 0) : min(c.j + 1, g.ny - 1);
    const int hslot = (c.w == 0) ? 0 : TY + 1;
    const long long hoff = (long long)(jh - min(c.j, g.ny - 1)) * g.px;
    const bool xok = c.i0 < g.nx;
    const bool eok_l = c.lane == 0 && c.i0 >= 1 && xok;
    const bool eok_r = c.lane == 63 && c.i0 + 2 < g.nx;
    const double2 zero = make_double2(0.0, 0.0);
    double accg = 0.0, accd = 0.0;
    long long idx = c.idx;
    double2 pm = xok ? ld2(r, idx - g.sz) : zero;
    double2 pc = xok ? ld2(r, idx) : zero;
    double2 hc = (xok && halo) ? ld2(r, idx + hoff) : zero;
    int buf = 0;
    for (int k = c.kb; k < c.ke; ++k, idx += g.ps) {
        const long long ip = idx + g.sz;
        const double2 pp = xok ? ld2(r, ip) : zero;
        const double2 hn = (xok && halo && k + 1 < c.ke) ? ld2(r, ip + hoff) : zero;
        const double el = eok_l ? r[idx - 1] : 0.0;
        const double er = eok_r ? r[idx + 2] : 0.0;
        rows[buf][c.w + 1][c.lane] = pc;
        if (halo) rows[buf][hslot][c.lane] = hc;
        __syncthreads();
        const double2 ys = rows[buf][c.w][c.lane];
        const double2 yn = rows[buf][c.w + 2][c.lane];
        double left = __shfl_up(pc.y, 1, 64);
        double right = __shfl_down(pc.x, 1, 64);
        if (c.lane == 0) left = el;
        if (c.lane == 63) right = er;
        const double w0 = -lap7(L, pc.x, left, pc.y, ys.x, yn.x, pm.x, pp.x);
        const double w1 = -lap7(L, pc.y, pc.x, right, ys.y, yn.y, pm.y, pp.y);
        if (WST && c.act) st2(w, idx, make_double2(c.in0 ? w0 : 0.0, c.in1 ? w1 : 0.0));
        if (c.in0) {
            accg += pc.x * pc.x;
            accd += w0 * pc.x;
        }
        if (c.in1) {
            accg += pc.y * pc.y;
            accd += w1 * pc.y;
        }
        pm = pc;
        pc = pp;
        hc = hn;
        buf ^= 1;
    }
    accg = wave_sum(accg);
    accd = wave_sum(accd);
    if (c.lane == 0) {
        sh[c.w] = accg;
        sh[TY + c.w] = accd;
    }
    __syncthreads();
    double bg = 0.0, bd = 0.0;
    if (threadIdx.x == 0)
        for (int q = 0; q < TY; ++q) {
            bg += sh[q];
            bd += sh[TY + q];
        }
    double tg, td;
    double* shs = (double*)&rows[0][0][0];
    if (grid_sum2_last<64 * TY>(bg, bd, partials, counter, shs, &flag, tg, td,
                                (unsigned)g.part_ofs, (unsigned)g.part_total) &&
        threadIdx.x == 0)
        cc_reduce_finish(st, tg, td, it, INIT, DIST, mb, dsum);
}

// ---------------------------------------------------------------------------
// Boundary conditions as pure gathers from interior cells (race-free):
//   Neumann  (boundary_conditions_core_impl.h:41-85): c -> clamp(c, 1, n-2)
//   Periodic (:90-134):                               0 -> n-2, n-1 -> 1
// The reference applies x faces, then y faces, then z faces in place; the
// composition of those copies is exactly this per-coordinate map, edges and
// corners included. Dirichlet (:139-186) keeps the z > y > x face precedence.
// Threads cover the boundary shell: z faces (3-D) plus the x/y ring of every
// plane. mode: 0 Neumann, 1 periodic, 2 Dirichlet.
// ---------------------------------------------------------------------------
struct DirVals {
    double left, right, top, bottom, front, back;
};

__device__ __forceinline__ int bc_map(int c, int n, int mode) {
    if (mode == 0) return c == 0 ? 1 : (c == n - 1 ? n - 2 : c);
    return c == 0 ? n - 2 : (c == n - 1 ? 1 : c);
}

// In a Z-slab the z faces exist only on the edge ranks (lo_face / hi_face);
// the x/y ring is applied on every local plane, halo planes included (their
// owner applies the identical gather to the same values).
// Boundary-shell cell e of the enumeration k_bc_shell / k_rx_shell share:
// the x/y ring of every local plane, then the z faces the rank owns.
__device__ __forceinline__ long long shell_total(const Geo& g) {
    const bool is3d = g.nz > 1;
    const long long ring = 2LL * g.nx + 2LL * (g.ny - 2);
    const long long plane = (long long)g.nx * g.ny;
    return ring * g.nz + ((is3d && g.lo_face) ? plane : 0) + ((is3d && g.hi_face) ? plane : 0);
}
__device__ __forceinline__ void shell_cell(const Geo& g, long long e, int& i, int& j, int& k,
                                           bool& zlo, bool& zhi) {
    const bool is3d = g.nz > 1;
    const bool lo = is3d && g.lo_face, hi = is3d && g.hi_face;
    const long long ring = 2LL * g.nx + 2LL * (g.ny - 2);  // x/y boundary ring of one plane
    const long long nring = ring * g.nz;
    const long long plane = (long long)g.nx * g.ny;
    if (e < nring) {
        k = (int)(e / ring);
        long long q = e % ring;
        if (q < g.nx) { i = (int)q; j = 0; }
        else if (q < 2LL * g.nx) { i = (int)(q - g.nx); j = g.ny - 1; }
        else if (q < 2LL * g.nx + (g.ny - 2)) { i = 0; j = (int)(q - 2LL * g.nx) + 1; }
        else { i = g.nx - 1; j = (int)(q - 2LL * g.nx - (g.ny - 2)) + 1; }
    } else {
        long long q = e - nring;
        k = (lo && q < plane) ? 0 : g.nz - 1;
        q = q % plane;
        j = (int)(q / g.nx);
        i = (int)(q % g.nx);
    }
    zlo = lo && k == 0;
    zhi = hi && k == g.nz - 1;
}

static __global__ __launch_bounds__(256) void k_bc_shell(Geo g, double* __restrict__ f, int mode,
                                                  DirVals dv) {
    const long long total = shell_total(g);
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {
        int i, j, k;
        bool zlo, zhi;
        shell_cell(g, e, i, j, k, zlo, zhi);
        const long long dst = cidx(g, i, j, k);
        if (mode == 2) {
            double v;
            if (zlo) v = dv.back;
            else if (zhi) v = dv.front;
            else if (j == 0) v = dv.bottom;
            else if (j == g.ny - 1) v = dv.top;
            else if (i == 0) v = dv.left;
            else v = dv.right;
            f[dst] = v;
        } else {
            int si = bc_map(i, g.nx, mode), sj = bc_map(j, g.ny, mode);
            int sk = (zlo || zhi) ? bc_map(k, g.nz, mode) : k;
            f[dst] = f[cidx(g, si, sj, sk)];
        }
    }
}

// Max over a full field (stats: max temperature, solver_registry.c:52-62),
// planes [k_first, k_first + gridDim.z).
static __global__ __launch_bounds__(256) void k_field_max(Geo g, const double* __restrict__ f,
                                                   unsigned long long* out, int k_first) {
    __shared__ double sh[4];
    const int i = blockIdx.x * 64 + (threadIdx.x & 63);
    const int j = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int k = k_first + (int)blockIdx.z;
    double m = -INFINITY;
    if (i < g.nx && j < g.ny) {
        double v = f[cidx(g, i, j, k)];
        if (!isnan(v)) m = v;
    }
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = fmax(fmax(sh[0], sh[1]), fmax(sh[2], sh[3]));
        atomicMax(out, ord_enc(a));
    }
}

// ---------------------------------------------------------------------------
// Energy equation (energy_solver.c:21-176): explicit Euler on the corrected
// velocity, T_new = T + dt(-(u.grad)T + alpha lap T), boundary cells copied;
// any non-finite T_new sets red[5] (the reference's CFD_ERROR_DIVERGED scan).
// 40 B/cell: read T (stencil), u, v, w; write T_new.
// ---------------------------------------------------------------------------
struct EnergyCoef {
    double inv_2dx, inv_2dy, inv_2dz, inv_dx2, inv_dy2, inv_dz2, alpha, dt;
};

static __global__ __launch_bounds__(256) void k_energy(Geo g, EnergyCoef ec, const double* __restrict__ T,
                                                const double* __restrict__ U,
                                                const double* __restrict__ V,
                                                const double* __restrict__ W,
                                                double* __restrict__ Tn,
                                                unsigned long long* red) {
    const int i = blockIdx.x * 64 + (threadIdx.x & 63);
    const int j = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int k = blockIdx.z;
    if (i >= g.nx || j >= g.ny) return;
    const long long idx = cidx(g, i, j, k);
    const bool interior = (i >= 1 && i <= g.nx - 2 && j >= 1 && j <= g.ny - 2 &&
                           k >= g.k0 && k < g.k1);
    double tn;
    if (interior) {
        const long long px = g.px, sz = g.sz;
        const double Tc = T[idx];
        double dT_dx = (T[idx + 1] - T[idx - 1]) * ec.inv_2dx;
        double dT_dy = (T[idx + px] - T[idx - px]) * ec.inv_2dy;
        double dT_dz = (T[idx + sz] - T[idx - sz]) * ec.inv_2dz;
        double adv = U[idx] * dT_dx + V[idx] * dT_dy + W[idx] * dT_dz;
        double d2x = (T[idx + 1] - 2.0 * Tc + T[idx - 1]) * ec.inv_dx2;
        double d2y = (T[idx + px] - 2.0 * Tc + T[idx - px]) * ec.inv_dy2;
        double d2z = (T[idx + sz] - 2.0 * Tc + T[idx - sz]) * ec.inv_dz2;
        double diff = ec.alpha * (d2x + d2y + d2z);
        double dT = ec.dt * (-adv + diff + 0.0);
        tn = Tc + dT;
    } else {
        tn = T[idx];
    }
    Tn[idx] = tn;
    if (!isfinite(tn)) atomicOr(&red[5], 1ull);
}

// Thermal boundary conditions (energy_solver.c:204-334), in the reference's
// face order as three gather passes: pass 0 = left/right (x faces, every
// local plane), pass 1 = bottom/top (reads the x-face values pass 0 wrote),
// pass 2 = back/front (whole planes, edge ranks only). Types per face:
// 0 periodic, 1 Neumann, 2 Dirichlet (bc_type_t); -1 = leave the face.
struct ThermalFaces {
    int type[6];   // left, right, bottom, top, back, front
    double val[6];
};

static __global__ __launch_bounds__(256) void k_thermal_bc(Geo g, double* __restrict__ T, ThermalFaces tf,
                                                    int pass) {
    const long long plane = (long long)g.nx * g.ny;
    long long total;
    if (pass == 0) total = 2LL * g.ny * g.nz;
    else if (pass == 1) total = 2LL * g.nx * g.nz;
    else total = 2LL * plane;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {
        int i, j, k, face;
        if (pass == 0) {
            face = (int)(e % 2);           // 0 left, 1 right
            long long q = e / 2;
            j = (int)(q % g.ny);
            k = (int)(q / g.ny);
            i = face == 0 ? 0 : g.nx - 1;
        } else if (pass == 1) {
            face = 2 + (int)(e % 2);       // 2 bottom, 3 top
            long long q = e / 2;
            i = (int)(q % g.nx);
            k = (int)(q / g.nx);
            j = face == 2 ? 0 : g.ny - 1;
        } else {
            face = 4 + (int)(e / plane);   // 4 back, 5 front
            if ((face == 4 && !g.lo_face) || (face == 5 && !g.hi_face)) continue;
            long long q = e % plane;
            j = (int)(q / g.nx);
            i = (int)(q % g.nx);
            k = face == 4 ? 0 : g.nz - 1;
        }
        const int t = tf.type[face];
        if (t < 0) continue;
        const long long dst = cidx(g, i, j, k);
        if (t == 2) {
            T[dst] = tf.val[face];
            continue;
        }
        int si = i, sj = j, sk = k;
        const bool per = (t == 0);
        switch (face) {
            case 0: si = per ? g.nx - 2 : 1; break;
            case 1: si = per ? 1 : g.nx - 2; break;
            case 2: sj = per ? g.ny - 2 : 1; break;
            case 3: sj = per ? 1 : g.ny - 2; break;
            case 4: sk = per ? g.nz - 2 : 1; break;
            default: sk = per ? 1 : g.nz - 2; break;
        }
        T[dst] = T[cidx(g, si, sj, sk)];
    }
}

// ---------------------------------------------------------------------------
// RK4 (solver_rk4.c:69-259) with the shared momentum RHS
// (ns_momentum_rhs_scalar.h:49-190). One fused kernel per stage s:
//   k      = RHS(cur)                      (interior; 0 on boundary cells)
//   acc    = k | acc + 2k | acc + 2k       (s = 0, 1, 2: the reference's
//                                           k1 + 2 k2 + 2 k3 + k4, left to right)
//   out    = clamp(Q0 + fac_s k)           (s < 3; fac = dt/2, dt/2, dt)
//   out    = clamp(Q0 + dt/6 (acc + k))    (s = 3, written in place over Q0)
// so the stage derivatives never touch HBM. The stencil uses the
// reference's periodic neighbour indices (i = 1 reads nx-2, not the ghost).
// ---------------------------------------------------------------------------
struct RkCoef {
    double inv_2dz, inv_dz2;
    double mu, beta, T_ref, g0, g1, g2;
    double fac;   // dt/2, dt/2, dt, dt/6
};

struct Fld4 {
    double* f[4];  // u, v, w, p
};

__device__ __forceinline__ double clampl(double x, double lim) { return fmax(-lim, fmin(lim, x)); }

// One cell's RHS (ns_momentum_rhs_scalar.h:49-190 operation order): the 7
// values of u, v, w, p around the cell (periodic neighbour indices already
// resolved), rho, dx[i], dy[j], the source-table entries and T; kr = 0 where
// the reference skips the cell (rho or a spacing below 1e-10).
struct RkNbr {
    double c[4], l[4], r[4], d[4], u[4], m[4], p[4];  // centre, x-, x+, y-, y+, z-, z+
};

template <bool BUOY>
__device__ __forceinline__ void rk_rhs(const RkCoef& rc, const RkNbr& n, double r, double dxi,
                                       double dyj, double su, double sv, double Tc,
                                       double (&kr)[4]) {
    if (!(r <= 1e-10) && !(fabs(dxi) < 1e-10) && !(fabs(dyj) < 1e-10)) {
        const double tdx = 2.0 * dxi, tdy = 2.0 * dyj;
        const double dxx = dxi * dxi, dyy = dyj * dyj;
        const double uc = n.c[0], vc = n.c[1], wc = n.c[2];
        double du_dx = (n.r[0] - n.l[0]) / tdx, du_dy = (n.u[0] - n.d[0]) / tdy;
        double du_dz = (n.p[0] - n.m[0]) * rc.inv_2dz;
        double dv_dx = (n.r[1] - n.l[1]) / tdx, dv_dy = (n.u[1] - n.d[1]) / tdy;
        double dv_dz = (n.p[1] - n.m[1]) * rc.inv_2dz;
        double dw_dx = (n.r[2] - n.l[2]) / tdx, dw_dy = (n.u[2] - n.d[2]) / tdy;
        double dw_dz = (n.p[2] - n.m[2]) * rc.inv_2dz;
        double dp_dx = (n.r[3] - n.l[3]) / tdx, dp_dy = (n.u[3] - n.d[3]) / tdy;
        double dp_dz = (n.p[3] - n.m[3]) * rc.inv_2dz;
        double d2u_dx2 = (n.r[0] - 2.0 * uc + n.l[0]) / dxx;
        double d2u_dy2 = (n.u[0] - 2.0 * uc + n.d[0]) / dyy;
        double d2u_dz2 = (n.p[0] - 2.0 * uc + n.m[0]) * rc.inv_dz2;
        double d2v_dx2 = (n.r[1] - 2.0 * vc + n.l[1]) / dxx;
        double d2v_dy2 = (n.u[1] - 2.0 * vc + n.d[1]) / dyy;
        double d2v_dz2 = (n.p[1] - 2.0 * vc + n.m[1]) * rc.inv_dz2;
        double d2w_dx2 = (n.r[2] - 2.0 * wc + n.l[2]) / dxx;
        double d2w_dy2 = (n.u[2] - 2.0 * wc + n.d[2]) / dyy;
        double d2w_dz2 = (n.p[2] - 2.0 * wc + n.m[2]) * rc.inv_dz2;
        double nu = rc.mu / fmax(r, 1e-10);
        nu = fmin(nu, 1.0);
        du_dx = clampl(du_dx, 100.0); du_dy = clampl(du_dy, 100.0); du_dz = clampl(du_dz, 100.0);
        dv_dx = clampl(dv_dx, 100.0); dv_dy = clampl(dv_dy, 100.0); dv_dz = clampl(dv_dz, 100.0);
        dw_dx = clampl(dw_dx, 100.0); dw_dy = clampl(dw_dy, 100.0); dw_dz = clampl(dw_dz, 100.0);
        dp_dx = clampl(dp_dx, 100.0); dp_dy = clampl(dp_dy, 100.0); dp_dz = clampl(dp_dz, 100.0);
        d2u_dx2 = clampl(d2u_dx2, 1000.0); d2u_dy2 = clampl(d2u_dy2, 1000.0);
        d2u_dz2 = clampl(d2u_dz2, 1000.0); d2v_dx2 = clampl(d2v_dx2, 1000.0);
        d2v_dy2 = clampl(d2v_dy2, 1000.0); d2v_dz2 = clampl(d2v_dz2, 1000.0);
        d2w_dx2 = clampl(d2w_dx2, 1000.0); d2w_dy2 = clampl(d2w_dy2, 1000.0);
        d2w_dz2 = clampl(d2w_dz2, 1000.0);
        double sw = 0.0;
        if (BUOY) {
            const double dT = Tc - rc.T_ref;
            su += -rc.beta * dT * rc.g0;
            sv += -rc.beta * dT * rc.g1;
            sw += -rc.beta * dT * rc.g2;
        }
        kr[0] = -uc * du_dx - vc * du_dy - wc * du_dz - dp_dx / r +
                nu * (d2u_dx2 + d2u_dy2 + d2u_dz2) + su;
        kr[1] = -uc * dv_dx - vc * dv_dy - wc * dv_dz - dp_dy / r +
                nu * (d2v_dx2 + d2v_dy2 + d2v_dz2) + sv;
        kr[2] = -uc * dw_dx - vc * dw_dy - wc * dw_dz - dp_dz / r +
                nu * (d2w_dx2 + d2w_dy2 + d2w_dz2) + sw;
        double div = du_dx + dv_dy + dw_dz;
        div = fmax(-10.0, fmin(10.0, div));
        kr[3] = -0.1 * r * div;
    }
}

template <int STAGE, bool BUOY>
__global__ __launch_bounds__(256) void k_rk_stage(Geo g, RkCoef rc, Fld4 cur, Fld4 q0, Fld4 acc,
                                                  Fld4 out, const double* __restrict__ rho,
                                                  const double* __restrict__ T,
                                                  const double* __restrict__ dxa,
                                                  const double* __restrict__ dya,
                                                  const double* __restrict__ su_row,
                                                  const double* __restrict__ sv_col) {
    const int i = blockIdx.x * 64 + (threadIdx.x & 63);
    const int j = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int k = blockIdx.z;
    if (i >= g.nx || j >= g.ny) return;
    const long long idx = cidx(g, i, j, k);
    const bool interior = (i >= 1 && i <= g.nx - 2 && j >= 1 && j <= g.ny - 2 &&
                           k >= g.k0 && k < g.k1);
    double kr[4] = {0.0, 0.0, 0.0, 0.0};
    if (interior) {
        const long long il = (i > 1) ? idx - 1 : cidx(g, g.nx - 2, j, k);
        const long long ir = (i < g.nx - 2) ? idx + 1 : cidx(g, 1, j, k);
        const long long jd = (j > 1) ? idx - g.px : cidx(g, i, g.ny - 2, k);
        const long long ju = (j < g.ny - 2) ? idx + g.px : cidx(g, i, 1, k);
        long long kd = idx, ku = idx;   // 2-D: z terms vanish (stride 0)
        if (g.sz) {
            kd = (k > 1) ? idx - g.sz : cidx(g, i, j, g.nz - 2);
            ku = (k < g.nz - 2) ? idx + g.sz : cidx(g, i, j, 1);
        }
        RkNbr n;
#pragma unroll
        for (int f = 0; f < 4; ++f) {
            n.c[f] = cur.f[f][idx];
            n.l[f] = cur.f[f][il];
            n.r[f] = cur.f[f][ir];
            n.d[f] = cur.f[f][jd];
            n.u[f] = cur.f[f][ju];
            n.m[f] = cur.f[f][kd];
            n.p[f] = cur.f[f][ku];
        }
        rk_rhs<BUOY>(rc, n, rho[idx], dxa[i], dya[j], su_row[j], sv_col[i],
                     BUOY ? T[idx] : 0.0, kr);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        double o;
        if (STAGE == 0) {
            acc.f[q][idx] = kr[q];
            o = q0.f[q][idx] + rc.fac * kr[q];
        } else if (STAGE < 3) {
            acc.f[q][idx] = acc.f[q][idx] + 2.0 * kr[q];
            o = q0.f[q][idx] + rc.fac * kr[q];
        } else {
            o = q0.f[q][idx] + rc.fac * (acc.f[q][idx] + kr[q]);
        }
        if (q < 3) o = fmax(-100.0, fmin(100.0, o));
        out.f[q][idx] = o;
    }
}

// First and second differences of one field at the cells (i0, i0 + 1) of a
// pair (r02b): c2 the pair, d2 / u2 the
// (periodically resolved) y- / y+ rows, m2 / p2 the z- / z+ planes, xl the
// left of i0, ar the right of i0, bl the left of i0 + 1, xr the right of
// i0 + 1. Same expressions and order as rk_rhs, so the values are bitwise.
struct RkD1 {
    double dx, dy, dz, xx, yy, zz;
};

__device__ __forceinline__ void rk_pair_diffs(const RkCoef& rc, double2 c2, double2 d2, double2 u2,
                                              double2 m2, double2 p2, double xl, double ar,
                                              double bl, double xr, double dxa0, double dxa1,
                                              double dyj, RkD1& da, RkD1& db) {
    const double tdxa = 2.0 * dxa0, tdxb = 2.0 * dxa1, tdy = 2.0 * dyj;
    const double dxxa = dxa0 * dxa0, dxxb = dxa1 * dxa1, dyy = dyj * dyj;
    da.dx = (ar - xl) / tdxa;
    da.dy = (u2.x - d2.x) / tdy;
    da.dz = (p2.x - m2.x) * rc.inv_2dz;
    da.xx = (ar - 2.0 * c2.x + xl) / dxxa;
    da.yy = (u2.x - 2.0 * c2.x + d2.x) / dyy;
    da.zz = (p2.x - 2.0 * c2.x + m2.x) * rc.inv_dz2;
    db.dx = (xr - bl) / tdxb;
    db.dy = (u2.y - d2.y) / tdy;
    db.dz = (p2.y - m2.y) * rc.inv_2dz;
    db.xx = (xr - 2.0 * c2.y + bl) / dxxb;
    db.yy = (u2.y - 2.0 * c2.y + d2.y) / dyy;
    db.zz = (p2.y - 2.0 * c2.y + m2.y) * rc.inv_dz2;
}

// The stage derivatives of a pair (rk_rhs's expressions): diffs(f, da, db)
// yields field f's differences; p first (its gradient enters u, v, w), then
// u, v, w, so only one field's neighbourhood is live at a time.
template <bool BUOY, class Diffs>
__device__ __forceinline__ void rk_pair_kr(const RkCoef& rc, Diffs diffs, double2 uc, double2 vc,
                                           double2 wc, double2 r2, double2 t2, double su,
                                           double sv0, double sv1, bool oka, bool okb,
                                           double (&kra)[4], double (&krb)[4]) {
    RkD1 pa_, pb_;
    diffs(3, pa_, pb_);
    const double dpxa = clampl(pa_.dx, 100.0), dpya = clampl(pa_.dy, 100.0),
                 dpza = clampl(pa_.dz, 100.0);
    const double dpxb = clampl(pb_.dx, 100.0), dpyb = clampl(pb_.dy, 100.0),
                 dpzb = clampl(pb_.dz, 100.0);
    const double nua = fmin(rc.mu / fmax(r2.x, 1e-10), 1.0);
    const double nub = fmin(rc.mu / fmax(r2.y, 1e-10), 1.0);
    double sa[3] = {su, sv0, 0.0};
    double sb[3] = {su, sv1, 0.0};
    if (BUOY) {
        const double dTa = t2.x - rc.T_ref, dTb = t2.y - rc.T_ref;
        sa[0] += -rc.beta * dTa * rc.g0;
        sa[1] += -rc.beta * dTa * rc.g1;
        sa[2] += -rc.beta * dTa * rc.g2;
        sb[0] += -rc.beta * dTb * rc.g0;
        sb[1] += -rc.beta * dTb * rc.g1;
        sb[2] += -rc.beta * dTb * rc.g2;
    }
    const double gpa[3] = {dpxa, dpya, dpza}, gpb[3] = {dpxb, dpyb, dpzb};
    double diva = 0.0, divb = 0.0;  // du_dx + dv_dy + dw_dz (clamped terms)
#pragma unroll
    for (int f = 0; f < 3; ++f) {
        RkD1 da, db;
        diffs(f, da, db);
        da.dx = clampl(da.dx, 100.0); da.dy = clampl(da.dy, 100.0); da.dz = clampl(da.dz, 100.0);
        db.dx = clampl(db.dx, 100.0); db.dy = clampl(db.dy, 100.0); db.dz = clampl(db.dz, 100.0);
        da.xx = clampl(da.xx, 1000.0); da.yy = clampl(da.yy, 1000.0); da.zz = clampl(da.zz, 1000.0);
        db.xx = clampl(db.xx, 1000.0); db.yy = clampl(db.yy, 1000.0); db.zz = clampl(db.zz, 1000.0);
        if (oka)
            kra[f] = -uc.x * da.dx - vc.x * da.dy - wc.x * da.dz - gpa[f] / r2.x +
                     nua * (da.xx + da.yy + da.zz) + sa[f];
        if (okb)
            krb[f] = -uc.y * db.dx - vc.y * db.dy - wc.y * db.dz - gpb[f] / r2.y +
                     nub * (db.xx + db.yy + db.zz) + sb[f];
        const double ta = (f == 0) ? da.dx : (f == 1 ? da.dy : da.dz);
        const double tb = (f == 0) ? db.dx : (f == 1 ? db.dy : db.dz);
        diva = (f == 0) ? ta : diva + ta;
        divb = (f == 0) ? tb : divb + tb;
    }
    if (oka) kra[3] = -0.1 * r2.x * fmax(-10.0, fmin(10.0, diva));
    if (okb) krb[3] = -0.1 * r2.y * fmax(-10.0, fmin(10.0, divb));
}

// The stage update of one pair of field q (solver_rk4.c stage sums): stage
// 0 stores k into the running sum, 1-2 add 2k, 3 forms the final state.
template <int STAGE, int FL = 0>
__device__ __forceinline__ void rk_pair_update(const RkCoef& rc, const Fld4& q0, const Fld4& acc,
                                               const Fld4& out, int q, long long idx, double ka,
                                               double kb) {
    const double2 q02 = ld2v<FL>(q0.f[q], idx);
    double2 o;
    if (STAGE == 0) {
        st2v<FL>(acc.f[q], idx, make_double2(ka, kb));
        o = make_double2(q02.x + rc.fac * ka, q02.y + rc.fac * kb);
    } else if (STAGE < 3) {
        const double2 a2 = ld2v<FL>(acc.f[q], idx);
        st2v<FL>(acc.f[q], idx, make_double2(a2.x + 2.0 * ka, a2.y + 2.0 * kb));
        o = make_double2(q02.x + rc.fac * ka, q02.y + rc.fac * kb);
    } else {
        const double2 a2 = ld2v<FL>(acc.f[q], idx);
        o = make_double2(q02.x + rc.fac * (a2.x + ka), q02.y + rc.fac * (a2.y + kb));
    }
    if (q < 3) {
        o.x = fmax(-100.0, fmin(100.0, o.x));
        o.y = fmax(-100.0, fmin(100.0, o.y));
    }
    st2v<FL>(out.f[q], idx, o);
}

// The same stage on x pairs (r02b): each lane owns cells (i0, i0 + 1) and
// moves every field with 16-B loads / stores; the cell's x neighbours are the
// pair's other cell or one scalar load (the periodic indices of i = 1 and
// nx - 2 by address), y / z neighbours are pair loads of the (periodically
// resolved) neighbour row / plane. Half the load instructions of k_rk_stage;
// rk_rhs's expressions, so the values are bitwise the per-cell kernel's.
template <int STAGE, bool BUOY>
__global__ __launch_bounds__(256) void k_rk_stage2(Geo g, RkCoef rc, Fld4 cur, Fld4 q0, Fld4 acc,
                                                   Fld4 out, const double* __restrict__ rho,
                                                   const double* __restrict__ T,
                                                   const double* __restrict__ dxa,
                                                   const double* __restrict__ dya,
                                                   const double* __restrict__ su_row,
                                                   const double* __restrict__ sv_col) {
    const int i0 = blockIdx.x * 128 + 2 * (threadIdx.x & 63);
    const int j = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int k = blockIdx.z;
    if (i0 >= g.nx || j >= g.ny) return;
    const long long idx = cidx(g, i0, j, k);
    const bool rowin = (j >= 1 && j <= g.ny - 2 && k >= g.k0 && k < g.k1);
    const bool ina = rowin && i0 >= 1 && i0 <= g.nx - 2;
    const bool inb = rowin && i0 + 1 <= g.nx - 2;
    double kra[4] = {0.0, 0.0, 0.0, 0.0}, krb[4] = {0.0, 0.0, 0.0, 0.0};
    if (ina || inb) {
        const long long row = idx - i0;
        const long long jd = (j > 1) ? idx - g.px : cidx(g, i0, g.ny - 2, k);
        const long long ju = (j < g.ny - 2) ? idx + g.px : cidx(g, i0, 1, k);
        long long kd = idx, ku = idx;  // 2-D: z terms vanish (stride 0)
        if (g.sz) {
            kd = (k > 1) ? idx - g.sz : cidx(g, i0, j, g.nz - 2);
            ku = (k < g.nz - 2) ? idx + g.sz : cidx(g, i0, j, 1);
        }
        // x neighbours outside the pair: left of i0, right of i0 + 1
        const long long la = (i0 > 1) ? idx - 1 : row + (g.nx - 2);
        const long long rb = (i0 + 1 < g.nx - 2) ? idx + 2 : row + 1;
        const double2 r2 = ld2(rho, idx);
        const double2 t2 = BUOY ? ld2(T, idx) : make_double2(0.0, 0.0);
        const double dyj = dya[j], su = su_row[j];
        const double dxa0 = dxa[i0], dxa1 = dxa[min(i0 + 1, g.nx - 1)];
        const bool oka = ina && !(r2.x <= 1e-10) && !(fabs(dxa0) < 1e-10) && !(fabs(dyj) < 1e-10);
        const bool okb = inb && !(r2.y <= 1e-10) && !(fabs(dxa1) < 1e-10) && !(fabs(dyj) < 1e-10);
        const double2 uc = ld2(cur.f[0], idx), vc = ld2(cur.f[1], idx), wc = ld2(cur.f[2], idx);
        auto diffs = [&](int f, RkD1& da, RkD1& db) __attribute__((always_inline)) {
            const double* F = cur.f[f];
            const double2 c2 = ld2(F, idx), d2 = ld2(F, jd), u2 = ld2(F, ju);
            const double2 m2 = ld2(F, kd), p2 = ld2(F, ku);
            const double xl = F[la], xr = F[rb];
            const double ar = (i0 < g.nx - 2) ? c2.y : F[row + 1];
            const double bl = (i0 + 1 > 1) ? c2.x : F[row + (g.nx - 2)];
            rk_pair_diffs(rc, c2, d2, u2, m2, p2, xl, ar, bl, xr, dxa0, dxa1, dyj, da, db);
        };
        rk_pair_kr<BUOY>(rc, diffs, uc, vc, wc, r2, t2, su, sv_col[i0],
                         sv_col[min(i0 + 1, g.nx - 1)], oka, okb, kra, krb);
    }
#pragma unroll
    for (int q = 0; q < 4; ++q) rk_pair_update<STAGE>(rc, q0, acc, out, q, idx, kra[q], krb[q]);
}

// max |u|, max |p| and the non-finite flag over the owned planes (the
// stats / NaN scan of the RK wrappers, solver_registry.c:31-49,760-768)
static __global__ __launch_bounds__(256) void k_vel_stats(Geo g, const double* __restrict__ U,
                                                          const double* __restrict__ V,
                                                          const double* __restrict__ W,
                                                          const double* __restrict__ P,
                                                          unsigned long long* red) {
    __shared__ double shv[4], shp[4];
    __shared__ int shbad;
    if (threadIdx.x == 0) shbad = 0;
    __syncthreads();
    const int i = blockIdx.x * 64 + (threadIdx.x & 63);
    const int j = blockIdx.y * 4 + (threadIdx.x >> 6);
    const int k = blockIdx.z;
    double mv = 0.0, mp = 0.0;
    if (i < g.nx && j < g.ny) {
        const long long idx = cidx(g, i, j, k);
        const double u = U[idx], v = V[idx], w = W[idx], p = P[idx];
        if (!isfinite(u) || !isfinite(v) || !isfinite(w) || !isfinite(p)) shbad = 1;
        const double vel2 = (u * u) + (v * v) + (w * w);  // sqrt on the host (cell_stats)
        if (vel2 > mv) mv = vel2;
        const double ap = fabs(p);
        if (ap > mp) mp = ap;
    }
    mv = wave_max(mv);
    mp = wave_max(mp);
    if ((threadIdx.x & 63) == 0) {
        shv[threadIdx.x >> 6] = mv;
        shp[threadIdx.x >> 6] = mp;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicMax(&red[0], ord_enc(fmax(fmax(shv[0], shv[1]), fmax(shv[2], shv[3]))));
        atomicMax(&red[1], ord_enc(fmax(fmax(shp[0], shp[1]), fmax(shp[2], shp[3]))));
        if (shbad) atomicOr(&red[2], 1ull);
    }
}

// ---------------------------------------------------------------------------
// Relaxation solvers.
// Red-Black SOR colour pass (linear_solver_redblack.c:97-133). `parity` is the
// (i+j+k) parity updated in this pass: the reference's first ("red") pass
// updates odd cells, the second even cells. Each cell reads only the other
// colour, so the in-place update is race-free and bitwise the reference's.
// Jacobi (linear_solver_jacobi.c:92-109) reads xin, writes xout.
// ---------------------------------------------------------------------------
struct RelaxCoef {
    double dx2, dy2, inv_dz2, inv_factor, omega;
    double rdx2, rdy2;  // RN(1 / dx2), RN(1 / dy2) for divc
};

// a / d, correctly rounded, for the constant divisors dx2 / dy2 of the
// relaxation sweeps, from the correctly rounded reciprocal r = RN(1/d):
// q = RN(a r) is within 1 ulp of a/d, a - q d is exact in one FMA, and the
// corrected q + (a - q d) r rounds to RN(a/d) (Markstein's correction, the
// IA-64 division scheme) -- 3 VALU ops instead of the ~14-op generic fp64
// division, bitwise the reference's `/` (checked on 9.6e8 random quotients,
// tools/divc_check.c, and by the bitwise relaxation tests). Quotients near the
// underflow/overflow range, zeros (sign of zero) and non-finite values take
// the generic division.
__device__ __forceinline__ double divc(double a, double d, double r) {
    const double q = a * r;
    const double aq = fabs(q);
    if (!(aq >= 0x1p-900 && aq <= 0x1p+900)) return a / d;  // residual stays normal
    return fma(fma(-q, d, a), r, q);
}

// Division functors for the stencil helpers. DivC: divc, its range test a
// branch per division. DivFastZ (below, with divz) defers the test: the fast
// quotient's range check goes into a lane flag (compare masks, no branch) and
// the caller recomputes the lanes whose flag dropped with DivExact behind ONE
// wave-uniform branch; where the flag held the value is divz's, so results
// are bitwise either way. That form helps the predictor (fewer, longer basic
// blocks) but spilled in k_rb1 and made it slower (0.845 vs 0.751 ms at
// 512^3, profiles/r02_deferred_div.jsonl), which keeps DivC.
struct DivC {  // divc, its range test branching per division
    __device__ __forceinline__ double operator()(double a, double d, double r) const {
        return divc(a, d, r);
    }
};
struct DivExact {  // the reference's division (the recompute path)
    __device__ __forceinline__ double operator()(double a, double d, double) const { return a / d; }
};
// true when some lane of the wave dropped its flag (wave-uniform)
__device__ __forceinline__ bool wave_any_bad(bool ok) {
    return __builtin_amdgcn_ballot_w64(!ok) != 0;
}

static __global__ __launch_bounds__(NT) void k_rb_pass(Geo g, RelaxCoef rc, double* __restrict__ x,
                                                const double* __restrict__ rhs, int parity) {
    const int ntiles = g.tiles_x * g.tiles_y * g.tiles_z;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        TileCoord c = tile_coord(g, t);
        if (!c.active) continue;
        long long idx = cidx(g, c.i, c.j, c.kb);
        for (int k = c.kb; k < c.ke; ++k, idx += g.ps) {
            if (((c.i + c.j + k + g.kofs) & 1) != parity) continue;  // global parity
            double pn = -(rhs[idx] - (x[idx + 1] + x[idx - 1]) / rc.dx2 -
                          (x[idx + g.px] + x[idx - g.px]) / rc.dy2 -
                          (x[idx + g.sz] + x[idx - g.sz]) * rc.inv_dz2) *
                        rc.inv_factor;
            double xo = x[idx];
            x[idx] = xo + rc.omega * (pn - xo);
        }
    }
}

static __global__ __launch_bounds__(NT) void k_jacobi(Geo g, RelaxCoef rc, const double* __restrict__ xin,
                                               double* __restrict__ xout,
                                               const double* __restrict__ rhs) {
    const int ntiles = g.tiles_x * g.tiles_y * g.tiles_z;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        TileCoord c = tile_coord(g, t);
        if (!c.active) continue;
        long long idx = cidx(g, c.i, c.j, c.kb);
        for (int k = c.kb; k < c.ke; ++k, idx += g.ps) {
            xout[idx] = -(rhs[idx] - (xin[idx + 1] + xin[idx - 1]) / rc.dx2 -
                          (xin[idx + g.px] + xin[idx - g.px]) / rc.dy2 -
                          (xin[idx + g.sz] + xin[idx - g.sz]) * rc.inv_dz2) *
                         rc.inv_factor;
        }
    }
}

// L-infinity residual |lap(x) - rhs| (linear_solver.c:304-346, division form).
struct ResCoef {
    double dx2, dy2, inv_dz2;
};

static __global__ __launch_bounds__(NT) void k_residual_linf(Geo g, ResCoef rc,
                                                      const double* __restrict__ x,
                                                      const double* __restrict__ rhs,
                                                      unsigned long long* out) {
    __shared__ double sh[NWAVE];
    double m = 0.0;
    const int ntiles = g.tiles_x * g.tiles_y * g.tiles_z;
    for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
        TileCoord c = tile_coord(g, t);
        if (!c.active) continue;
        long long idx = cidx(g, c.i, c.j, c.kb);
        for (int k = c.kb; k < c.ke; ++k, idx += g.ps) {
            double lap = (x[idx + 1] - 2.0 * x[idx] + x[idx - 1]) / rc.dx2 +
                         (x[idx + g.px] - 2.0 * x[idx] + x[idx - g.px]) / rc.dy2 +
                         (x[idx + g.sz] + x[idx - g.sz] - 2.0 * x[idx]) * rc.inv_dz2;
            double res = fabs(lap - rhs[idx]);
            if (res > m) m = res;
        }
    }
    m = wave_max(m);
    if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = sh[0];
        for (int w = 1; w < NWAVE; ++w) a = fmax(a, sh[w]);
        atomicMax(out, ord_enc(a));
    }
}

// ---------------------------------------------------------------------------
// Relaxation iterations on the row-pair sweep tiling (single device), with
// the common loop's convergence test (linear_solver.c:397-485) on the device.
// Ping-pong buffers: iteration it reads X = buf[it & 1] (the iterate after
// it - 1 iterations, BCs applied) and leaves buf[(it + 1) & 1].
//   RB-SOR:  k_rx<RX_RED>   X -> Y: first-colour ((i+j+k) odd, the CPU
//                           reference's "red", linear_solver_redblack.c:97-114)
//                           cells SOR-updated, the other cells copied; and the
//                           L-inf residual of X;
//            k_rx_shell     boundary shell X -> Y (the sweeps read it);
//            k_rx<RX_BLACK> Y in place: second-colour cells (:116-133);
//            k_rx_shell     Neumann BC on Y (poisson_solver_apply_bc).
//   Jacobi:  k_rx<RX_JACOBI> X -> Y (linear_solver_jacobi.c:92-109) + the
//            residual of X; k_rx_shell Neumann on Y.
// The residual of the iterate after iteration it - 1 is thus computed by the
// first sweep of iteration it, which has to read X anyway (16 B/cell of the
// reference's separate residual pass saved); when it shows convergence the
// result is X, still intact in its buffer, and everything launched after it
// returns at once (RxState.done). Per-cell arithmetic is the reference's, and
// L-inf (a max) is order-independent, so iterates, residuals and iteration
// counts are bitwise the reference's.
// ---------------------------------------------------------------------------
struct RxState {
    double tol, abs_tol, rel_tol, res0, res;
    int iterations, done, status, max_iter, check_interval, result;  // result: buffer index
    // two iterations per sweep (k_rb2, rb2.hpp): the iterate index the loop
    // stopped on, whether `res` is that iterate's exact residual, the
    // host-resolved exact residual of iterate ovr_it (-1: none), and max |rhs|
    int res_it, res_exact, ovr_it, pad0;
    double ovr_m, bmax;
    double xmax;  // max |X| of a k_rb2 sweep's input when it certifies X (k_rb2_xmax)
};

constexpr int RX_RED = 0;
constexpr int RX_BLACK = 1;
constexpr int RX_JACOBI = 2;

// m = L-inf residual of the iterate after it - 1 iterations (it = 0: x0)
__device__ __forceinline__ void rx_finish(RxState* st, double m, int it) {
    if (it == 0) {  // linear_solver.c:415-437
        st->res0 = m;
        st->res = m;
        double tol = st->rel_tol * m;
        if (tol < st->abs_tol) tol = st->abs_tol;
        st->tol = tol;
        if (m < st->abs_tol) {
            st->done = 1;
            st->status = ST_CONVERGED;
            st->iterations = 0;
            st->result = 0;
            st->res_it = 0;
        }
        return;
    }
    const int prev = it - 1;  // :443-468, iteration prev just completed
    if (prev % st->check_interval == 0) {
        st->res = m;
        if (m < st->tol || m < st->abs_tol) {
            st->done = 1;
            st->status = ST_CONVERGED;
            st->iterations = it;  // iter + 1 at the break
            st->result = it & 1;
            st->res_it = it;
            return;
        }
    }
    if (it >= st->max_iter) {  // loop ran out: iterations = iter + 1 = max_iter + 1 (:472)
        st->done = 1;
        st->status = ST_MAX_ITER;
        st->iterations = st->max_iter + 1;
        st->result = it & 1;
        st->res_it = it;
    }
}

static __global__ void k_rx_init(RxState* st, double rel_tol, double abs_tol, int max_iter,
                                 int check_interval) {
    if (threadIdx.x == 0) {
        st->tol = 0.0;
        st->abs_tol = abs_tol;
        st->rel_tol = rel_tol;
        st->res0 = st->res = 0.0;
        st->iterations = 0;
        st->done = 0;
        st->status = ST_MAX_ITER;
        st->max_iter = max_iter;
        st->check_interval = check_interval;
        st->result = 0;
        st->res_it = 0;
        st->res_exact = 1;
        st->ovr_it = -1;
        st->pad0 = 0;
        st->ovr_m = 0.0;
        st->bmax = 0.0;
    }
}

// Boundary shell of an iteration: mode 0 copies src -> dst, mode 1 applies
// the Neumann gathers to dst.
static __global__ __launch_bounds__(256) void k_rx_shell(Geo g, const RxState* st,
                                                  const double* __restrict__ src,
                                                  double* __restrict__ dst, int mode) {
    if (st->done) return;
    const long long total = shell_total(g);
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {
        int i, j, k;
        bool zlo, zhi;
        shell_cell(g, e, i, j, k, zlo, zhi);
        const long long d = cidx(g, i, j, k);
        if (mode == 0) {
            dst[d] = src[d];
        } else {
            const int sk = (zlo || zhi) ? bc_map(k, g.nz, 0) : k;
            dst[d] = dst[cidx(g, bc_map(i, g.nx, 0), bc_map(j, g.ny, 0), sk)];
        }
    }
}

// Z-slabs (DIST): the residual is an all-ranks max, through the device
// mailbox (mb) or, without one, left encoded in dred[0] for an RCCL max
// all-reduce + k_rx_finish.
template <int TY, int MODE, int FL, bool DIST = false>
static __global__ __launch_bounds__(64 * TY, sweep_min_waves<FL>()) void k_rx(
    SGeo g, RelaxCoef rc, const double* __restrict__ xin, double* __restrict__ xout,
    const double* __restrict__ rhs, RxState* st, double* partials, unsigned* counter, int it,
    Mbox* mb, unsigned long long* dred) {
    constexpr bool PF = (FL & SW_PREFETCH) != 0;
    constexpr bool RES = MODE != RX_BLACK;
    __shared__ double2 rows[2][TY + 2][64];
    __shared__ double sh[TY];
    __shared__ int flag;
    if (st->done) return;
    // stencil field: X (red / Jacobi) or Y in place (black)
    const double* xs = (MODE == RX_BLACK) ? xout : xin;
    RowPair c = row_pair<TY>(g);
    const bool halo = (c.w == 0) || (c.w == TY - 1);
    const int jh = (c.w == 0) ? max(c.j - 1, 0) : min(c.j + 1, g.ny - 1);
    const int hslot = (c.w == 0) ? 0 : TY + 1;
    const long long hoff = (long long)(jh - min(c.j, g.ny - 1)) * g.px;
    const bool xok = c.i0 < g.nx;
    const bool eok = (c.lane == 0 && c.i0 >= 1 && xok) || (c.lane == 63 && c.i0 + 2 < g.nx);
    const long long eoff = (c.lane == 0) ? -1 : 2;
    // parity (i+j+k) of the pair's first cell at local plane k is
    // (j + k + kofs) & 1 (i0 even); the first colour pass updates odd cells
    const int upd = (MODE == RX_RED) ? 1 : 0;
    const double2 zero = make_double2(0.0, 0.0);
    struct Bundle {
        double2 pp, hp, rr;  // X centre / y-halo of plane k+1; rhs of plane k
        double el;           // x-edge cell of plane k
    };
    auto issue = [&](int k, long long ix) __attribute__((always_inline)) {
        const double2 zero = make_double2(0.0, 0.0);
        Bundle b;
        const long long ip = ix + g.sz;
        b.pp = xok ? ld2(xs, ip) : zero;
        b.hp = (xok && halo && k + 1 < c.ke) ? ld2(xs, ip + hoff) : zero;
        b.rr = xok ? ld2v<FL>(rhs, ix) : zero;
        b.el = eok ? xs[ix + eoff] : 0.0;
        return b;
    };
    double m = 0.0;
    long long idx = c.idx;
    double2 pm = xok ? ld2(xs, idx - g.sz) : zero;
    double2 pc = xok ? ld2(xs, idx) : zero;
    double2 hc = (xok && halo) ? ld2(xs, idx + hoff) : zero;
    Bundle cur;
    if (PF) cur = issue(c.kb, idx);
    int buf = 0;
    for (int k = c.kb; k < c.ke; ++k, idx += g.ps) {
        Bundle nxt;
        if (PF) {
            if (k + 1 < c.ke) nxt = issue(k + 1, idx + g.ps);
        } else {
            cur = issue(k, idx);
        }
        rows[buf][c.w + 1][c.lane] = pc;
        if (halo) rows[buf][hslot][c.lane] = hc;
        __syncthreads();
        const double2 ys = rows[buf][c.w][c.lane];
        const double2 yn = rows[buf][c.w + 2][c.lane];
        const double2 pp = cur.pp;
        double left = __shfl_up(pc.y, 1, 64);
        double right = __shfl_down(pc.x, 1, 64);
        if (c.lane == 0) left = cur.el;
        if (c.lane == 63) right = cur.el;
        // cell 0: (xm, xp) = (left, pc.y); cell 1: (pc.x, right)
        if (RES) {  // linear_solver.c:304-346 (k_residual_linf's expression)
            const double l0 = divc(pc.y - 2.0 * pc.x + left, rc.dx2, rc.rdx2) +
                              divc(yn.x - 2.0 * pc.x + ys.x, rc.dy2, rc.rdy2) +
                              (pp.x + pm.x - 2.0 * pc.x) * rc.inv_dz2;
            const double l1 = divc(right - 2.0 * pc.y + pc.x, rc.dx2, rc.rdx2) +
                              divc(yn.y - 2.0 * pc.y + ys.y, rc.dy2, rc.rdy2) +
                              (pp.y + pm.y - 2.0 * pc.y) * rc.inv_dz2;
            const double r0 = fabs(l0 - cur.rr.x), r1 = fabs(l1 - cur.rr.y);
            if (c.in0 && r0 > m) m = r0;
            if (c.in1 && r1 > m) m = r1;
        }
        double2 out = pc;
        if (MODE == RX_JACOBI) {
            const double pn0 = -(cur.rr.x - divc(pc.y + left, rc.dx2, rc.rdx2) -
                                 divc(yn.x + ys.x, rc.dy2, rc.rdy2) -
                                 (pp.x + pm.x) * rc.inv_dz2) *
                               rc.inv_factor;
            const double pn1 = -(cur.rr.y - divc(right + pc.x, rc.dx2, rc.rdx2) -
                                 divc(yn.y + ys.y, rc.dy2, rc.rdy2) -
                                 (pp.y + pm.y) * rc.inv_dz2) *
                               rc.inv_factor;
            if (c.in0) out.x = pn0;
            if (c.in1) out.y = pn1;
        } else {
            // one cell of the pair has this pass's colour: gather its stencil
            // (wave-uniform choice: the parity depends on j and k only)
            const bool first = ((c.j + k + g.kofs) & 1) == upd;  // global parity
            const double xc = first ? pc.x : pc.y;
            const double xl = first ? left : pc.x, xr = first ? pc.y : right;
            const double yl = first ? ys.x : ys.y, yr = first ? yn.x : yn.y;
            const double zl = first ? pm.x : pm.y, zr = first ? pp.x : pp.y;
            const double rh = first ? cur.rr.x : cur.rr.y;
            const double pn = -(rh - divc(xr + xl, rc.dx2, rc.rdx2) -
                                divc(yr + yl, rc.dy2, rc.rdy2) - (zr + zl) * rc.inv_dz2) *
                              rc.inv_factor;
            const double xn = xc + rc.omega * (pn - xc);
            if (first) {
                if (c.in0) out.x = xn;
            } else if (c.in1) {
                out.y = xn;
            }
        }
        if (c.act) st2v<FL>(xout, idx, out);
        pm = pc;
        pc = pp;
        hc = cur.hp;
        if (PF) cur = nxt;
        buf ^= 1;
    }
    if (!RES) return;
    m = wave_max(m);
    if (c.lane == 0) sh[c.w] = m;
    __syncthreads();
    double* shs = (double*)&rows[0][0][0];
    if (threadIdx.x == 0) {
        double a = 0.0;
        for (int q = 0; q < TY; ++q) a = fmax(a, sh[q]);
        store_sc1(&partials[blockIdx.x], a);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned t = __hip_atomic_fetch_add((gu32*)counter, 1u, __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_AGENT);
        flag = (t == gridDim.x - 1) ? 1 : 0;
    }
    __syncthreads();
    if (flag == 0) return;
    double a = 0.0;
    for (unsigned b = threadIdx.x; b < gridDim.x; b += 64 * TY) a = fmax(a, load_sc1(&partials[b]));
    a = wave_max(a);
    if (c.lane == 0) shs[c.w] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        double tot = 0.0;
        for (int q = 0; q < TY; ++q) tot = fmax(tot, shs[q]);
        __hip_atomic_store((gu32*)counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!DIST) {
            rx_finish(st, tot, it);
        } else if (mb) {
            double gm;
            if (mbox_allreduce(mb, tot, &gm, true)) {
                rx_finish(st, gm, it);
            } else {
                st->done = 1;
                st->status = ST_COMM_TIMEOUT;
            }
        } else {
            dred[0] = ord_enc(tot);
        }
    }
}

__device__ __forceinline__ double ord_dec_dev(unsigned long long e) {
    const unsigned long long b =
        (e & 0x8000000000000000ull) ? (e & 0x7FFFFFFFFFFFFFFFull) : ~e;
    return __longlong_as_double((long long)b);
}

// after the RCCL max all-reduce of dred (Z-slabs without a device mailbox)
static __global__ void k_rx_finish(RxState* st, const unsigned long long* gred, int it) {
    if (threadIdx.x == 0 && !st->done) rx_finish(st, ord_dec_dev(gred[0]), it);
}

// ---------------------------------------------------------------------------
// Single-pass Red-Black SOR iteration (3-D, single device): X -> Y in one
// z-march. For plane q the tile forms R_q = X_q with its first-colour ("red",
// (i+j+k) odd) interior cells SOR-updated (linear_solver_redblack.c:97-114);
// then the second colour of plane q-1 is updated from R (:116-133), and the
// L-inf residual of X at plane q (linear_solver.c:304-346) rides along. R at
// a tile's y/x halo is recomputed locally (overlapped tiles: 128 x 16 cells
// loaded per plane, 124 x 12 written), so each cell of X and rhs is read
// once from HBM and Y written once: 24 B/cell per iteration instead of the
// two colour passes' 48. R values are computed from the same X values by the
// same expression as the first pass would, so Y is bitwise the two-pass
// result.
// ---------------------------------------------------------------------------

// One SOR update of a cell (linear_solver_redblack.c:103-112 operation order).
template <class Dv>
__device__ __forceinline__ double sor1(const RelaxCoef& rc, Dv dv, double vc, double vl, double vr,
                                       double vs, double vn, double vm, double vp, double vb) {
    const double pn = -(vb - dv(vr + vl, rc.dx2, rc.rdx2) - dv(vn + vs, rc.dy2, rc.rdy2) -
                        (vp + vm) * rc.inv_dz2) *
                      rc.inv_factor;
    return vc + rc.omega * (pn - vc);
}

// |lap(x) - rhs| of one cell (linear_solver.c:304-346, the division form).
template <class Dv>
__device__ __forceinline__ double res1(const RelaxCoef& rc, Dv dv, double c, double xl, double xr,
                                       double ys, double yn, double zm, double zp, double b) {
    const double l = dv(xr - 2.0 * c + xl, rc.dx2, rc.rdx2) +
                     dv(yn - 2.0 * c + ys, rc.dy2, rc.rdy2) + (zp + zm - 2.0 * c) * rc.inv_dz2;
    return fabs(l - b);
}

template <bool V>
using BoolC = std::integral_constant<bool, V>;
template <int V>
using IntC = std::integral_constant<int, V>;

// Tile shapes (r02b). A workgroup is 16 waves; lane l of wave w owns the x
// pair c = l % TC of tile row r = w + 16 (l / TC), so a tile is TC pairs (2 TC
// columns) by TR = 1024 / TC rows. Rows w and w + 16 h have the same parity,
// so the colour pattern of a step stays wave-uniform for every TC. R is
// recomputed on the tile's one-cell halo: 2 TC - 4 columns and TR - 4 rows are
// written per tile. TC = 64 (16 rows) loads 1.38x the cells it writes, TC = 32
// (32 rows) 1.22x, and the narrower tiles also waste less on the last x tile
// (512: 5 x 124 columns for 510 vs 9 x 60).
template <int TC>
constexpr int rb1_rows() { return 1024 / TC; }
template <int TC>
constexpr int rb1_ox() { return 2 * TC - 4; }  // output columns per tile
template <int TC>
constexpr int rb1_oy() { return 1024 / TC - 4; }  // output rows per tile

// Issue-model details (r02; profiles/r02_rb_variants.jsonl, r02_pmc_rb.jsonl):
//  - the colour pattern of a step is wave-uniform ((j + q) parity): the z
//    loop is unrolled by two planes and each step is compiled for its
//    pattern, so no per-lane selects pick the updated cell of a pair
//    (VALU instructions per launch 321 M -> 196 M at 512^3);
//  - x neighbours come from the row the wave already published in LDS (one
//    ds_read_b64 each side) instead of two ds_bpermute per double, and every
//    LDS operand of a step is read right after its barrier (one LDS round
//    trip per step);
//  - rhs is not loaded on the two halo rows, which never use it.
// PF = the register-ring prefetch below (r02: 0.90 -> 0.76 ms per iteration at
// 512^3 on one box, 128 VGPRs); the product instantiates PF = true.
// DIST (Z-slabs): R on a halo plane that has a neighbour (rh_lo: plane k0 - 1,
// rh_hi: plane k1) is the neighbour's R of its edge plane, exchanged into RH
// beforehand (k_rb_edge_r + halo); it cannot be formed here, since that needs
// X two planes beyond the halo. The L-inf residual leaves as in k_rx: the
// device mailbox's max, or dred for an RCCL max all-reduce + k_rx_finish.
// LDS of one k_rb1 workgroup: X and R rows of two plane parities (the same
// 64 KB for every tile width), the waves' residual maxima and the
// last-workgroup flag.
struct Rb1Lds {
    double xb[2 * 1024 * 2];
    double rb[2 * 1024 * 2];
    double sh[16];
    int flag;
};

// The body of k_rb1 for the tile width TC; bid = this workgroup's tile-block
// index within its geometry g (k_rb1m runs two geometries in one grid).
template <int FL, int TC, bool PF, bool DIST, bool REV = false>
__device__ __forceinline__ void rb1_body(
    Rb1Lds& L, int bid, SGeo g, RelaxCoef rc, const double* __restrict__ X,
    double* __restrict__ Y, const double* __restrict__ rhs, RxState* st, double* partials,
    unsigned* counter, int it, const double* __restrict__ RH, int rh_lo, int rh_hi, Mbox* mb,
    unsigned long long* dred, int neu) {
    constexpr int NW = 16;  // waves
    constexpr int TR = rb1_rows<TC>();
    constexpr int OX = rb1_ox<TC>(), OY = rb1_oy<TC>();
    // X and R rows by plane parity; a row is stored as its TC .x cells, then
    // its TC .y cells, so a pair is one ds_read2/ds_write2_b64 and an x
    // neighbour (one double of the adjacent lane) a conflict-free ds_read_b64
    // (with double2 rows those 8-B reads at a 16-B lane stride conflicted)
    auto& xb = *reinterpret_cast<double(*)[2][TR][2][TC]>(L.xb);
    auto& rb = *reinterpret_cast<double(*)[2][TR][2][TC]>(L.rb);
    auto& sh = L.sh;
    auto& flag = L.flag;
    // every LDS read stays a ds_read_b64 (2 LDS cycles per wave; a pair
    // merged into ds_read2_b64 takes 8): a scheduling barrier that lets every
    // instruction class cross it ends the pairing pass's search window
    auto lrd = [&](const double& v) __attribute__((always_inline)) {
        __builtin_amdgcn_sched_barrier(0x7ff);
        return v;
    };
    auto lget = [&](double (&a)[2][TR][2][TC], int p, int r, int l) __attribute__((always_inline)) {
        const double x = lrd(a[p][r][0][l]);
        return make_double2(x, lrd(a[p][r][1][l]));
    };
    auto lput = [&](double (&a)[2][TR][2][TC], int p, int r, int l, double2 v)
                    __attribute__((always_inline)) {
        a[p][r][0][l] = v.x;
        a[p][r][1][l] = v.y;
    };
    if (st->done) return;
    // tile = block index: round-robin dispatch spreads consecutive tiles over
    // the eight XCDs (r03: faster here than xcd_tile's contiguous ranges,
    // 2.86-2.87 -> 2.82-2.83 ms per iteration at 1024^2 x 512, equal at 512^3,
    // profiles/r03_tile_order.jsonl)
    const int t = bid;
    const int tx = t % g.tiles_x;
    const int rest = t / g.tiles_x;
    const int ty = rest % g.tiles_y;
    const int tz = rest / g.tiles_y;
    const int lane = threadIdx.x & 63;
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int c = lane % TC;                     // pair within the row
    const int r = w + NW * (lane / TC);          // tile row
    const int cm = max(c - 1, 0), cp = min(c + 1, TC - 1);  // x neighbours' pairs
    const int rlo = max(r - 1, 0), rhi = min(r + 1, TR - 1);  // y neighbours' rows
    const int i0 = g.xofs + tx * OX - 2 + 2 * c;  // even; the pair is (i0, i0 + 1)
    const int j = ty * OY - 2 + r;       // grid row
    // kmode 1: the slab's two edge planes (tz 0 -> k0, tz 1 -> k1 - 1);
    // kmode 2: the planes [kt0, kt1); else [k0, k1). A march over a plane
    // range still forms R on its two lower neighbour planes (prologue), so
    // the ranges of one iteration's launches give the one-launch Y.
    int kb, ke;
    if (g.kmode == 1) {
        kb = (tz == 0) ? g.k0 : g.k1 - 1;
        ke = kb + 1;
    } else {
        const int kt0 = (g.kmode == 2) ? g.kt0 : g.k0;
        const int kt1 = (g.kmode == 2) ? g.kt1 : g.k1;
        kb = kt0 + tz * g.kc;
        ke = min(kb + g.kc, kt1);
    }
    const bool xin = (i0 >= 0 && i0 < g.nx);
    const bool ld = xin && j >= 0 && j < g.ny;
    const bool jin = (j >= 1 && j <= g.ny - 2);
    const bool in0 = jin && i0 >= 1 && i0 <= g.nx - 2;
    const bool in1 = jin && i0 + 1 <= g.nx - 2;
    const bool orow = (r >= 2 && r < 2 + OY);
    const bool own = orow && c >= 1 && c <= TC - 2;
    // wave-uniform skips: with TC = 64 a wave is one row, so its halo rows
    // (no R work: rows 0, 15; no output: rows 0, 1, 14, 15) skip whole
    // phases; narrower tiles mix rows in a wave and mask per lane instead
    const bool wr = (TC == 64) ? (r >= 1 && r <= TR - 2) : true;
    const bool wo = (TC == 64) ? orow : true;
    const long long col = (long long)max(min(j, g.ny - 1), 0) * g.px + max(i0, 0);
    // the folded Neumann shell (neu): this lane's x-face roles and whether it
    // stores (pairs (nx-1, pad) of odd nx leave cell nx-1 to role 4)
    const int nrole = (i0 == 0 ? 1 : 0) | (i0 + 1 == g.nx - 1 ? 2 : 0) |
                      (i0 + 1 == g.nx - 2 ? 4 : 0) |
                      ((own && jin && i0 <= g.nx - 2) ? 8 : 0);
    // Loads are issued unconditionally from clamped (always valid) addresses
    // and never masked: with the same loads on every control path and no
    // select right behind them, the compiler's vmcnt counting waits for a
    // plane only where a step consumes it (a load some path skips, or a
    // select on the loaded value, forces vmcnt(0) right after the prefetch of
    // the next plane, i.e. a full memory latency per step). Positions outside
    // the grid (ld false, k out of range) then hold other cells' values; they
    // only ever feed boundary cells, which are not updated, and halo lanes,
    // which are not stored or reduced. The halo rows 0 and TR - 1 (no R work)
    // load the adjacent row's rhs, which that row's lanes load too (an L2 hit).
    const int ic = (i0 < g.nx) ? max(i0, 0) : g.nx - 2 - ((g.nx - 2) & 1);
    const int jr = j + (r == 0 ? 1 : (r == TR - 1 ? -1 : 0));
    const long long colx = (long long)max(min(j, g.ny - 1), 0) * g.px + ic;
    const long long colr = (long long)max(min(jr, g.ny - 1), 0) * g.px + ic;
    auto ldx = [&](int k) -> double2 {
        return ld2(X, (long long)min(max(k, 0), g.nz - 1) * g.ps + colx);
    };
    auto ldr = [&](int k) -> double2 {
        return ld2v<FL>(rhs, (long long)min(max(k, 0), g.nz - 1) * g.ps + colr);
    };
    const double2 zero = make_double2(0.0, 0.0);
    // Step q forms R_{q+1} and updates the second colour of plane q.
    // Per lane: X_q, X_{q+1}, X_{q+2} (xm, xc, xp); R_{q-1}, R_q (rmm, rm);
    // rhs_{q+1} (bq). Of rhs_q and R_{q-1} only the component of the cell
    // this step's second-colour update touches is kept (bmh, rmmh): the
    // pattern alternates per plane, so the end of step q keeps the component
    // step q + 1 will use. LDS at the top of step q: X_{q+1} rows in
    // xb[(q+1)&1], R_q rows in rb[q&1].
    // PF (register ring): the X planes sit in a ring of four register slots
    // and rhs in a ring of two, indexed by the step's phase P = (q - q0) mod 4
    // at compile time (the z loop is unrolled by four), and step q issues the
    // loads of X_{q+3} and rhs_{q+2} into the free slots before its barrier:
    // a full step of latency hiding, and no register copy of a loaded value
    // (a copy would wait for the load). Without PF the loads are issued at
    // the end of step q and the three X planes shift through xm, xc, xp.
    // REV (r03, one device): the march runs z downwards, D = -1: step q forms
    // R_{q-1} and updates plane q, "ahead" is q - 1. Every cell's operands
    // keep their z roles (z- / z+ are picked by direction), R depends on X
    // only and the second colour on R only, and the residual is a max, so Y
    // and the iteration's decision are bitwise the upward march's. The host
    // alternates the direction per iteration, so each sweep starts on the
    // planes the previous one wrote last (in the Infinity Cache).
    constexpr int D = REV ? -1 : 1;
    const int q0 = REV ? ke + 1 : kb - 2;  // the first step
    double2 xr[4], br[2], rm;
    double bmh, rmmh;
    xr[0] = ldx(q0);
    xr[1] = ldx(q0 + D);
    xr[2] = ldx(q0 + 2 * D);
    xr[3] = zero;
    br[0] = ldr(q0 + D);
    br[1] = zero;
    rm = zero;
    bmh = rmmh = 0.0;
    lput(xb, (q0 + D) & 1, r, c, xr[1]);
    double m = 0.0;
    // E: cell i0 of the pair is the cell both updates of this step touch (the
    // first colour, (i+j+k) odd, of plane q+1 and the second of plane q)
    auto step = [&](auto Ec, auto Pc, int q) __attribute__((always_inline)) {
        constexpr bool E = decltype(Ec)::value;
        constexpr int P = PF ? decltype(Pc)::value : 0;  // ring phase
        constexpr int IM = P & 3, IC = (P + 1) & 3, IP = (P + 2) & 3, IN = (P + 3) & 3;
        constexpr int BQ = P & 1, BN = (P + 1) & 1;
        if constexpr (PF) {
            xr[IN] = ldx(q + 3 * D);
            br[BN] = ldr(q + 2 * D);
        }
        // behind / centre / ahead of plane qa, then its z- / z+ neighbours
        const double2 xbh = xr[IM], xc = xr[IC], xah = xr[IP], bq = br[BQ];
        const double2 xm = REV ? xah : xbh, xp = REV ? xbh : xah;
        __syncthreads();
        const int qa = q + D;
        const bool qin = (qa >= g.k0 && qa < g.k1);
        const bool rin = qin && qa >= kb && qa < ke;
        // the output's LDS operands (R_q rows) are read up front, so one LDS
        // round trip after the barrier serves both halves of the step
        const double2 rys = lget(rb, q & 1, rlo, c);
        const double2 ryn = lget(rb, q & 1, rhi, c);
        const double rlr = lrd(E ? rb[q & 1][r][1][cm] : rb[q & 1][r][0][cp]);
        double2 R = xc;
        if constexpr (DIST) {
            if ((qa == g.k0 - 1 && rh_lo) || (qa == g.k1 && rh_hi))
                R = ld2(RH, (long long)qa * g.ps + colx);
        }
        const double2 ys = lget(xb, qa & 1, rlo, c);
        const double2 yn = lget(xb, qa & 1, rhi, c);
        const double left = lrd(xb[qa & 1][r][1][cm]);
        const double right = lrd(xb[qa & 1][r][0][cp]);
        if (wr && qin) {
            if (E) {
                const double v = sor1(rc, DivC{}, xc.x, left, xc.y, ys.x, yn.x, xm.x, xp.x, bq.x);
                if (in0) R.x = v;
            } else {
                const double v = sor1(rc, DivC{}, xc.y, xc.x, right, ys.y, yn.y, xm.y, xp.y, bq.y);
                if (in1) R.y = v;
            }
            if (wo && rin) {
                const double a0 = res1(rc, DivC{}, xc.x, left, xc.y, ys.x, yn.x, xm.x, xp.x, bq.x);
                const double a1 = res1(rc, DivC{}, xc.y, xc.x, right, ys.y, yn.y, xm.y, xp.y, bq.y);
                if (own && in0 && a0 > m) m = a0;
                if (own && in1 && a1 > m) m = a1;
            }
        }
        // ---- second colour of plane q from R_{q-1}, R_q, R_{q+1} ----
        // (rmmh: R behind, R: R ahead; REV swaps their z roles)
        if ((REV ? q < ke : q >= kb) && wo) {
            double2 out = rm;
            if (E) {
                const double rzm = REV ? R.x : rmmh, rzp = REV ? rmmh : R.x;
                const double v = sor1(rc, DivC{}, rm.x, rlr, rm.y, rys.x, ryn.x, rzm, rzp, bmh);
                if (own && in0) out.x = v;
            } else {
                const double rzm = REV ? R.y : rmmh, rzp = REV ? rmmh : R.y;
                const double v = sor1(rc, DivC{}, rm.y, rm.x, rlr, rys.y, ryn.y, rzm, rzp, bmh);
                if (own && in1) out.y = v;
            }
            if (neu) {
                // the iteration's Neumann BC (linear_solver_redblack.c:139) folded
                // into the stores: every boundary cell of Y is the gather
                // k_bc_shell / k_rx_shell mode 1 makes, Y at the clamped-inward
                // position (bc_map), so the writer of that source cell stores
                // it to its mirror positions too: x faces within the pair (or
                // one 8-B store when nx is odd), y faces as a copy of rows 1 /
                // ny-2, z faces (global, not a slab's halo) as copies of
                // planes k0 / k1-1
                // nrole (lane constant): 1 = pair (0, 1), 2 = pair (nx-2, nx-1),
                // 4 = nx odd and .y is cell nx-2 (cell nx-1 <- .y), 8 = store
                if (nrole & 1) out.x = out.y;
                if (nrole & 2) out.y = out.x;
                if (nrole & 8) {
                    // j is wave-uniform with TC = 64 (one row per wave), so
                    // are q and the z-face tests: scalar branches
                    auto put = [&](long long base) __attribute__((always_inline)) {
                        st2v<FL>(Y, base, out);
                        if (nrole & 4) Y[base + 2] = out.y;
                        if (j == 1 || j == g.ny - 2) {
                            const long long b2 = base + (j == 1 ? -g.px : g.px);
                            st2v<FL>(Y, b2, out);
                            if (nrole & 4) Y[b2 + 2] = out.y;
                        }
                    };
                    const long long base = (long long)q * g.ps + col;
                    put(base);
                    if (q == g.k0 && !rh_lo) put(base - g.ps);
                    if (q == g.k1 - 1 && !rh_hi) put(base + g.ps);
                }
            } else if (own && ld && jin) {
                st2v<FL>(Y, (long long)q * g.ps + col, out);
            }
        }
        // step q + D updates the .x cell iff this step did not
        rmmh = E ? rm.y : rm.x;
        rm = R;
        bmh = E ? bq.y : bq.x;
        if constexpr (!PF) {
            xr[0] = xc;
            xr[1] = xah;
            xr[2] = ldx(q + 3 * D);
            br[0] = ldr(q + 2 * D);
        }
        // publish X_{q+2} and R_{q+1} for step q + 1 (their buffers were last
        // read in step q - 1, before this step's barrier)
        lput(xb, (q + 2 * D) & 1, r, c, xah);
        lput(rb, (q + D) & 1, r, c, rm);
    };
    // E(q) for the lane's row: ((j + q + kofs) & 1) == 0; E(kb - 2) == E(kb);
    // rows r and r + 16 h share the parity, so E is wave-uniform
    const bool E0 = __builtin_amdgcn_readfirstlane(((j + q0 + g.kofs) & 1) == 0 ? 1 : 0) != 0;
    // steps q0, q0 + D, ...: ke - kb + 2 of them (R is formed one plane ahead)
    const int nsteps = ke - kb + 2;
    int n = 0;
    auto march = [&](auto E0c) __attribute__((always_inline)) {
        constexpr bool A = decltype(E0c)::value;
        using TA = BoolC<A>;
        using TB = BoolC<!A>;
        if constexpr (PF) {
            for (; n + 3 < nsteps; n += 4) {
                step(TA{}, IntC<0>{}, q0 + D * n);
                step(TB{}, IntC<1>{}, q0 + D * (n + 1));
                step(TA{}, IntC<2>{}, q0 + D * (n + 2));
                step(TB{}, IntC<3>{}, q0 + D * (n + 3));
            }
            if (n < nsteps) step(TA{}, IntC<0>{}, q0 + D * n);
            if (n + 1 < nsteps) step(TB{}, IntC<1>{}, q0 + D * (n + 1));
            if (n + 2 < nsteps) step(TA{}, IntC<2>{}, q0 + D * (n + 2));
        } else {
            for (; n + 1 < nsteps; n += 2) {
                step(TA{}, IntC<0>{}, q0 + D * n);
                step(TB{}, IntC<0>{}, q0 + D * (n + 1));
            }
            if (n < nsteps) step(TA{}, IntC<0>{}, q0 + D * n);
        }
    };
    if (E0) march(BoolC<true>{});
    else march(BoolC<false>{});
    m = wave_max(m);
    if (lane == 0) sh[w] = m;
    __syncthreads();
    double* shs = &xb[0][0][0][0];
    // an iteration split over several launches (slabs: kmode 1 / 2) shares
    // one partials array: this launch owns [part_ofs, part_ofs + gridDim.x)
    // of part_total, and the last of all part_total workgroups (the last
    // launch on the stream) finishes the max
    const unsigned ptot = g.part_total ? (unsigned)g.part_total : gridDim.x;
    if (threadIdx.x == 0) {
        double a = 0.0;
        for (int v = 0; v < NW; ++v) a = fmax(a, sh[v]);
        store_sc1(&partials[g.part_ofs + blockIdx.x], a);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        unsigned tk = __hip_atomic_fetch_add((gu32*)counter, 1u, __ATOMIC_RELAXED,
                                             __HIP_MEMORY_SCOPE_AGENT);
        flag = (tk == ptot - 1) ? 1 : 0;
    }
    __syncthreads();
    if (flag == 0) return;
    double a = 0.0;
    for (unsigned b = threadIdx.x; b < ptot; b += 1024) a = fmax(a, load_sc1(&partials[b]));
    a = wave_max(a);
    if (lane == 0) shs[w] = a;
    __syncthreads();
    if (threadIdx.x == 0) {
        double tot = 0.0;
        for (int v = 0; v < NW; ++v) tot = fmax(tot, shs[v]);
        __hip_atomic_store((gu32*)counter, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!DIST) {
            rx_finish(st, tot, it);
        } else if (mb) {
            double gm;
            if (mbox_allreduce(mb, tot, &gm, true)) {
                rx_finish(st, gm, it);
            } else {
                st->done = 1;
                st->status = ST_COMM_TIMEOUT;
            }
        } else {
            dred[0] = ord_enc(tot);
        }
    }
}

template <int FL, int TC, bool PF, bool DIST = false, bool REV = false>
static __global__ __launch_bounds__(1024, 4) void k_rb1(
    SGeo g, RelaxCoef rc, const double* __restrict__ X, double* __restrict__ Y,
    const double* __restrict__ rhs, RxState* st, double* partials, unsigned* counter, int it,
    const double* __restrict__ RH, int rh_lo, int rh_hi, Mbox* mb, unsigned long long* dred,
    int neu) {
    __shared__ Rb1Lds L;
    rb1_body<FL, TC, PF, DIST, REV>(L, blockIdx.x, g, rc, X, Y, rhs, st, partials, counter, it, RH,
                               rh_lo, rh_hi, mb, dred, neu);
}

// One device, one launch: the full-width (TC 64) tiles of g64 in blocks
// [0, nb64) and the narrow strip of the columns past them (g2, tile width
// TC2) in the rest. A row's last TC-64 tile would be partial unless 124
// divides it, and costs a full tile's steps for its few columns (512^3: 14
// of 124); the strip's TC-16 / TC-32 tiles are 60 / 28 rows tall, so the
// column strip needs 4.8x / 2.2x fewer workgroups. Both geometries share the
// grid-wide residual reduction (part_total 0: gridDim.x workgroups).
template <int FL, int TC2, bool REV = false>
static __global__ __launch_bounds__(1024, 4) void k_rb1m(
    SGeo g64, SGeo g2, int nb64, RelaxCoef rc, const double* __restrict__ X,
    double* __restrict__ Y, const double* __restrict__ rhs, RxState* st, double* partials,
    unsigned* counter, int it, int neu) {
    __shared__ Rb1Lds L;
    if ((int)blockIdx.x < nb64)
        rb1_body<FL, 64, true, false, REV>(L, blockIdx.x, g64, rc, X, Y, rhs, st, partials,
                                           counter, it, nullptr, 0, 0, nullptr, nullptr, neu);
    else
        rb1_body<FL, TC2, true, false, REV>(L, blockIdx.x - nb64, g2, rc, X, Y, rhs, st,
                                            partials, counter, it, nullptr, 0, 0, nullptr,
                                            nullptr, neu);
}

// R (the first colour SOR-updated, linear_solver_redblack.c:97-114) of a
// slab's two edge planes k0 and k1 - 1 into RH, for the neighbours' k_rb1
// (DIST); same operands and order as k_rb1's R, so bitwise equal to it.
static __global__ __launch_bounds__(256) void k_rb_edge_r(SGeo g, RelaxCoef rc,
                                                         const double* __restrict__ X,
                                                         const double* __restrict__ rhs,
                                                         double* __restrict__ RH) {
    const long long plane = (long long)g.nx * g.ny;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < 2 * plane;
         e += (long long)gridDim.x * blockDim.x) {
        const int k = (e < plane) ? g.k0 : g.k1 - 1;
        const long long q = e % plane;
        const int j = (int)(q / g.nx), i = (int)(q % g.nx);
        if (i < 1 || i > g.nx - 2 || j < 1 || j > g.ny - 2) continue;
        const long long c = (long long)k * g.ps + (long long)j * g.px + i;
        double v = X[c];
        if (((i + j + k + g.kofs) & 1) == 1)
            v = sor1(rc, DivC{}, X[c], X[c - 1], X[c + 1], X[c - g.px], X[c + g.px], X[c - g.ps],
                     X[c + g.ps], rhs[c]);
        RH[c] = v;
    }
}


// ===========================================================================
// Predictor (solver_projection.c:116-185, with compute_source_terms
// solver_explicit_euler.c:317-333 at iter = 0 as per-row / per-column tables
// and energy_compute_buoyancy energy_solver.c:185-196) and corrector
// (solver_projection.c:230-250 + the boundary restore :277-278, the NaN scan
// :281-289 and the stats of solver_registry.c:31-49), on a row-pair z-march.
//
// Tile = 128 (x) x 4 rows (one per wave) x kc planes, 256 threads. Each lane
// owns an x pair and moves it with 16-B loads/stores; x neighbours come from
// the adjacent lanes (the tile's two outer cells from one per-lane load by
// lanes 0 and 63), z neighbours from registers (each field read once per
// plane from HBM), y neighbours from the rows the neighbouring waves load in
// the same step (L1/L2 hits). No LDS and no barrier: the waves of a CU run
// independently, so memory latency hides behind the other resident waves.
// Divisions by the constant spacings use divz (correctly rounded, bitwise
// the reference's `/`), the reference's operation order is kept, and the
// file is compiled with -ffp-contract=off, so u*, v*, w*, u, v, w are
// bitwise the per-cell kernels'. Boundary cells of the tile's rows (i = 0,
// nx - 1) are copies; the rest of the boundary shell (rows j = 0, ny - 1, the
// z faces) is done by k_shell_copy / k_shell_stats.
// ===========================================================================
#ifndef CFD_PR_SYNC
#define CFD_PR_SYNC 1
#endif
#ifndef CFD_PR_TY
#define CFD_PR_TY 4
#endif
constexpr int PR_TY = CFD_PR_TY;  // rows (waves) per workgroup

// a / d correctly rounded, like divc, for operands that are often exactly
// zero (derivatives of a field at rest): e = q d - a and q - e r give the
// signed zero of a / d for a = +-0, so zeros stay on the fast path.
__device__ __forceinline__ double divz(double a, double d, double r) {
    const double q = a * r;
    const double aq = fabs(q);
    if (!(aq <= 0x1p+900 && (aq >= 0x1p-900 || aq == 0.0))) return a / d;
    return fma(-fma(q, d, -a), r, q);
}
// divz with the range test deferred into a lane flag (see DivC)
struct DivFastZ {
    bool& ok;
    __device__ __forceinline__ double operator()(double a, double d, double r) const {
        const double q = a * r;
        const double aq = fabs(q);
        ok &= (aq <= 0x1p+900) & ((aq >= 0x1p-900) | (aq == 0.0));
        return fma(-fma(q, d, -a), r, q);
    }
};

struct ZTile {
    int i0, j, kb, ke, lane;
    bool xok, in0, in1;
    long long col;   // j * px + x offset of the pair (clamped in-row when i0 >= nx)
    long long eoff;  // lanes 0 / 63: offset of the tile's outer x neighbour
    bool eok;
};

__device__ __forceinline__ ZTile ztile(const SGeo& g) {
    ZTile z;
    const int nt = g.tiles_x * g.tiles_y * g.tiles_z;
    const int t = xcd_tile(blockIdx.x, nt);
    const int tx = t % g.tiles_x;
    const int rest = t / g.tiles_x;
    const int ty = rest % g.tiles_y;
    const int tz = rest / g.tiles_y;
    z.lane = threadIdx.x & 63;
    z.i0 = tx * 128 + 2 * z.lane;
    z.j = ty * PR_TY + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    z.kb = g.k0 + tz * g.kc;
    z.ke = min(z.kb + g.kc, g.k1);
    z.xok = z.i0 < g.nx;
    z.in0 = z.xok && z.i0 >= 1 && z.i0 <= g.nx - 2;
    z.in1 = z.xok && z.i0 + 1 <= g.nx - 2;
    const int ic = z.xok ? z.i0 : g.nx - 2 - ((g.nx - 2) & 1);  // even, 16-B aligned
    z.col = (long long)z.j * g.px + ic;
    z.eok = (z.lane == 0 && z.i0 >= 1 && z.xok) || (z.lane == 63 && z.i0 + 2 < g.nx);
    z.eoff = (z.lane == 0) ? -1 : 2;
    return z;
}

// x neighbours of a lane's pair: .x = left of cell i0, .y = right of i0 + 1
__device__ __forceinline__ double2 xnbr(const ZTile& z, double2 c, double edge) {
    const double l = __shfl_up(c.y, 1, 64);
    const double r = __shfl_down(c.x, 1, 64);
    return make_double2(z.lane == 0 ? edge : l, z.lane == 63 ? edge : r);
}

struct PredCoef2 {
    double two_dx, two_dy, inv_2dz;  // first derivatives
    double dx_sq, dy_sq, inv_dz2;    // second derivatives
    double r_two_dx, r_two_dy, r_dx_sq, r_dy_sq;  // RN(1 / divisor) for divz
    double dt, nu;
    double beta, T_ref, g0, g1, g2;
};

// solver_projection.c:121-182 for one cell: c = centre (u, v, w), f = the
// field the output belongs to (0, 1, 2) with its 6 neighbours
template <class Dv>
__device__ __forceinline__ double pred_cell(const PredCoef2& pc, Dv dv, double u, double v,
                                            double w, double fc, double xm, double xp, double ym,
                                            double yp, double zm, double zp, double src) {
    const double d_dx = dv(xp - xm, pc.two_dx, pc.r_two_dx);
    const double d_dy = dv(yp - ym, pc.two_dy, pc.r_two_dy);
    const double d_dz = (zp - zm) * pc.inv_2dz;
    const double conv = u * d_dx + v * d_dy + w * d_dz;
    const double d2x = dv(xp - 2.0 * fc + xm, pc.dx_sq, pc.r_dx_sq);
    const double d2y = dv(yp - 2.0 * fc + ym, pc.dy_sq, pc.r_dy_sq);
    const double d2z = (zp - 2.0 * fc + zm) * pc.inv_dz2;
    const double visc = pc.nu * (d2x + d2y + d2z);
    const double a = fc + pc.dt * (-conv + visc + src);
    return fmax(-100.0, fmin(100.0, a));
}

// The loads of plane k + 1 (the z+ centre row, the two y rows, the x-edge
// cells, T) are issued while plane k is computed: two register slots
// alternate over an unrolled pair of planes, so a slot is first read one
// step after its loads were issued.
struct PredBundle {
    double2 pp[3], ym[3], yp[3], tc;
    double e[3];
};

// PF: 0 = each plane's loads issued in its own step, 1 = one plane ahead in
// two alternating register slots (more VGPRs, two waves per SIMD).
template <int PF>
constexpr int pred_min_waves() { return PF ? 2 : 4; }

template <bool BUOY, int PF>
static __global__ __launch_bounds__(64 * PR_TY, pred_min_waves<PF>()) void k_pred2(
    SGeo g, PredCoef2 pc, const double* __restrict__ U, const double* __restrict__ V,
    const double* __restrict__ W, const double* __restrict__ T,
    const double* __restrict__ src_u_row, const double* __restrict__ src_v_col,
    double* __restrict__ us, double* __restrict__ vs, double* __restrict__ ws) {
    const ZTile z = ztile(g);
    if (z.j < 1 || z.j > g.ny - 2) {  // boundary rows: k_shell_copy
        if (CFD_PR_SYNC)
            for (int k = z.kb; k < z.ke; ++k) __syncthreads();
        return;
    }
    const double su = src_u_row[z.j];
    const double sv0 = z.xok ? src_v_col[z.i0] : 0.0;
    const double sv1 = z.in1 ? src_v_col[z.i0 + 1] : 0.0;
    const double* F[3] = {U, V, W};
    double* O[3] = {us, vs, ws};
    const long long idx0 = (long long)z.kb * g.ps + z.col;
    auto issue = [&](PredBundle& b, long long idx) __attribute__((always_inline)) {
#pragma unroll
        for (int f = 0; f < 3; ++f) {
            b.pp[f] = ld2(F[f], idx + g.sz);
            b.ym[f] = ld2(F[f], idx - g.px);
            b.yp[f] = ld2(F[f], idx + g.px);
            b.e[f] = z.eok ? F[f][idx + z.eoff] : 0.0;
        }
        b.tc = BUOY ? ld2(T, idx) : make_double2(0.0, 0.0);
    };
    double2 pm[3], pc3[3];
#pragma unroll
    for (int f = 0; f < 3; ++f) {
        pm[f] = ld2(F[f], idx0 - g.sz);
        pc3[f] = ld2(F[f], idx0);
    }
    // plane k from bundle b; the loads of plane k + 1 go to nb first
    auto step = [&](const PredBundle& b0, PredBundle& nb, int k) __attribute__((always_inline)) {
        if (CFD_PR_SYNC) __syncthreads();  // keep the tile's waves on one plane
        const long long idx = idx0 + (long long)(k - z.kb) * g.ps;
        PredBundle cur;
        if (PF) {
            if (k + 1 < z.ke) issue(nb, idx + g.ps);
        } else {
            issue(cur, idx);
        }
        const PredBundle& b = PF ? b0 : cur;
        const double u0 = pc3[0].x, u1 = pc3[0].y;
        const double v0 = pc3[1].x, v1 = pc3[1].y;
        const double w0 = pc3[2].x, w1 = pc3[2].y;
        // sources: compute_source_terms + energy_compute_buoyancy
        // (solver_explicit_euler.c:317-333, energy_solver.c:185-196)
        double s0[3] = {su, sv0, 0.0}, s1[3] = {su, sv1, 0.0};
        if (BUOY) {
            const double dT0 = b.tc.x - pc.T_ref, dT1 = b.tc.y - pc.T_ref;
            s0[0] += -pc.beta * dT0 * pc.g0;
            s0[1] += -pc.beta * dT0 * pc.g1;
            s0[2] += -pc.beta * dT0 * pc.g2;
            s1[0] += -pc.beta * dT1 * pc.g0;
            s1[1] += -pc.beta * dT1 * pc.g1;
            s1[2] += -pc.beta * dT1 * pc.g2;
        }
#pragma unroll
        for (int f = 0; f < 3; ++f) {
            const double2 lr = xnbr(z, pc3[f], b.e[f]);
            // fast divisions, then one wave-uniform check per field: lanes
            // with a quotient outside divz's range redo the pair with the
            // generic division (bitwise the same where both apply)
            double r0, r1;
            auto compute = [&](auto dv) __attribute__((always_inline)) {
                r0 = pred_cell(pc, dv, u0, v0, w0, pc3[f].x, lr.x, pc3[f].y, b.ym[f].x,
                               b.yp[f].x, pm[f].x, b.pp[f].x, s0[f]);
                r1 = pred_cell(pc, dv, u1, v1, w1, pc3[f].y, pc3[f].x, lr.y, b.ym[f].y,
                               b.yp[f].y, pm[f].y, b.pp[f].y, s1[f]);
            };
            bool ok = true;
            compute(DivFastZ{ok});
            if (__builtin_expect(wave_any_bad(ok), 0)) {
                if (!ok) compute(DivExact{});
            }
            double2 o = pc3[f];  // boundary cells: u* = u
            if (z.in0) o.x = r0;
            if (z.in1) o.y = r1;
            if (z.xok) st2(O[f], idx, o);
        }
#pragma unroll
        for (int f = 0; f < 3; ++f) {
            pm[f] = pc3[f];
            pc3[f] = b.pp[f];
        }
    };
    PredBundle A, B;
    if constexpr (PF != 0) {
        issue(A, idx0);
        int k = z.kb;
        for (; k + 1 < z.ke; k += 2) {
            step(A, B, k);
            step(B, A, k + 1);
        }
        if (k < z.ke) step(A, B, k);
    } else {
        for (int k = z.kb; k < z.ke; ++k) step(A, B, k);
    }
}

// Boundary shell of the predictor: u* = u on every cell the z-march does not
// write (rows j = 0, ny - 1 of every plane, the x edges, the z faces).
static __global__ __launch_bounds__(256) void k_shell_copy(Geo g, const double* __restrict__ U,
                                                           const double* __restrict__ V,
                                                           const double* __restrict__ W,
                                                           double* __restrict__ us,
                                                           double* __restrict__ vs,
                                                           double* __restrict__ ws) {
    const long long total = shell_total(g);
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {
        int i, j, k;
        bool zlo, zhi;
        shell_cell(g, e, i, j, k, zlo, zhi);
        const long long d = cidx(g, i, j, k);
        us[d] = U[d];
        vs[d] = V[d];
        ws[d] = W[d];
    }
}

// Corrector (solver_projection.c:230-250) on the interior rows and planes +
// NaN/Inf scan and max |u|, max |p| of those cells; boundary cells of the
// tile's rows keep u (== u*) and join the scan. The rest of the shell is
// scanned by k_shell_stats. red[0] = max |u|^2 (encoded), [1] = max |p|,
// [2] = non-finite flag.
struct CorrCoef2 {
    double two_dx, two_dy, inv_2dz;
    double r_two_dx, r_two_dy;
    double dt_over_rho;
};

__device__ __forceinline__ void corr_reduce(double mv, double mp, bool bad,
                                            unsigned long long* red) {
    __shared__ double shv[PR_TY], shp[PR_TY];
    __shared__ int shbad;
    if (threadIdx.x == 0) shbad = 0;
    __syncthreads();
    mv = wave_max(mv);
    mp = wave_max(mp);
    if (bad) shbad = 1;
    if ((threadIdx.x & 63) == 0) {
        shv[threadIdx.x >> 6] = mv;
        shp[threadIdx.x >> 6] = mp;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = shv[0], b = shp[0];
        for (int q = 1; q < PR_TY; ++q) {
            a = fmax(a, shv[q]);
            b = fmax(b, shp[q]);
        }
        atomicMax(&red[0], ord_enc(a));
        atomicMax(&red[1], ord_enc(b));
        if (shbad) atomicOr(&red[2], 1ull);
    }
}

__device__ __forceinline__ void cell_stats(double u, double v, double w, double p, double& mv,
                                           double& mp, bool& bad) {
    if (!isfinite(u) || !isfinite(v) || !isfinite(w) || !isfinite(p)) bad = true;
    // solver_registry.c:31-49 takes max sqrt(u^2 + v^2 + w^2); sqrt is
    // correctly rounded, hence monotone, so the maximum of the squared speeds
    // is reduced (red[0]) and the host takes one sqrt of it: bitwise the same
    // value, and no fp64 sqrt sequence per cell
    const double vel2 = (u * u) + (v * v) + (w * w);
    if (vel2 > mv) mv = vel2;
    const double ap = fabs(p);
    if (ap > mp) mp = ap;
}

struct CorrBundle {
    double2 pp, ym, yp, a, b, c;
    double e;
};

// PF as in k_pred2: 1 = the loads of plane k + 1 are issued during plane k
template <int PF>
static __global__ __launch_bounds__(64 * PR_TY, PF ? 3 : 4) void k_corr2(
    SGeo g, CorrCoef2 cc, const double* __restrict__ us, const double* __restrict__ vs,
    const double* __restrict__ ws, const double* __restrict__ P, double* __restrict__ U,
    double* __restrict__ V, double* __restrict__ W, unsigned long long* red) {
    const ZTile z = ztile(g);
    double mv = 0.0, mp = 0.0;
    bool bad = false;
    if (z.j >= 1 && z.j <= g.ny - 2) {  // wave-uniform
        const long long idx0 = (long long)z.kb * g.ps + z.col;
        double2 pm = ld2(P, idx0 - g.sz), pc = ld2(P, idx0);
        auto issue = [&](CorrBundle& q, long long idx) __attribute__((always_inline)) {
            q.pp = ld2(P, idx + g.sz);
            q.ym = ld2(P, idx - g.px);
            q.yp = ld2(P, idx + g.px);
            q.e = z.eok ? P[idx + z.eoff] : 0.0;
            q.a = ld2(us, idx);
            q.b = ld2(vs, idx);
            q.c = ld2(ws, idx);
        };
        auto step = [&](const CorrBundle& q0, CorrBundle& nq, int k) __attribute__((always_inline)) {
            if (CFD_PR_SYNC) __syncthreads();  // keep the tile's waves on one plane
            const long long idx = idx0 + (long long)(k - z.kb) * g.ps;
            CorrBundle cur;
            if (PF) {
                if (k + 1 < z.ke) issue(nq, idx + g.ps);
            } else {
                issue(cur, idx);
            }
            const CorrBundle& q = PF ? q0 : cur;
            const double2 lr = xnbr(z, pc, q.e);
            const double left = lr.x, right = lr.y;
            double2 nu = q.a, nv = q.b, nw = q.c;  // boundary cells: u = u* (== u)
            // fast divisions, one wave-uniform check, generic division for
            // lanes whose quotients left divz's range (as in k_pred2)
            double dx0, dy0, dx1, dy1;
            auto compute = [&](auto dv) __attribute__((always_inline)) {
                dx0 = dv(pc.y - left, cc.two_dx, cc.r_two_dx);
                dy0 = dv(q.yp.x - q.ym.x, cc.two_dy, cc.r_two_dy);
                dx1 = dv(right - pc.x, cc.two_dx, cc.r_two_dx);
                dy1 = dv(q.yp.y - q.ym.y, cc.two_dy, cc.r_two_dy);
            };
            bool ok = true;
            compute(DivFastZ{ok});
            if (__builtin_expect(wave_any_bad(ok), 0)) {
                if (!ok) compute(DivExact{});
            }
            {
                const double dp_dz = (q.pp.x - pm.x) * cc.inv_2dz;
                const double x0 = fmax(-100.0, fmin(100.0, q.a.x - cc.dt_over_rho * dx0));
                const double y0 = fmax(-100.0, fmin(100.0, q.b.x - cc.dt_over_rho * dy0));
                const double w0 = fmax(-100.0, fmin(100.0, q.c.x - cc.dt_over_rho * dp_dz));
                if (z.in0) {
                    nu.x = x0;
                    nv.x = y0;
                    nw.x = w0;
                }
            }
            {
                const double dp_dz = (q.pp.y - pm.y) * cc.inv_2dz;
                const double x1 = fmax(-100.0, fmin(100.0, q.a.y - cc.dt_over_rho * dx1));
                const double y1 = fmax(-100.0, fmin(100.0, q.b.y - cc.dt_over_rho * dy1));
                const double w1 = fmax(-100.0, fmin(100.0, q.c.y - cc.dt_over_rho * dp_dz));
                if (z.in1) {
                    nu.y = x1;
                    nv.y = y1;
                    nw.y = w1;
                }
            }
            if (z.xok) {
                st2(U, idx, nu);
                st2(V, idx, nv);
                st2(W, idx, nw);
                cell_stats(nu.x, nv.x, nw.x, pc.x, mv, mp, bad);
                if (z.i0 + 1 < g.nx) cell_stats(nu.y, nv.y, nw.y, pc.y, mv, mp, bad);
            }
            pm = pc;
            pc = q.pp;
        };
        CorrBundle A, B;
        if constexpr (PF != 0) {
            issue(A, idx0);
            int k = z.kb;
            for (; k + 1 < z.ke; k += 2) {
                step(A, B, k);
                step(B, A, k + 1);
            }
            if (k < z.ke) step(A, B, k);
        } else {
            for (int k = z.kb; k < z.ke; ++k) step(A, B, k);
        }
    } else if (CFD_PR_SYNC) {
        for (int k = z.kb; k < z.ke; ++k) __syncthreads();
    }
    corr_reduce(mv, mp, bad, red);
}

// ---------------------------------------------------------------------------
// r03: the predictor and corrector on the CG sweeps' 128 x 16 tiles with the
// y neighbours from LDS (k_pred3, k_corr3). Each wave owns one row of the
// tile, the two edge waves also load the row beyond it (the y halo), and
// every wave publishes its centre row once per plane: a stencil field's rows
// are read from HBM 18 times per 16 rows written, where the 4-row tiles of
// k_pred2 / k_corr2 need L2 hits for 6 reads per 4 rows (k_pred2 fetched
// 45.8 B/cell for 24 B of reads, profiles/r02e_rocprof_summary.txt). One
// barrier per plane, rows double-buffered by plane parity. Operands and
// operation order are k_pred2's / k_corr2's, so the results are bitwise
// theirs. FL: SW_NT_STORE = non-temporal stores of the outputs, SW_NT_LOAD =
// non-temporal loads of the pointwise inputs (the corrector's u*, v*, w*).
// ---------------------------------------------------------------------------
constexpr int PC_TY = 16;

template <bool BUOY, int FL>
static __global__ __launch_bounds__(64 * PC_TY, 1) void k_pred3(
    SGeo g, PredCoef2 pc, const double* __restrict__ U, const double* __restrict__ V,
    const double* __restrict__ W, const double* __restrict__ T,
    const double* __restrict__ src_u_row, const double* __restrict__ src_v_col,
    double* __restrict__ us, double* __restrict__ vs, double* __restrict__ ws) {
    constexpr int TY = PC_TY;
    __shared__ double2 rows[2][3][TY + 2][64];
    const RowPair c = row_pair<TY>(g);
    const bool halo = (c.w == 0) || (c.w == TY - 1);
    const int jc = min(c.j, g.ny - 1);
    const int jh = (c.w == 0) ? max(c.j - 1, 0) : min(c.j + 1, g.ny - 1);
    const int hslot = (c.w == 0) ? 0 : TY + 1;
    const long long hoff = (long long)(jh - jc) * g.px;
    const bool xok = c.i0 < g.nx;
    const bool eok = (c.lane == 0 && c.i0 >= 1 && xok) || (c.lane == 63 && c.i0 + 2 < g.nx);
    const long long eoff = (c.lane == 0) ? -1 : 2;
    const double su = src_u_row[jc];
    const double sv0 = xok ? src_v_col[c.i0] : 0.0;
    const double sv1 = c.in1 ? src_v_col[c.i0 + 1] : 0.0;
    const double* F[3] = {U, V, W};
    double* O[3] = {us, vs, ws};
    const double2 zero = make_double2(0.0, 0.0);
    long long idx = c.idx;
    // rows of plane k are published into rows[k & 1] at the end of step
    // k - 1 (that buffer was last read in step k - 2, before the barrier of
    // step k - 1), so no row value is held in registers across a barrier
    double2 pm[3], pcv[3];
#pragma unroll
    for (int f = 0; f < 3; ++f) {
        pm[f] = ld2(F[f], idx - g.sz);
        pcv[f] = ld2(F[f], idx);
        rows[0][f][c.w + 1][c.lane] = pcv[f];
        if (halo) rows[0][f][hslot][c.lane] = ld2(F[f], idx + hoff);
    }
    int buf = 0;
    for (int k = c.kb; k < c.ke; ++k, idx += g.ps) {
        // this plane's loads: the z+ centre row, the halo row of plane k + 1,
        // the x-edge cells, T
        double2 pp[3], hn[3];
        double e[3];
#pragma unroll
        for (int f = 0; f < 3; ++f) {
            pp[f] = ld2(F[f], idx + g.sz);
            hn[f] = halo ? ld2(F[f], idx + g.sz + hoff) : zero;
            e[f] = eok ? F[f][idx + eoff] : 0.0;
        }
        const double2 tc = BUOY ? ld2(T, idx) : zero;
        __syncthreads();
        const double u0 = pcv[0].x, u1 = pcv[0].y;
        const double v0 = pcv[1].x, v1 = pcv[1].y;
        const double w0 = pcv[2].x, w1 = pcv[2].y;
        double s0[3] = {su, sv0, 0.0}, s1[3] = {su, sv1, 0.0};
        if (BUOY) {
            const double dT0 = tc.x - pc.T_ref, dT1 = tc.y - pc.T_ref;
            s0[0] += -pc.beta * dT0 * pc.g0;
            s0[1] += -pc.beta * dT0 * pc.g1;
            s0[2] += -pc.beta * dT0 * pc.g2;
            s1[0] += -pc.beta * dT1 * pc.g0;
            s1[1] += -pc.beta * dT1 * pc.g1;
            s1[2] += -pc.beta * dT1 * pc.g2;
        }
#pragma unroll
        for (int f = 0; f < 3; ++f) {
            const double2 ys = rows[buf][f][c.w][c.lane];
            const double2 yn = rows[buf][f][c.w + 2][c.lane];
            const double l = __shfl_up(pcv[f].y, 1, 64);
            const double rr = __shfl_down(pcv[f].x, 1, 64);
            const double left = c.lane == 0 ? e[f] : l;
            const double right = c.lane == 63 ? e[f] : rr;
            double r0, r1;
            auto compute = [&](auto dv) __attribute__((always_inline)) {
                r0 = pred_cell(pc, dv, u0, v0, w0, pcv[f].x, left, pcv[f].y, ys.x, yn.x, pm[f].x,
                               pp[f].x, s0[f]);
                r1 = pred_cell(pc, dv, u1, v1, w1, pcv[f].y, pcv[f].x, right, ys.y, yn.y, pm[f].y,
                               pp[f].y, s1[f]);
            };
            bool ok = true;
            compute(DivFastZ{ok});
            if (__builtin_expect(wave_any_bad(ok), 0)) {
                if (!ok) compute(DivExact{});
            }
            double2 o = pcv[f];  // boundary cells: u* = u
            if (c.in0) o.x = r0;
            if (c.in1) o.y = r1;
            if (c.act) st2v<FL>(O[f], idx, o);
        }
        buf ^= 1;
#pragma unroll
        for (int f = 0; f < 3; ++f) {
            pm[f] = pcv[f];
            pcv[f] = pp[f];
            rows[buf][f][c.w + 1][c.lane] = pp[f];
            if (halo) rows[buf][f][hslot][c.lane] = hn[f];
        }
    }
}

template <int NW>
__device__ __forceinline__ void corr_reduce_n(double mv, double mp, bool bad,
                                              unsigned long long* red) {
    __shared__ double shv[NW], shp[NW];
    __shared__ int shbad;
    if (threadIdx.x == 0) shbad = 0;
    __syncthreads();
    mv = wave_max(mv);
    mp = wave_max(mp);
    if (bad) shbad = 1;
    if ((threadIdx.x & 63) == 0) {
        shv[threadIdx.x >> 6] = mv;
        shp[threadIdx.x >> 6] = mp;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double a = shv[0], b = shp[0];
        for (int q = 1; q < NW; ++q) {
            a = fmax(a, shv[q]);
            b = fmax(b, shp[q]);
        }
        atomicMax(&red[0], ord_enc(a));
        atomicMax(&red[1], ord_enc(b));
        if (shbad) atomicOr(&red[2], 1ull);
    }
}

template <int FL>
static __global__ __launch_bounds__(64 * PC_TY, 1) void k_corr3(
    SGeo g, CorrCoef2 cc, const double* __restrict__ us, const double* __restrict__ vs,
    const double* __restrict__ ws, const double* __restrict__ P, double* __restrict__ U,
    double* __restrict__ V, double* __restrict__ W, unsigned long long* red) {
    constexpr int TY = PC_TY;
    __shared__ double2 rows[2][TY + 2][64];
    const RowPair c = row_pair<TY>(g);
    const bool halo = (c.w == 0) || (c.w == TY - 1);
    const int jc = min(c.j, g.ny - 1);
    const int jh = (c.w == 0) ? max(c.j - 1, 0) : min(c.j + 1, g.ny - 1);
    const int hslot = (c.w == 0) ? 0 : TY + 1;
    const long long hoff = (long long)(jh - jc) * g.px;
    const bool xok = c.i0 < g.nx;
    const bool eok = (c.lane == 0 && c.i0 >= 1 && xok) || (c.lane == 63 && c.i0 + 2 < g.nx);
    const long long eoff = (c.lane == 0) ? -1 : 2;
    const double2 zero = make_double2(0.0, 0.0);
    double mv = 0.0, mp = 0.0;
    bool bad = false;
    long long idx = c.idx;
    double2 pm = ld2(P, idx - g.sz), pcv = ld2(P, idx);
    rows[0][c.w + 1][c.lane] = pcv;  // publishing as in k_pred3
    if (halo) rows[0][hslot][c.lane] = ld2(P, idx + hoff);
    int buf = 0;
    for (int k = c.kb; k < c.ke; ++k, idx += g.ps) {
        const double2 pp = ld2(P, idx + g.sz);
        const double2 hn = halo ? ld2(P, idx + g.sz + hoff) : zero;
        const double e = eok ? P[idx + eoff] : 0.0;
        const double2 qa = ld2v<FL>(us, idx), qb = ld2v<FL>(vs, idx), qc = ld2v<FL>(ws, idx);
        __syncthreads();
        const double2 ys = rows[buf][c.w][c.lane];
        const double2 yn = rows[buf][c.w + 2][c.lane];
        const double l = __shfl_up(pcv.y, 1, 64);
        const double rr = __shfl_down(pcv.x, 1, 64);
        const double left = c.lane == 0 ? e : l;
        const double right = c.lane == 63 ? e : rr;
        double2 nu = qa, nv = qb, nw = qc;  // boundary cells: u = u* (== u)
        double dx0, dy0, dx1, dy1;
        auto compute = [&](auto dv) __attribute__((always_inline)) {
            dx0 = dv(pcv.y - left, cc.two_dx, cc.r_two_dx);
            dy0 = dv(yn.x - ys.x, cc.two_dy, cc.r_two_dy);
            dx1 = dv(right - pcv.x, cc.two_dx, cc.r_two_dx);
            dy1 = dv(yn.y - ys.y, cc.two_dy, cc.r_two_dy);
        };
        bool ok = true;
        compute(DivFastZ{ok});
        if (__builtin_expect(wave_any_bad(ok), 0)) {
            if (!ok) compute(DivExact{});
        }
        {
            const double dp_dz = (pp.x - pm.x) * cc.inv_2dz;
            const double x0 = fmax(-100.0, fmin(100.0, qa.x - cc.dt_over_rho * dx0));
            const double y0 = fmax(-100.0, fmin(100.0, qb.x - cc.dt_over_rho * dy0));
            const double w0 = fmax(-100.0, fmin(100.0, qc.x - cc.dt_over_rho * dp_dz));
            if (c.in0) {
                nu.x = x0;
                nv.x = y0;
                nw.x = w0;
            }
        }
        {
            const double dp_dz = (pp.y - pm.y) * cc.inv_2dz;
            const double x1 = fmax(-100.0, fmin(100.0, qa.y - cc.dt_over_rho * dx1));
            const double y1 = fmax(-100.0, fmin(100.0, qb.y - cc.dt_over_rho * dy1));
            const double w1 = fmax(-100.0, fmin(100.0, qc.y - cc.dt_over_rho * dp_dz));
            if (c.in1) {
                nu.y = x1;
                nv.y = y1;
                nw.y = w1;
            }
        }
        if (c.act) {
            st2v<FL>(U, idx, nu);
            st2v<FL>(V, idx, nv);
            st2v<FL>(W, idx, nw);
            cell_stats(nu.x, nv.x, nw.x, pcv.x, mv, mp, bad);
            if (c.i0 + 1 < g.nx) cell_stats(nu.y, nv.y, nw.y, pcv.y, mv, mp, bad);
        }
        pm = pcv;
        pcv = pp;
        buf ^= 1;
        rows[buf][c.w + 1][c.lane] = pp;
        if (halo) rows[buf][hslot][c.lane] = hn;
    }
    corr_reduce_n<TY>(mv, mp, bad, red);
}

// Stats over the boundary shell cells the corrector's z-march does not visit
// (rows j = 0, ny - 1 of the owned planes, the global z faces): u, v, w are
// the caller's boundary values there. Planes [ks, ke) as in the corrector.
static __global__ __launch_bounds__(256) void k_shell_stats(Geo g, const double* __restrict__ U,
                                                            const double* __restrict__ V,
                                                            const double* __restrict__ W,
                                                            const double* __restrict__ P,
                                                            unsigned long long* red) {
    __shared__ double shv[4], shp[4];
    __shared__ int shbad;
    if (threadIdx.x == 0) shbad = 0;
    __syncthreads();
    const int ks = (g.nz > 1 && !g.lo_face) ? 1 : 0;
    const int ke = (g.nz > 1 && !g.hi_face) ? g.nz - 1 : g.nz;
    const long long total = shell_total(g);
    double mv = 0.0, mp = 0.0;
    bool bad = false;
    for (long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (long long)gridDim.x * blockDim.x) {
        int i, j, k;
        bool zlo, zhi;
        shell_cell(g, e, i, j, k, zlo, zhi);
        // the z-march covers i = 0 / nx - 1 of its rows on interior planes
        const bool marched = (j >= 1 && j <= g.ny - 2 && k >= g.k0 && k < g.k1);
        if (k < ks || k >= ke || marched) continue;
        const long long d = cidx(g, i, j, k);
        cell_stats(U[d], V[d], W[d], P[d], mv, mp, bad);
    }
    mv = wave_max(mv);
    mp = wave_max(mp);
    if (bad) shbad = 1;
    if ((threadIdx.x & 63) == 0) {
        shv[threadIdx.x >> 6] = mv;
        shp[threadIdx.x >> 6] = mp;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        atomicMax(&red[0], ord_enc(fmax(fmax(shv[0], shv[1]), fmax(shv[2], shv[3]))));
        atomicMax(&red[1], ord_enc(fmax(fmax(shp[0], shp[1]), fmax(shp[2], shp[3]))));
        if (shbad) atomicOr(&red[2], 1ull);
    }
}

}  // namespace cfdhip
