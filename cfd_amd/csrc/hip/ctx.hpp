// ctx.hpp -- the device context behind the hip_proj_* C-ABI and the helpers
// shared by its translation units (projection_hip.hip: projection step and
// Poisson solvers; rk4_hip.hip: the RK4 integrator). Private to the library.
#pragma once

#include "kernels.hpp"
#include "slab_comm.hpp"

#include "cfd_hip/projection_hip.h"

#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <initializer_list>
#include <vector>

using namespace cfdhip;

// Error reporting goes through the host library's thread-local error state
// (cfd_set_error, logging.c:39-46 in the reference). Weak, so the library
// links against either the reference's host library or ours.
extern "C" void cfd_set_error(cfd_status_t status, const char* message) __attribute__((weak));

static inline void set_err(cfd_status_t s, const char* msg) {
    if (cfd_set_error) cfd_set_error(s, msg);
}

#define HIP_TRY(call)                                                              \
    do {                                                                           \
        hipError_t e_ = (call);                                                    \
        if (e_ != hipSuccess) {                                                    \
            char buf_[256];                                                        \
            snprintf(buf_, sizeof(buf_), "HIP error %s at %s:%d (%s)",             \
                     hipGetErrorString(e_), __FILE__, __LINE__, #call);            \
            set_err(CFD_ERROR, buf_);                                              \
            return CFD_ERROR;                                                      \
        }                                                                          \
    } while (0)

namespace {

struct TimedLaunch {
    hipEvent_t a, b;
    int kind;
    int iter;  // CG iteration of a sweep launch, -1 otherwise
};

}  // namespace

struct hip_proj_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    size_t nx = 0, ny = 0, nz = 0;
    long long px = 0, ps = 0;
    Geo geo{};
    SGeo sgeo{};       // row-pair CG sweep tiling
    SGeo sg_edge{}, sg_int{};  // slabs: sweep B split into edge planes + interior
    SGeo rgeo{};               // single-pass RB-SOR tiling (k_rb1)
    // slabs: one k_rb1 iteration as three launches sharing one reduction --
    // interior part 1 (overlaps the R halo exchange), the two edge planes,
    // interior part 2 (overlaps the exchange of the new iterate's edge planes)
    SGeo rg_in1{}, rg_edge{}, rg_in2{};
    int split_rb = 0;
    // one device: k_rb1's full-width (TC 64) tiles stop at x = 124 T, and the
    // remaining columns run as a strip of narrow tiles (TC 16 / 32) in a
    // second launch sharing the residual reduction (rb_strip_tc 0: none)
    SGeo rg_main{}, rg_strip{};
    int rb_strip_tc = 0;
    int rb1_tc = 64;           // k_rb1 tile width in x pairs (64, 32, 16)
    SGeo pgeo{};               // predictor / corrector z-march tiling (k_pred2, k_corr2)
    SGeo pgeo16{};             // k_pred3 / k_corr3: 128 x 16 tiles, y rows in LDS
    int pc3 = 1;  // 0: k_pred2 / k_corr2; k_pred3 / k_corr3 with 1: FL 0 (default), 2: NT stores, 4: + NT loads
    int split_b = 0;
    int sweep_ty = 8;  // waves (y rows) per CG sweep workgroup
    int sweep_variant = 0;  // SW_NT_* flags of the CG sweeps
    int sweep_variant_fold = 0;  // the fold sweep's flags (0: sweep_variant)
    int grid_cap = 2048;
    hip_proj_config_t cfg{};
    // Z-slab decomposition (nranks == 1: the whole grid, no communicator)
    SlabComm* comm = nullptr;
    int rank = 0, nranks = 1;
    size_t nzg = 0;    // global nz
    size_t kofs = 0;   // global index of local plane 0
    double* dsum = nullptr;            // [0] local dot total, [1] all-reduced
    unsigned long long* clk = nullptr;  // k_ccf clock sample: sum d memtime, d memrealtime, count
    hipStream_t hstream = nullptr;     // side stream: halo of r overlaps the (r,r) all-reduce
    hipEvent_t ev_b = nullptr, ev_h = nullptr;
    unsigned long long* redg = nullptr;  // all-reduced red[]
    // fields
    double *u = nullptr, *v = nullptr, *w = nullptr, *p = nullptr, *T = nullptr;
    double *us = nullptr, *vs = nullptr, *ws = nullptr, *pn = nullptr;
    double *r = nullptr, *pa = nullptr, *pb = nullptr;  // r; CG search directions
    double *pc4 = nullptr, *pd4 = nullptr;               // (ring of CG_XFOLD = 4: pa pb pc4 pd4)
    double *rhs = nullptr, *xt = nullptr;
    // RK4 borrows r, p_a, p_b, x_tmp as stage buffers and leaves wall values in
    // them; the CG needs zero wall cells in r and the p ring (lagged-BC
    // semantics), so the next CG solve clears them first.
    int cg_scratch_dirty = 0;
    // boundary handling of the pressure solve in progress (hip_poisson_bc_t):
    // NEUMANN = the reference's default apply_bc; NONE = boundary cells of x
    // never written (the caller's apply_bc runs on the host); FIXED = after
    // every relaxation iteration the shell is copied from bcfix
    int poisson_bc = 0;
    double* bcfix = nullptr;
    // resident mode of the host-buffer step (cfg.dirty_faces): the device
    // fields equal the caller's host arrays res_ptr[] except in the cells the
    // caller may have changed since (the boundary shell); any other entry
    // that changes device state clears `resident`
    int resident = 0;
    const double* res_ptr[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
    long long res_steps = 0;     // host steps since the last full download
    // dirty_verify_interval: hash of the host arrays' interior as the last
    // resident step left it (valid when hash_ok)
    unsigned long long host_hash[5] = {0, 0, 0, 0, 0};   // deep interior (hash_ok)
    unsigned long long host_hash1[5] = {0, 0, 0, 0, 0};  // layer 1, after the last step
    int hash_ok = 0, hash_nf = 0;
    double* shell_dev = nullptr;  // packed shell staging (device / pinned host)
    double* shell_host = nullptr;
    size_t shell_cap = 0;
    double *cw = nullptr, *cs = nullptr;  // cg_variant 1: w = A r, s = A p (lazily allocated)
    double* Tn = nullptr;  // energy equation output (swapped with T)
    double* rho = nullptr;  // per-cell density (RK4 reads rho[idx]); lazily allocated
    double* rk_acc[4] = {nullptr, nullptr, nullptr, nullptr};  // RK4 k1 + 2k2 + 2k3
    double *dxa = nullptr, *dya = nullptr;  // grid->dx[], grid->dy[] (RK4 per-index spacing)
    double *src_u_row = nullptr, *src_v_col = nullptr;
    // pinned host staging of the source-term tables (ny rows, then nx columns):
    // a plain DMA each step, never a staged pageable copy; ev_src marks the
    // last upload, so the host rewrites the tables only after it landed
    double* h_src = nullptr;
    hipEvent_t ev_src = nullptr;
    // reductions / state
    CgState* st = nullptr;
    RxState* rxst = nullptr;             // fused relaxation loop state
    RxState* rxst2 = nullptr;            // scratch state of k_rb2's recompute sweeps
    void* rb2dec = nullptr;              // k_rb2's decision constants (Rb2Dec, rb2.hpp)
    SGeo r2geo{};                        // two-iterations-per-sweep RB-SOR tiling (k_rb2)
    SGeo ccgeo{};                        // fused single-reduction CG tiling (k_ccf)
    SGeo cc_edge{}, cc_int{};            // slabs: k_ccf on the edge planes, then the rest
    // slabs, fused form: cc_int with stage c and a shared reduction, and
    // k_cc2's tiling of the two edge planes completing it (tiles_x 0: off)
    SGeo cc_int_red{}, cc2_edge{};
    int ccf_tail = 0, ccf_kc2 = 0;       // k_ccf tail layers of shorter runs (ccf_layout)
    std::vector<float> placement_ms;     // placement draws: ms per probe iteration, per draw
    int placement_pick = -1;             // the draw kept (-1: no draws)
    double* r2 = nullptr;                // k_ccf: r_{it+1} when r_it is in r (by parity)
    double* partials = nullptr;
    unsigned* counter = nullptr;
    unsigned long long* red = nullptr;   // [0] max |u|^2, [1] max |p|, [2] nonfinite, [3] max T, [4] residual
    CgState* h_state = nullptr;          // pinned, 2 slots + final
    unsigned long long* h_red = nullptr; // pinned, 8
    hipEvent_t ev_poll[2] = {nullptr, nullptr};
    double rho0 = 1.0;
    double max_T = 0.0;
    int have_T = 0;
    int T_dirty = 0;  // T changed since max_T was computed
    poisson_solver_stats_t pstats{};
    size_t bytes = 0;
    std::vector<void*> allocs;  // hipMalloc bases of the field arrays
    size_t stagger_bytes = 0;
    // Environment switches of the solve paths, read ONCE when the context
    // is created (init_ctx), never per step or per solve: rank threads of an
    // in-process group would otherwise call getenv while another thread of
    // the process (a test fixture, the runtime) may change the environment,
    // and getenv is not safe against a concurrent setenv / putenv. Tests set
    // the variables before they create contexts.
    struct {
        bool ccf_off = false;     // CFD_HIP_CCF=0: k_cc1 + k_cc2 instead of k_ccf
        int cg_small = -1;        // CFD_HIP_CG_SMALL (-1 unset, 0 never, 1 up to 1M cells)
        int rb2_test = 0;         // CFD_HIP_RB2_TEST: force k_rb2's host paths
        int rb2_xmap = 0;         // CFD_HIP_RB2_XMAP (experiments)
        bool rb2_log = false;     // CFD_HIP_RB2_LOG (diagnostics)
        int rb2 = 1;              // CFD_HIP_RB2: 1 certified fast, 2 exact, 0 k_rb1
        int ccf_xmap = 0;         // CFD_HIP_CCF_XMAP: k_ccf tile order (experiments)
        bool cgb_rev = true;      // CFD_HIP_CGB_REV=0: sweep B marches upwards
        bool rb1_pf = true;       // CFD_HIP_RB1_PF=0: k_rb1 end-of-step loads
        bool rb1_alt = true;      // CFD_HIP_RB1_ALT=0: every k_rb1 sweep upwards
        bool rb1_fold = true;     // CFD_HIP_RB1_FOLD=0: separate k_rx_shell launch
        bool rk_pair = true;      // CFD_HIP_RK_PAIR=0: per-cell RK4 stage
        bool alloc_contig = false;  // CFD_HIP_ALLOC=contig: contiguous field allocations
        bool ccf_edge_side = true;  // CFD_HIP_CCF_EDGE_SIDE=0: slab edge march before the interior
    } env;
    // timing
    int timing = 0;
    std::vector<hipEvent_t> ev_pool;
    size_t ev_used = 0;
    std::vector<TimedLaunch> pending;
    hipEvent_t ta = nullptr, tb = nullptr;  // events of the launch being timed
    double kt_ms[HIP_KT_COUNT] = {0};
    long long kt_n[HIP_KT_COUNT] = {0};
};

// ---------------------------------------------------------------------------
// small helpers
// ---------------------------------------------------------------------------
// Field arrays start at staggered offsets (k-th allocation shifted by
// k * stagger bytes, a multiple of 256 B) so that the streams a sweep reads
// and writes at the same index do not all begin on the same HBM channel.
static cfd_status_t dalloc(hip_proj_ctx* c, double** ptr, size_t n) {
    const size_t off = (size_t)c->allocs.size() * c->stagger_bytes;
    void* base = nullptr;
    // CFD_HIP_ALLOC=contig (experiments, r06): physically contiguous fields
    // (hipDeviceMallocContiguous), so the march's plane-strided accesses
    // translate through large pages whatever the box's memory history;
    // falls back to hipMalloc when the driver cannot place one
    if (c->env.alloc_contig &&
        hipExtMallocWithFlags(&base, n * sizeof(double) + off, hipDeviceMallocContiguous) != hipSuccess) {
        (void)hipGetLastError();
        base = nullptr;
    }
    if (!base) HIP_TRY(hipMalloc(&base, n * sizeof(double) + off));
    c->allocs.push_back(base);
    *ptr = (double*)((char*)base + off);
    HIP_TRY(hipMemsetAsync(*ptr, 0, n * sizeof(double), c->stream));
    c->bytes += n * sizeof(double) + off;
    return CFD_SUCCESS;
}

static size_t field_elems(const hip_proj_ctx* c) { return (size_t)c->ps * c->nz; }

static double* field_ptr(hip_proj_ctx* c, int id) {
    switch (id) {
        case HIP_FIELD_U: return c->u;
        case HIP_FIELD_V: return c->v;
        case HIP_FIELD_W: return c->w;
        case HIP_FIELD_P: return c->p;
        case HIP_FIELD_T: return c->T;
        case HIP_FIELD_RHO: return c->rho;
        default: return nullptr;
    }
}

static hipEvent_t take_event(hip_proj_ctx* c) {
    if (c->ev_used == c->ev_pool.size()) {
        hipEvent_t e;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        c->ev_pool.push_back(e);
    }
    return c->ev_pool[c->ev_used++];
}

// cg_limit: CG sweep launches of iterations >= cg_limit ran after convergence
// (launched ahead of the host poll, they return at once) and are not counted.
static void flush_timing(hip_proj_ctx* c, int cg_limit = 0x7fffffff) {
    for (auto& t : c->pending) {
        if (t.iter >= cg_limit) continue;
        float ms = 0.f;
        if (hipEventElapsedTime(&ms, t.a, t.b) == hipSuccess) {
            c->kt_ms[t.kind] += ms;
            c->kt_n[t.kind] += 1;
        }
    }
    c->pending.clear();
    c->ev_used = 0;
}

// Time a launch when timing is enabled: the kernel launched inside `launch`
// goes through hipExtLaunchKernelGGL with the context's (ta, tb), so the
// start/stop timestamps are taken by the dispatch packet itself (the kernel's
// own duration, no extra marker packets in the stream). The pool is flushed
// at every host synchronisation point.
template <typename F>
static void timed(hip_proj_ctx* c, int kind, F&& launch, int iter = -1) {
    if (!c->timing) {
        launch();
        return;
    }
    hipEvent_t a = take_event(c), b = take_event(c);
    if (!a || !b) {
        launch();
        return;
    }
    c->ta = a;
    c->tb = b;
    launch();
    c->ta = c->tb = nullptr;
    c->pending.push_back({a, b, kind, iter});
}

// Time a span of stream work that is not one kernel (RCCL calls, halo
// copies) with events recorded around it on stream `s`.
template <typename F>
static cfd_status_t timed_span(hip_proj_ctx* c, hipStream_t s, int kind, F&& fn, int iter = -1) {
    if (!c->timing) return fn();
    hipEvent_t a = take_event(c), b = take_event(c);
    if (!a || !b) return fn();
    if (hipEventRecord(a, s) != hipSuccess) return fn();
    cfd_status_t r = fn();
    if (hipEventRecord(b, s) == hipSuccess) c->pending.push_back({a, b, kind, iter});
    return r;
}

static int tile_grid(const hip_proj_ctx* c) {
    long long nt = (long long)c->geo.tiles_x * c->geo.tiles_y * c->geo.tiles_z;
    return (int)std::max(1LL, std::min<long long>(nt, c->grid_cap));
}

static int sweep_grid(const hip_proj_ctx* c) {
    return c->sgeo.tiles_x * c->sgeo.tiles_y * c->sgeo.tiles_z;
}

static bool dist(const hip_proj_ctx* c) { return c->nranks > 1; }

// one-shot device all-reduce mailbox of the slab communicator (or nullptr)
static inline Mbox* mbox(const hip_proj_ctx* c) {
    return (c->nranks > 1 && c->comm) ? c->comm->device_mailbox() : nullptr;
}

static dim3 cell_grid(const hip_proj_ctx* c) {
    return dim3((unsigned)((c->nx + 63) / 64), (unsigned)((c->ny + 3) / 4), (unsigned)c->nz);
}

static unsigned shell_blocks(const hip_proj_ctx* c) {
    long long ring = 2LL * c->nx + 2LL * (c->ny - 2);
    long long total = ring * (long long)c->nz + (c->nz > 1 ? 2LL * c->nx * c->ny : 0);
    long long b = (total + 255) / 256;
    return (unsigned)std::max(1LL, std::min(b, 65535LL));
}

static void launch_bc(hip_proj_ctx* c, double* f, int mode, const DirVals& dv) {
    hipExtLaunchKernelGGL(k_bc_shell, dim3(shell_blocks(c)), dim3(256), 0, c->stream, c->ta, c->tb, 0, c->geo, f,
                       mode, dv);
}

static __global__ void k_init_red(unsigned long long* red) {
    if (threadIdx.x == 0) {
        red[0] = 0x8000000000000000ull;  // enc(+0.0): reference maxima start at 0.0
        red[1] = 0x8000000000000000ull;
        red[2] = 0ull;
        red[5] = 0ull;
        red[3] = 0x000FFFFFFFFFFFFFull;  // enc(-inf)
        red[4] = 0x8000000000000000ull;
    }
}

static double ord_dec(unsigned long long e) {
    unsigned long long b = (e & 0x8000000000000000ull) ? (e & 0x7FFFFFFFFFFFFFFFull) : ~e;
    double d;
    memcpy(&d, &b, sizeof(d));
    return d;
}

static Lap make_lap(double dx, double dy, double dz) {
    Lap L;
    L.dx2_inv = 1.0 / (dx * dx);
    L.dy2_inv = 1.0 / (dy * dy);
    L.inv_dz2 = (dz > 0.0) ? (1.0 / (dz * dz)) : 0.0;
    return L;
}

// Refresh the halo planes of the given slab fields (no-op on one rank).
static cfd_status_t halo(hip_proj_ctx* c, std::initializer_list<double*> fs,
                         bool periodic = false) {
    if (!dist(c)) return CFD_SUCCESS;
    double* f[8];
    int n = 0;
    for (double* x : fs) f[n++] = x;
    return c->comm->halo(c->stream, f, n, c->ps, (int)c->nz, periodic);
}

// Sum the per-rank dot total dsum[0] into dsum[1].
static cfd_status_t reduce_dot(hip_proj_ctx* c) {
    return c->comm->allreduce_sum(c->stream, c->dsum, c->dsum + 1, 1);
}

// Device copy of the maxima/flags in red[] that every rank agrees on.
static const unsigned long long* reduce_red(hip_proj_ctx* c, cfd_status_t* st) {
    *st = CFD_SUCCESS;
    if (!dist(c)) return c->red;
    *st = c->comm->allreduce_max_u64(c->stream, c->red, c->redg, 8);
    return c->redg;
}

#define ST_TRY(expr)                            \
    do {                                        \
        cfd_status_t s_ = (expr);               \
        if (s_ != CFD_SUCCESS) return s_;       \
    } while (0)

// compute_source_terms at `iter` (solver_explicit_euler.c:317-333) on the
// host with the reference's libm expressions, uploaded to src_u_row /
// src_v_col from the pinned staging
static cfd_status_t upload_source_tables(hip_proj_ctx* c, const grid* g,
                                         const ns_solver_params_t* prm, int iter) {
    const size_t nx = c->nx, ny = c->ny;
    const double dt = prm->dt;
    HIP_TRY(hipEventSynchronize(c->ev_src));
    double* hu = c->h_src;
    double* hv = c->h_src + ny;
    for (size_t j = 0; j < ny; j++)
        hu[j] = prm->source_amplitude_u * sin(M_PI * g->y[j]) *
                exp(-prm->source_decay_rate * iter * dt);
    for (size_t i = 0; i < nx; i++)
        hv[i] = prm->source_amplitude_v * sin(2.0 * M_PI * g->x[i]) *
                exp(-prm->source_decay_rate * iter * dt);
    HIP_TRY(hipMemcpyAsync(c->src_u_row, hu, ny * sizeof(double), hipMemcpyHostToDevice,
                           c->stream));
    HIP_TRY(hipMemcpyAsync(c->src_v_col, hv, nx * sizeof(double), hipMemcpyHostToDevice,
                           c->stream));
    HIP_TRY(hipEventRecord(c->ev_src, c->stream));
    return CFD_SUCCESS;
}

// In-process Z-slab groups (slab_comm.hip LocalComm) drive their ranks'
// contexts from several host threads of one process. Their host work is
// serialised: a hip_proj_* entry point on a group context holds the group's
// host lock for the whole call, and a rank gives it up only while it waits
// at a group barrier (hip_proj_group::barrier). The device work of the ranks
// still overlaps (each rank has its own streams); what can no longer happen
// is two rank threads inside the HIP runtime or this library at once
// (the intermittent host segfault of the 3-rank Jacobi test).
// RCCL contexts (one process per GPU) and single-device contexts: no lock.
void group_host_enter(hip_proj_group* g) __attribute__((visibility("hidden")));
void group_host_leave(hip_proj_group* g) __attribute__((visibility("hidden")));
struct GroupHostLock {
    hip_proj_group* g;
    explicit GroupHostLock(const hip_proj_ctx* c)
        : g((c && c->comm) ? c->comm->host_group() : nullptr) {
        group_host_enter(g);
    }
    ~GroupHostLock() { group_host_leave(g); }
    GroupHostLock(const GroupHostLock&) = delete;
    GroupHostLock& operator=(const GroupHostLock&) = delete;
};


// Shared by the integrators (defined in projection_hip.hip).
cfd_status_t ctx_apply_thermal_bcs(hip_proj_ctx* c, const ns_thermal_bc_config_t& t, bool is3d)
    __attribute__((visibility("hidden")));
// Energy equation on the current velocity (alpha > 0 only), then the thermal
// BCs when apply_bcs; sets red[5] on non-finite T.
cfd_status_t ctx_energy_step(hip_proj_ctx* c, const grid* g, const ns_solver_params_t* prm,
                             bool apply_bcs) __attribute__((visibility("hidden")));
// Field validation shared by the step functions (grid match, callbacks,
// thermal BC types).
cfd_status_t ctx_validate_params(const hip_proj_ctx* c, const grid* g,
                                 const ns_solver_params_t* prm)
    __attribute__((visibility("hidden")));
// compute_max_temperature into red[3] when T changed; call before reduce_red.
void ctx_queue_max_T(hip_proj_ctx* c) __attribute__((visibility("hidden")));
// Boundary-shell transfers (shell_io.hip): depth-`depth` shell of nf fields
// between caller host arrays (nx*ny*nz) and device fields.
bool ctx_shell_fits(const hip_proj_ctx* c, int depth) __attribute__((visibility("hidden")));
cfd_status_t ctx_shell_put(hip_proj_ctx* c, const double* const* host, double* const* dev, int nf,
                           int depth) __attribute__((visibility("hidden")));
cfd_status_t ctx_shell_get(hip_proj_ctx* c, double* const* host, double* const* dev, int nf,
                           int depth) __attribute__((visibility("hidden")));
// compute_max_temperature over a host array (the reference's sequential
// result, computed on up to 16 threads; shell_io.hip).
double ctx_host_max(const double* T, size_t n) __attribute__((visibility("hidden")));
// Position-weighted 64-bit hashes of each host array's deep interior (all
// indices in [2, n-3]; layer1 = false) or of the layer next to the boundary
// (layer1 = true), multithreaded (shell_io.hip).
void ctx_host_hash(const hip_proj_ctx* c, const double* const* host, int nf, bool layer1,
                   unsigned long long* out) __attribute__((visibility("hidden")));
