/*
 * projection_hip.h -- C-ABI of the MI355X-native Chorin projection step.
 *
 * This is the drop-in boundary. Two layers:
 *
 *  1. The plugin factory `create_projection_hip_solver` returns an ns_solver_t
 *     (cfd_abi.h) whose step/solve have exactly the semantics of the
 *     reference's scalar `projection` solver (solver_registry.c:921-972 ->
 *     solver_projection.c:46-297), so a reference build registers it with
 *        cfd_registry_register(registry, "projection_hip", create_projection_hip_solver);
 *     next to `projection_gpu` (solver_registry.c:233-240) and drives it
 *     unchanged through init_simulation* / run_simulation_step / solver_step.
 *     `projection_hip_rbsor` and `projection_hip_jacobi` select the Red-Black
 *     SOR / Jacobi pressure solver instead of CG (the reference hard-codes CG
 *     in the projection, solver_projection.c:217-218). `projection_hip_cg1`
 *     runs the single-reduction (Chronopoulos-Gear) CG, hip_proj_config_t
 *     .cg_variant = 1: the same stopping rule and stats, one reduction per
 *     iteration, iterates equal to textbook CG's up to rounding.
 *
 *  2. The thin context API (`hip_proj_*`) the plugin calls. It owns all
 *     device memory, so it also serves device-resident drivers (bench.py,
 *     long runs): upload once, step many times in HBM, download at the end.
 *     It replaces the reference's per-call CUDA driver
 *     solve_projection_method_gpu (lib/src/solvers/gpu/solver_projection_gpu.cu:617-770)
 *     and the persistent-context API of lib/include/cfd/core/gpu_device.h:145-194.
 *
 * No HIP or torch types appear in any signature.
 */
#ifndef CFD_HIP_PROJECTION_HIP_H
#define CFD_HIP_PROJECTION_HIP_H

#include "cfd_hip/cfd_abi.h"

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NS_SOLVER_TYPE_PROJECTION_HIP        "projection_hip"
#define NS_SOLVER_TYPE_PROJECTION_HIP_RBSOR  "projection_hip_rbsor"
#define NS_SOLVER_TYPE_PROJECTION_HIP_JACOBI "projection_hip_jacobi"
#define NS_SOLVER_TYPE_PROJECTION_HIP_CG1    "projection_hip_cg1"
#define NS_SOLVER_TYPE_RK4_HIP               "rk4_hip"

/* Pressure-Poisson method used inside the HIP projection step. */
typedef enum {
    HIP_POISSON_CG = 0,       /* textbook CG, linear_solver_cg.c:290-461 */
    HIP_POISSON_REDBLACK = 1, /* Red-Black SOR, linear_solver_redblack.c:80-147 */
    HIP_POISSON_JACOBI = 2    /* Jacobi, linear_solver_jacobi.c:76-129 */
} hip_poisson_method_t;

/* Device/solver configuration (role of gpu_config_t, gpu_device.h:32-53). The
 * Poisson defaults are the CPU reference's (linear_solver.c:37-47), not the
 * reference GPU's looser 1e-3 / 1000 (solver_projection_gpu.cu:301-302). */
typedef struct {
    int device;                   /* HIP device ordinal; -1 = current device */
    int poisson_method;           /* hip_poisson_method_t */
    double poisson_tolerance;     /* relative residual tolerance (1e-6) */
    double poisson_abs_tolerance; /* absolute residual tolerance (1e-10) */
    int poisson_max_iter;         /* 5000 for CG/RB-SOR, 2000 for Jacobi */
    int poisson_check_interval;   /* convergence check period (1) */
    double sor_omega;             /* <= 0: optimal omega (linear_solver_internal.h:184-220) */
    int poll_interval;            /* iterations launched between host convergence polls */
    int kchunk;                   /* z planes per CG sweep tile; 0 = auto (64) */
    int verbose;
    int sweep_rows;               /* y rows (wavefronts) per CG sweep workgroup: 4, 8 or 16
                                     (default 16) */
    int sweep_variant;            /* CG sweep memory hints: bit0 non-temporal stores,
                                     bit1 non-temporal loads of single-use inputs, bit2 loads
                                     issued one plane ahead, bit3 both x-edge cells of a row
                                     in one load instruction, bit4 non-temporal loads of
                                     inner-wave centre rows (built: 0-3, 4, 7; with 16 rows
                                     also 15, 23, 31; default 15) */
    int rhs_density;              /* 1: rhs = (rho/dt) div u* (solver_projection.c:195-211,
                                     default); 0: div u* / dt, the reference GPU's
                                     (solver_projection_gpu.cu:706-707) */
    int poisson_fail_fatal;       /* 1: a pressure solve that stops unconverged fails the
                                     step with CFD_ERROR_MAX_ITER, field untouched
                                     (solver_projection.c:220-224, default); 0: the step
                                     continues with the capped solve, as the reference GPU
                                     does (solver_projection_gpu.cu:717-733) */
    int relax_two_pass;           /* RB-SOR / Jacobi: 0 = device loop, RB-SOR in one pass per
                                     iteration in 3-D, on one device or on Z-slabs (default);
                                     1 = separate colour passes + residual pass with a host
                                     check per iteration (the r01 form); 2 = device loop with
                                     the two colour sweeps */
    int sweep_variant_fold;       /* ignored since r02: x is folded by sweep A, with
                                     sweep_variant's hints (kept for layout stability) */
    int dirty_faces;              /* host-buffer step (hip_proj_step, the plugin's `step`):
                                     0 = upload and download u, v, w, p (T) in full every
                                     step (default); 1 = resident mode: the interior stays in
                                     HBM between steps on the same host arrays, a step uploads
                                     only the boundary shell (the cells a caller's BC routine
                                     writes) and downloads the two outer layers (what it
                                     reads). The rest of the host arrays is refreshed by
                                     hip_proj_sync_host, every dirty_sync_interval steps, and
                                     after a failed step. Any other entry that changes device
                                     state (set_field, fill, BCs, step_device, poisson_solve,
                                     checkpoint_read, RK4) or new host arrays end the resident
                                     run: the next step uploads the host arrays in full, so
                                     call hip_proj_sync_host before such an entry when the
                                     same host arrays go on. Single-device contexts. */
    int dirty_sync_interval;      /* resident mode: full download every N-th step (0 = only
                                     on hip_proj_sync_host / failure) */
    int cg_variant;               /* 0 = textbook CG, the reference's loop (linear_solver_cg.c:
                                     367-439; default); 1 = Chronopoulos-Gear CG: both dot
                                     products of an iteration in ONE reduction (one
                                     all-reduce per iteration on Z-slabs), same stopping rule
                                     and stats, iterates equal to rounding only */
    int dirty_verify_interval;    /* resident mode guard: every N-th resident step first
                                     checks that the caller left the interior of its host
                                     arrays (every cell but the outer layer) as the last
                                     step did (64-bit position-weighted hashes: per N
                                     steps, two multithreaded host passes at the checked
                                     step and one over the layer next to the boundary
                                     after the step before it). A changed interior fails
                                     the checked step with CFD_ERROR_INVALID before
                                     anything runs; the device state is kept. With N > 1
                                     a write is found up to N-1 steps after it was made,
                                     and those steps have run on the device's state.
                                     0 = off (default). */
} hip_proj_config_t;

typedef struct hip_proj_ctx hip_proj_ctx_t;

/* Which device array a helper addresses. */
typedef enum {
    HIP_FIELD_U = 0,
    HIP_FIELD_V = 1,
    HIP_FIELD_W = 2,
    HIP_FIELD_P = 3,
    HIP_FIELD_T = 4,
    HIP_FIELD_RHO = 5  /* per-cell density (read by RK4; the projection uses rho[0]) */
} hip_field_id_t;

/* Per-kernel timing (filled when profiling is enabled). */
typedef enum {
    HIP_KT_PREDICTOR = 0,
    HIP_KT_CG_SETUP = 1,
    HIP_KT_CG_SWEEP_A = 2, /* p = r + beta p, Ap on the fly, (p,Ap) */
    HIP_KT_CG_SWEEP_B = 3, /* even iterations: r -= alpha A p (Ap recomputed), (r,r) */
    HIP_KT_CORRECTOR = 4,
    HIP_KT_RELAX = 5,      /* one RB-SOR colour pass or one Jacobi sweep */
    HIP_KT_RESIDUAL = 6,   /* L-infinity residual for the relaxation methods */
    HIP_KT_ENERGY = 7,     /* energy equation (alpha > 0) */
    HIP_KT_RK_STAGE = 8,   /* one fused RK4 stage (RHS + stage update) */
    HIP_KT_CG_SWEEP_BX = 9,/* every 4th iteration: sweep A + x += alpha p of the previous 4 */
    HIP_KT_CC_UPDATE = 10, /* cg_variant 1: p, s, r (and the x fold) update */
    HIP_KT_CC_SPMV = 11,   /* cg_variant 1: w = A r + (r,r), (w,r) */
    HIP_KT_HALO = 12,      /* Z-slabs: CG halo exchange (span on its stream) */
    HIP_KT_ALLREDUCE = 13, /* Z-slabs: RCCL all-reduce of a CG dot (+ finish kernel); the
                              device-mailbox reduction runs inside the sweep instead */
    HIP_KT_CG_SMALL = 14,  /* small grids: the whole CG solve in one cooperative launch */
    HIP_KT_RELAX2 = 15,    /* RB-SOR: one sweep of TWO iterations (k_rb2, one device, 3-D) */
    HIP_KT_CC_FUSED = 16,  /* cg_variant 1: the whole iteration in one z-march (k_ccf, one
                              device, 3-D); the first and the plain launches (version 3) */
    HIP_KT_CC_FOLD = 17,   /* cg_variant 1: the k_ccf launches that also fold x (every 4th) */
    HIP_KT_COUNT = 18
} hip_kernel_timer_t;

CFD_HIP_EXPORT hip_proj_config_t hip_proj_config_default(void);

/* 1 if a HIP device is usable, else 0 (role of gpu_is_available). */
CFD_HIP_EXPORT int hip_projection_available(void);

/* Create a context for an nx*ny*nz grid (nz == 1: 2D). Returns NULL and sets
 * the thread-local error on failure. */
CFD_HIP_EXPORT hip_proj_ctx_t* hip_proj_create(size_t nx, size_t ny, size_t nz,
                                               const hip_proj_config_t* cfg);
CFD_HIP_EXPORT void hip_proj_destroy(hip_proj_ctx_t* ctx);

/* One projection step on caller-owned host buffers: upload u,v,w,p (and T),
 * run the step in HBM, download. Same contract as the reference `projection`
 * step: status codes, preserved caller boundary faces, stats. */
CFD_HIP_EXPORT cfd_status_t hip_proj_step(hip_proj_ctx_t* ctx, flow_field* field, const grid* g,
                                          const ns_solver_params_t* params,
                                          ns_solver_stats_t* stats);

/* Resident mode (cfg.dirty_faces): copy the whole of u, v, w, p (and T when
 * resident) to the caller's field, so that every host cell is current. A
 * no-op copy of the full fields otherwise. */
CFD_HIP_EXPORT cfd_status_t hip_proj_sync_host(hip_proj_ctx_t* ctx, flow_field* field);

/* Resident mode: the caller declares that its host arrays hold the state to
 * use (it re-initialised them, restored a checkpoint into them, or wrote
 * interior cells after hip_proj_sync_host); the next host-buffer step uploads
 * them in full. */
CFD_HIP_EXPORT cfd_status_t hip_proj_mark_host_dirty(hip_proj_ctx_t* ctx);

/* Device-resident path. */
CFD_HIP_EXPORT cfd_status_t hip_proj_upload(hip_proj_ctx_t* ctx, const flow_field* field);
CFD_HIP_EXPORT cfd_status_t hip_proj_download(hip_proj_ctx_t* ctx, flow_field* field);
CFD_HIP_EXPORT cfd_status_t hip_proj_step_device(hip_proj_ctx_t* ctx, const grid* g,
                                                 const ns_solver_params_t* params,
                                                 ns_solver_stats_t* stats);
/* Copy one device field (unpadded, nx*ny*nz doubles) to / from host memory. */
CFD_HIP_EXPORT cfd_status_t hip_proj_get_field(hip_proj_ctx_t* ctx, int field_id, double* host);
CFD_HIP_EXPORT cfd_status_t hip_proj_set_field(hip_proj_ctx_t* ctx, int field_id,
                                               const double* host);
/* Fill a device field with a constant. */
CFD_HIP_EXPORT cfd_status_t hip_proj_fill_field(hip_proj_ctx_t* ctx, int field_id, double value);
/* Density used by the step (the reference reads field->rho[0] only). */
CFD_HIP_EXPORT cfd_status_t hip_proj_set_density(hip_proj_ctx_t* ctx, double rho0);

/* Caller-side boundary conditions applied on the device between steps (what
 * the reference drivers do on the host with bc_apply_scalar_3d /
 * bc_apply_dirichlet_velocity_3d, boundary_conditions.h:1222-1255). */
CFD_HIP_EXPORT cfd_status_t hip_proj_apply_scalar_bc(hip_proj_ctx_t* ctx, int field_id,
                                                     bc_type_t type);
CFD_HIP_EXPORT cfd_status_t hip_proj_apply_dirichlet(hip_proj_ctx_t* ctx, int field_id,
                                                     const bc_dirichlet_values_t* values);

/* energy_apply_thermal_bcs (energy_solver.c:204-334) on the device T with
 * params->thermal_bc; a no-op when params->alpha <= 0, as in the reference. */
CFD_HIP_EXPORT cfd_status_t hip_proj_apply_thermal_bcs(hip_proj_ctx_t* ctx,
                                                       const ns_solver_params_t* params);

/* Pressure-solver statistics of the most recent step. */
CFD_HIP_EXPORT cfd_status_t hip_proj_get_poisson_stats(hip_proj_ctx_t* ctx,
                                                       poisson_solver_stats_t* stats);

/* Kernel timing with HIP events on the context's stream. */
CFD_HIP_EXPORT void hip_proj_enable_timing(hip_proj_ctx_t* ctx, int enable);
CFD_HIP_EXPORT void hip_proj_reset_timing(hip_proj_ctx_t* ctx);
/* total_ms[k] and launches[k] for k < min(capacity, HIP_KT_COUNT); returns the
 * number of entries written (arrays may be NULL). Callers size their arrays
 * with the HIP_KT_COUNT of the header they were built against. */
CFD_HIP_EXPORT int hip_proj_get_timing_n(hip_proj_ctx_t* ctx, double* total_ms,
                                         long long* launches, int capacity);
/* Legacy getter without a capacity: writes the first HIP_KT_COUNT_LEGACY (17)
 * entries, the count of the last header that shipped it as the only getter
 * (ABI version 1, round 4), so a caller built against that header gets every
 * entry it sized its arrays for. Use hip_proj_get_timing_n. */
#define HIP_KT_COUNT_LEGACY 17
CFD_HIP_EXPORT void hip_proj_get_timing(hip_proj_ctx_t* ctx, double* total_ms, long long* launches);

/* Effective shader clock of the single-reduction march (k_ccf) while timing is
 * enabled: every workgroup of a sampled launch (two in eight: CG iterations
 * 5 and 7 mod 8, a plain and an x-fold launch) stamps
 * s_memtime (shader cycles) and s_memrealtime (the 100 MHz constant clock) at
 * its start and end; *mhz = 100 * sum(d memtime) / sum(d memrealtime) over
 * those workgroups, *workgroups = how many stamped. Reset by
 * hip_proj_reset_timing. 0 and *mhz = 0 when nothing was sampled. */
CFD_HIP_EXPORT cfd_status_t hip_proj_get_clock_sample(hip_proj_ctx_t* ctx, double* mhz,
                                                      long long* workgroups);
/* Placement draws of a large single-reduction context (3-D, >= 2^24 cells; a
 * Z-slab rank probes its own fields as one device, nothing collective): at creation its seven CG fields are allocated 6 times
 * (CFD_HIP_PLACEMENT_DRAWS) and 40 assignments of those buffers to the seven
 * roles (CFD_HIP_PLACEMENT_TRIALS: the 6 sets, then random ones) are timed on a
 * short probe solve; the fastest is kept. Writes each draw's probe time (ms per CG iteration) into
 * ms_per_iter[0 .. min(capacity, count) - 1] and the kept draw's index into
 * *picked (-1: no draws); returns the number of draws. */
CFD_HIP_EXPORT int hip_proj_get_placement(hip_proj_ctx_t* ctx, double* ms_per_iter, int capacity,
                                          int* picked);

/* ABI version of this header (bumped when a struct layout, an enum's count or
 * a signature changes) and of the loaded library: a caller checks
 * hip_proj_abi_version() == HIP_PROJ_ABI_VERSION. Version 2: HIP_KT_COUNT 17,
 * hip_proj_get_timing_n, projection_hip_cg1. Version 3: HIP_KT_COUNT 18
 * (HIP_KT_CC_FOLD split from HIP_KT_CC_FUSED), hip_proj_get_clock_sample,
 * hip_proj_get_placement, hip_proj_comm_mailbox_bench; the legacy getter
 * writes 17 entries. */
#define HIP_PROJ_ABI_VERSION 3
CFD_HIP_EXPORT int hip_proj_abi_version(void);
/* sha256 prefix (16 hex digits) of the sources the library was built from
 * (cfd_amd/_sha.py: csrc/hip, csrc/host, include/cfd_hip), embedded at
 * build time; the Python loader refuses a library whose id differs from the
 * sources beside it. */
CFD_HIP_EXPORT const char* hip_proj_build_id(void);

CFD_HIP_EXPORT cfd_status_t hip_proj_synchronize(hip_proj_ctx_t* ctx);
/* Bytes of device memory held by the context. */
CFD_HIP_EXPORT size_t hip_proj_device_bytes(const hip_proj_ctx_t* ctx);
/* Row pitch (in doubles) of the padded device layout. */
CFD_HIP_EXPORT size_t hip_proj_row_pitch(const hip_proj_ctx_t* ctx);

/* Standalone fixed-iteration CG microbenchmark on the context's buffers:
 * solves lap(x) = rhs (rhs given on host, x0 = 0) for exactly `iters`
 * iterations with no early exit. Returns elapsed device ms (events). */
CFD_HIP_EXPORT double hip_proj_cg_fixed_iters(hip_proj_ctx_t* ctx, const double* rhs_host,
                                              double dx, double dy, double dz, int iters);
/* The same with the right-hand side of the most recent step: rhs_host == NULL
 * solves with rhs = rho_over_dt * div u* of the context's predictor output
 * (the RHS the step's CG setup forms, solver_projection.c:195-214), x0 = 0;
 * rhs_host != NULL is hip_proj_cg_fixed_iters. The context's cg_variant
 * selects the CG form. SURVEY.md §8d config 3's fixed-200-iteration run. */
CFD_HIP_EXPORT double hip_proj_cg_fixed_iters_ex(hip_proj_ctx_t* ctx, const double* rhs_host,
                                                 double dx, double dy, double dz, int iters,
                                                 double rho_over_dt);

/* Restart files of the device-resident state, in the reference's .cfdchk
 * format (cfd_checkpoint_write / cfd_checkpoint_read, lib/include/cfd/io/
 * checkpoint.h:49-115; same argument meaning, status codes and string-buffer
 * rules). Fields stream between HBM and the file through pinned staging and
 * their CRC-32 is computed on the GPU. write: g must match the context's
 * dimensions; the fields written are the context's u, v, w, p, rho (rho0
 * everywhere when no per-cell density was set), T (zeros when absent).
 * read: the file's dimensions must equal the context's (CFD_ERROR_INVALID
 * otherwise); the state is replaced only after the trailing CRC matched;
 * *out_grid (may be NULL) receives a newly allocated grid, freed with
 * grid_destroy. Single-device contexts only (Z-slab: CFD_ERROR_UNSUPPORTED). */
CFD_HIP_EXPORT cfd_status_t hip_proj_checkpoint_write(hip_proj_ctx_t* ctx, const char* path,
                                                      const grid* g,
                                                      const ns_solver_params_t* params,
                                                      double current_time,
                                                      const char* solver_name,
                                                      const char* run_prefix,
                                                      const char* output_base_dir);
CFD_HIP_EXPORT cfd_status_t hip_proj_checkpoint_read(hip_proj_ctx_t* ctx, const char* path,
                                                     grid** out_grid,
                                                     ns_solver_params_t* out_params,
                                                     double* out_current_time,
                                                     char* out_solver_name,
                                                     size_t solver_name_cap,
                                                     char* out_run_prefix, size_t run_prefix_cap,
                                                     char* out_output_base_dir,
                                                     size_t output_base_dir_cap);
/* IEEE CRC-32 (zlib's) of one device field in the packed reference layout
 * (idx = k*nx*ny + j*nx + i, little-endian doubles), computed on the GPU. */
CFD_HIP_EXPORT cfd_status_t hip_proj_field_crc32(hip_proj_ctx_t* ctx, int field_id,
                                                 uint32_t* crc);

/* Measurement helper (not a reference interface): BabelStream-style copy and
 * triad over fp64 arrays of n elements with 16-B lanes on `device`; best of
 * `reps` timed rounds, in GB/s (BabelStream byte counts). The measured HBM roof
 * bench.py reports beside the 8 TB/s spec. */
CFD_HIP_EXPORT cfd_status_t cfd_hip_stream_bench(int device, size_t n, int reps,
                                                 double* copy_gbps, double* triad_gbps);
/* Measurement helper (not a reference interface): `ni` streamed fp64 inputs
 * and `no` streamed outputs of n elements (pairs built: 1/1, 2/1, 3/1, 2/2,
 * 3/3, 4/3, 4/4, 5/3; others CFD_ERROR_INVALID), best of `reps` rounds, in GB/s
 * of (ni + no) x 8 B per element: the achievable rate of a kernel with that
 * stream mix (the predictor 3/3, the corrector 4/3, the CG sweeps 2/1). */
CFD_HIP_EXPORT cfd_status_t cfd_hip_stream_bench_nm(int device, size_t n, int ni, int no,
                                                    int reps, double* gbps);

/* VTK output of the resident state (vtk_output.c:196-275, write_vtk_flow_field
 * text): velocity, pressure, density (the resident per-cell rho, else rho0),
 * temperature (the resident T, else 0). Single-device contexts; g must match. */
CFD_HIP_EXPORT cfd_status_t hip_proj_write_vtk(hip_proj_ctx_t* ctx, const char* filename,
                                               const grid* g, double rho0);

/* Standalone pressure-Poisson solve on host buffers, the HIP counterpart of
 * poisson_solver_solve with a POISSON_BACKEND_GPU solver (linear_solver.c:487-509,
 * poisson_solver_cg_gpu.cu:135-178): upload x and rhs, solve lap(x) = rhs with
 * the method given (CG / RB-SOR / Jacobi; Neumann BCs as the reference's default
 * apply_bc), download x. params == NULL uses poisson_solver_params_default()
 * (Jacobi: max_iterations 2000, linear_solver.c:274-276). */
CFD_HIP_EXPORT cfd_status_t hip_proj_poisson_solve(hip_proj_ctx_t* ctx, int method, double* x,
                                                   const double* rhs, double dx, double dy,
                                                   double dz,
                                                   const poisson_solver_params_t* params,
                                                   poisson_solver_stats_t* stats);

/* Boundary handling of hip_proj_poisson_solve_ex. The reference solvers call
 * poisson_solver_apply_bc (linear_solver.c:348-392): the caller's
 * solver->apply_bc when set (test_poisson_3d.c:274), else Neumann.
 *   NEUMANN  the default apply_bc, on the device (what hip_proj_poisson_solve does);
 *   NONE     boundary cells of x are never written on the device: CG only
 *            reads them (linear_solver_cg.c applies the BC at :320 and :447,
 *            which the caller then runs on the host around the solve), and
 *            relaxation iterations keep x's own boundary;
 *   FIXED    after every relaxation iteration (linear_solver_redblack.c:139,
 *            linear_solver_jacobi.c:118) the boundary shell of x is set from
 *            bc_values (nx*ny*nz host doubles, only the shell read): an
 *            apply_bc that writes x-independent values, e.g. Dirichlet. */
typedef enum {
    HIP_POISSON_BC_NEUMANN = 0,
    HIP_POISSON_BC_NONE = 1,
    HIP_POISSON_BC_FIXED = 2
} hip_poisson_bc_t;

CFD_HIP_EXPORT cfd_status_t hip_proj_poisson_solve_ex(hip_proj_ctx_t* ctx, int method, double* x,
                                                      const double* rhs, double dx, double dy,
                                                      double dz,
                                                      const poisson_solver_params_t* params,
                                                      poisson_solver_stats_t* stats, int bc_mode,
                                                      const double* bc_values);

/* ---- Z-slab multi-GPU ------------------------------------------------------
 * The reference runs one device per simulation (solver_projection_gpu.cu has
 * no decomposition). Here the nz-2 interior planes of the
 * global grid are split into contiguous slabs, one per rank: rank r holds
 * nz_local = owned + 2 planes, local plane 0 being global plane k_offset.
 * The two outer local planes are the global z faces on the edge ranks and
 * halo copies of the neighbours' planes elsewhere. Every CG dot product is a
 * per-rank deterministic partial summed by an all-reduce; the textbook CG
 * iteration otherwise keeps its single-device semantics. Fields passed to
 * set_field/get_field/poisson_solve are the rank's nx*ny*nz_local slab; the
 * grid passed to step functions is the GLOBAL grid.
 *
 * Communicators: RCCL (one process per GPU; rank 0 creates the unique id, the
 * caller broadcasts its bytes, e.g. over torch.distributed) or an in-process
 * group whose ranks are slab contexts of one process, each driven from its
 * own host thread (all ranks call every step function concurrently). */
#define HIP_PROJ_UNIQUE_ID_BYTES 128
typedef struct hip_proj_comm hip_proj_comm_t;
typedef struct hip_proj_group hip_proj_group_t;

/* Split of nz (global points) for `rank` of `size`; host-only, no device. */
CFD_HIP_EXPORT cfd_status_t hip_proj_slab_layout(size_t nz, int rank, int size, size_t* k_offset,
                                                 size_t* nz_local);
CFD_HIP_EXPORT cfd_status_t hip_proj_comm_unique_id(unsigned char id[HIP_PROJ_UNIQUE_ID_BYTES]);
/* Collective over the `size` processes (ncclCommInitRank on `device`). */
CFD_HIP_EXPORT hip_proj_comm_t* hip_proj_comm_create_rccl(
    const unsigned char id[HIP_PROJ_UNIQUE_ID_BYTES], int rank, int size, int device);
CFD_HIP_EXPORT hip_proj_group_t* hip_proj_group_create(int size);
CFD_HIP_EXPORT void hip_proj_group_destroy(hip_proj_group_t* group);
CFD_HIP_EXPORT hip_proj_comm_t* hip_proj_comm_create_local(hip_proj_group_t* group, int rank,
                                                           int device);
CFD_HIP_EXPORT void hip_proj_comm_destroy(hip_proj_comm_t* comm);
CFD_HIP_EXPORT int hip_proj_comm_rank(const hip_proj_comm_t* comm);
CFD_HIP_EXPORT int hip_proj_comm_size(const hip_proj_comm_t* comm);
/* 1 when the CG dot products go through the one-shot peer-memory all-reduce
 * (RCCL communicators; verified at creation, CFD_HIP_DEVICE_ALLREDUCE=0 turns it
 * off), 0 when they use ncclAllReduce / the in-process group. */
CFD_HIP_EXPORT int hip_proj_comm_device_allreduce(const hip_proj_comm_t* comm);
/* Collective microbenchmark of the CG dot all-reduce of an RCCL communicator
 * (the N-rank per-iteration budget): `iters` two-value
 * all-reduces of rank-dependent values, timed with events on a stream of its
 * own. mode 0: all of them inside ONE one-wave kernel (the device mailbox's
 * round trip, mbox_allreduce2); mode 1: one one-wave kernel launch per
 * all-reduce (launch + mailbox, what a CG iteration pays); mode 2: one
 * 2-value ncclAllReduce per iteration (the fallback). *us = microseconds per
 * all-reduce; every rank checks the sums. CFD_ERROR_UNSUPPORTED for modes 0/1
 * without a mailbox or for an in-process group. */
CFD_HIP_EXPORT cfd_status_t hip_proj_comm_mailbox_bench(hip_proj_comm_t* comm, int iters,
                                                        int mode, double* us);
/* Slab context for rank comm_rank of the global nx*ny*nz grid (3-D only). The
 * communicator must outlive the context. */
CFD_HIP_EXPORT hip_proj_ctx_t* hip_proj_create_slab(size_t nx, size_t ny, size_t nz,
                                                    hip_proj_comm_t* comm,
                                                    const hip_proj_config_t* cfg);
CFD_HIP_EXPORT cfd_status_t hip_proj_slab_info(const hip_proj_ctx_t* ctx, size_t* k_offset,
                                               size_t* nz_local, int* rank, int* size);

/* ---- RK4 (solver_rk4.c:69-259) --------------------------------------------
 * Classical RK4 with the shared momentum RHS of ns_momentum_rhs_scalar.h:49-190
 * (periodic stencil indices, derivative clamps, pseudo-compressible pressure
 * update), energy equation after the update, periodic BCs on u,v,w,p,rho,T,
 * thermal BCs, NaN check: the reference `rk4` step on a context's fields. The
 * context needs HIP_FIELD_RHO (per-cell density) in addition to u,v,w,p (T when
 * beta != 0 or alpha > 0). Single device only. */
CFD_HIP_EXPORT cfd_status_t hip_rk4_step_device(hip_proj_ctx_t* ctx, const grid* g,
                                                const ns_solver_params_t* params,
                                                ns_solver_stats_t* stats);
/* Host-buffer step: upload u,v,w,p,rho(,T), one RK4 step, download. */
CFD_HIP_EXPORT cfd_status_t hip_rk4_step(hip_proj_ctx_t* ctx, flow_field* field, const grid* g,
                                         const ns_solver_params_t* params,
                                         ns_solver_stats_t* stats);

/* ---- plugin surface ------------------------------------------------------ */
CFD_HIP_EXPORT ns_solver_t* create_projection_hip_solver(void);
CFD_HIP_EXPORT ns_solver_t* create_projection_hip_rbsor_solver(void);
CFD_HIP_EXPORT ns_solver_t* create_projection_hip_jacobi_solver(void);
CFD_HIP_EXPORT ns_solver_t* create_projection_hip_cg1_solver(void);
CFD_HIP_EXPORT ns_solver_t* create_rk4_hip_solver(void);
/* poisson_solver_t GPU backend factories under the reference's names
 * (linear_solver_internal.h:54-57; reached via poisson_solver_create(method,
 * POISSON_BACKEND_GPU), linear_solver.c:150-235). Host-buffer semantics:
 * solve uploads x and rhs, iterates in HBM, downloads x. */
CFD_HIP_EXPORT poisson_solver_t* create_cg_gpu_solver(void);
CFD_HIP_EXPORT poisson_solver_t* create_redblack_gpu_solver(void);
CFD_HIP_EXPORT poisson_solver_t* create_jacobi_gpu_solver(void);
/* Registers the five names above through cfd_registry_register(). */
CFD_HIP_EXPORT void cfd_hip_register_solvers(ns_solver_registry_t* registry);

#ifdef __cplusplus
}
#endif

#endif /* CFD_HIP_PROJECTION_HIP_H */
