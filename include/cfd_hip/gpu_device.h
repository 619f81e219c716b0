/*
 * gpu_device.h -- the reference's device API (lib/include/cfd/core/gpu_device.h)
 * served by the MI355X library (libcfd_hip.so).
 *
 * Same names, same struct layouts, same argument meaning and error behaviour
 * as the reference, so a program written against the reference's
 * `cfd/core/gpu_device.h` links against libcfd_hip.so unchanged:
 *
 *   gpu_config_default / gpu_is_available / gpu_get_device_info /
 *   gpu_select_device / gpu_should_use          gpu_device.h:91-129
 *                                               (impl solver_projection_gpu.cu:294-373)
 *   gpu_solver_create / destroy / upload /
 *   download / step / get_stats / reset_stats    gpu_device.h:135-194
 *                                               (impl solver_projection_gpu.cu:375-588)
 *   solve_navier_stokes_gpu / solve_projection_method_gpu /
 *   solve_rk4_method_gpu                         gpu_device.h:200-247
 *                                               (impl solver_projection_gpu.cu:590-770,
 *                                                solver_rk_gpu.cu)
 *
 * The context here is a persistent HBM-resident hip_proj context (fields in
 * the padded SoA layout of DESIGN.md §2); `gpu_solver_step` runs the
 * reference's explicit pressure-relaxation step (solver_projection_gpu.cu:523-570)
 * as two fused HIP sweeps + boundary gathers, and `solve_projection_method_gpu`
 * runs the Chorin projection of projection_hip with the reference GPU's
 * solver settings (see the function comment). solve_rk2_method_gpu is not
 * provided (RK2 is outside the projection path).
 */
#ifndef CFD_HIP_GPU_DEVICE_H
#define CFD_HIP_GPU_DEVICE_H

#include "cfd_hip/cfd_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* gpu_device.h:32-53 */
typedef struct {
    int enable_gpu;
    size_t min_grid_size;
    int min_steps;
    int block_size_x;          /* accepted for ABI compatibility; the HIP kernels pick */
    int block_size_y;          /* their own gfx950 tiling */
    int poisson_max_iter;
    double poisson_tolerance;
    int persistent_memory;
    int async_transfers;
    int sync_after_kernel;
    int verbose;
} gpu_config_t;

/* gpu_device.h:58-69 */
typedef struct {
    int device_id;
    char name[256];
    size_t total_memory;
    size_t free_memory;
    int compute_capability_major;  /* gfx950: 9 */
    int compute_capability_minor;  /* gfx950: 5 */
    int multiprocessor_count;      /* compute units */
    int max_threads_per_block;
    int warp_size;                 /* 64 (wavefront) */
    int is_available;
} gpu_device_info_t;

/* gpu_device.h:74-82 */
typedef struct {
    double kernel_time_ms;
    double transfer_time_ms;
    double poisson_time_ms;
    int poisson_iterations;
    double poisson_residual;
    size_t memory_allocated;
    int kernels_launched;
} gpu_solver_stats_t;

typedef struct gpu_solver_context_t gpu_solver_context_t;

CFD_HIP_EXPORT gpu_config_t gpu_config_default(void);
CFD_HIP_EXPORT int gpu_is_available(void);
CFD_HIP_EXPORT int gpu_get_device_info(gpu_device_info_t* info, int max_devices);
CFD_HIP_EXPORT cfd_status_t gpu_select_device(int device_id);
CFD_HIP_EXPORT int gpu_should_use(const gpu_config_t* config, size_t nx, size_t ny, size_t nz,
                                  int num_steps);

CFD_HIP_EXPORT gpu_solver_context_t* gpu_solver_create(size_t nx, size_t ny, size_t nz,
                                                       const gpu_config_t* config);
CFD_HIP_EXPORT void gpu_solver_destroy(gpu_solver_context_t* ctx);
CFD_HIP_EXPORT cfd_status_t gpu_solver_upload(gpu_solver_context_t* ctx, const flow_field* field);
CFD_HIP_EXPORT cfd_status_t gpu_solver_download(gpu_solver_context_t* ctx, flow_field* field);
CFD_HIP_EXPORT cfd_status_t gpu_solver_step(gpu_solver_context_t* ctx, const grid* grid,
                                            const ns_solver_params_t* params,
                                            gpu_solver_stats_t* stats);
CFD_HIP_EXPORT gpu_solver_stats_t gpu_solver_get_stats(const gpu_solver_context_t* ctx);
CFD_HIP_EXPORT void gpu_solver_reset_stats(gpu_solver_context_t* ctx);

/* solver_projection_gpu.cu:590-612: params->max_iter explicit steps. */
CFD_HIP_EXPORT cfd_status_t solve_navier_stokes_gpu(flow_field* field, const grid* grid,
                                                    const ns_solver_params_t* params,
                                                    const gpu_config_t* config);
/* solver_projection_gpu.cu:617-770: params->max_iter Chorin projection steps
 * in HBM with the reference GPU's settings: Poisson CG to
 * config->poisson_tolerance (relative, absolute 0) capped at
 * config->poisson_max_iter with a capped solve non-fatal, RHS div(u*)/dt,
 * no default source term; boundary faces are the caller's. */
CFD_HIP_EXPORT cfd_status_t solve_projection_method_gpu(flow_field* field, const grid* grid,
                                                        const ns_solver_params_t* params,
                                                        const gpu_config_t* config);
/* solver_rk_gpu.cu (solve_rk4_method_gpu): params->max_iter RK4 steps. */
CFD_HIP_EXPORT cfd_status_t solve_rk4_method_gpu(flow_field* field, const grid* grid,
                                                 const ns_solver_params_t* params,
                                                 const gpu_config_t* config);
/* solver_rk_gpu.cu:535-545 integrators outside the projection path: they
 * return CFD_ERROR_UNSUPPORTED. Exported so that libcfd_hip.so defines every
 * symbol of the reference's no-CUDA stub (solver_gpu_stub.c:15-161): a link
 * that names libcfd_hip.so before libcfd_core.a then never pulls the stub's
 * object in. */
CFD_HIP_EXPORT cfd_status_t solve_explicit_euler_method_gpu(flow_field* field, const grid* grid,
                                                            const ns_solver_params_t* params,
                                                            const gpu_config_t* config);
CFD_HIP_EXPORT cfd_status_t solve_rk2_method_gpu(flow_field* field, const grid* grid,
                                                 const ns_solver_params_t* params,
                                                 const gpu_config_t* config);

#ifdef __cplusplus
}
#endif

#endif /* CFD_HIP_GPU_DEVICE_H */
