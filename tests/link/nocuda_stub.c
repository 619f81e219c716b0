/*
 * Test fixture: a from-scratch restatement of the reference's no-CUDA stub
 * object (lib/src/solvers/gpu/solver_gpu_stub.c:15-161), which the reference
 * always compiles into libcfd_core.a (lib/CMakeLists.txt:182-185,247-251).
 * Same symbol set, same "no GPU" answers; built into a static archive by
 * tests/test_reference_link.py to show which definition a link picks.
 */
#include <string.h>

#include "cfd_hip/cfd_abi.h"
#include "cfd_hip/gpu_device.h"

static cfd_status_t unsupported(void) { return CFD_ERROR_UNSUPPORTED; }

gpu_config_t gpu_config_default(void) {
    gpu_config_t c;
    memset(&c, 0, sizeof(c));
    c.enable_gpu = 0; /* the stub's marker: the HIP library answers 1 */
    c.min_grid_size = 10000;
    c.min_steps = 10;
    c.block_size_x = c.block_size_y = 16;
    c.poisson_max_iter = 1000;
    c.poisson_tolerance = 1e-3;
    c.persistent_memory = c.async_transfers = 1;
    return c;
}
int gpu_is_available(void) { return 0; }
int gpu_get_device_info(gpu_device_info_t* info, int n) { (void)info; (void)n; return 0; }
cfd_status_t gpu_select_device(int id) { (void)id; return unsupported(); }
int gpu_should_use(const gpu_config_t* c, size_t nx, size_t ny, size_t nz, int s) {
    (void)c; (void)nx; (void)ny; (void)nz; (void)s;
    return 0;
}
gpu_solver_context_t* gpu_solver_create(size_t nx, size_t ny, size_t nz, const gpu_config_t* c) {
    (void)nx; (void)ny; (void)nz; (void)c;
    return NULL;
}
void gpu_solver_destroy(gpu_solver_context_t* ctx) { (void)ctx; }
cfd_status_t gpu_solver_upload(gpu_solver_context_t* ctx, const flow_field* f) {
    (void)ctx; (void)f;
    return unsupported();
}
cfd_status_t gpu_solver_download(gpu_solver_context_t* ctx, flow_field* f) {
    (void)ctx; (void)f;
    return unsupported();
}
cfd_status_t gpu_solver_step(gpu_solver_context_t* ctx, const grid* g, const ns_solver_params_t* p,
                             gpu_solver_stats_t* s) {
    (void)ctx; (void)g; (void)p; (void)s;
    return unsupported();
}
gpu_solver_stats_t gpu_solver_get_stats(const gpu_solver_context_t* ctx) {
    gpu_solver_stats_t s;
    (void)ctx;
    memset(&s, 0, sizeof(s));
    return s;
}
void gpu_solver_reset_stats(gpu_solver_context_t* ctx) { (void)ctx; }

#define STUB_SOLVE(name)                                                                    \
    cfd_status_t name(flow_field* f, const grid* g, const ns_solver_params_t* p,            \
                      const gpu_config_t* c) {                                              \
        (void)f; (void)g; (void)p; (void)c;                                                 \
        return unsupported();                                                               \
    }
STUB_SOLVE(solve_navier_stokes_gpu)
STUB_SOLVE(solve_projection_method_gpu)
STUB_SOLVE(solve_explicit_euler_method_gpu)
STUB_SOLVE(solve_rk2_method_gpu)
STUB_SOLVE(solve_rk4_method_gpu)
