/*
 * Test fixture standing in for the reference's solver_registry.o (an object
 * of libcfd_api.a): it references the GPU entry points the way the registry
 * does -- gpu_is_available() from cfd_backend_is_available
 * (solver_registry.c:1615-1616) and the solve_*_gpu drivers from the GPU
 * solver wrappers (:1121-1153, :1219-1245) -- and reports where they resolved.
 */
#include "cfd_hip/cfd_abi.h"
#include "cfd_hip/gpu_device.h"

int probe_backend_gpu_available(void) { return gpu_is_available(); }

void* probe_gpu_is_available(void) { return (void*)&gpu_is_available; }
void* probe_solve_projection_method_gpu(void) { return (void*)&solve_projection_method_gpu; }
void* probe_solve_rk4_method_gpu(void) { return (void*)&solve_rk4_method_gpu; }
int probe_config_enable_gpu(void) { return gpu_config_default().enable_gpu; }
