/*
 * boundary_conditions_gpu.h -- the reference's device-pointer boundary
 * conditions (lib/include/cfd/boundary/boundary_conditions_gpu.cuh:32-151)
 * served by libcfd_hip.so for device arrays in the reference's packed layout
 * (idx = k*nx*ny + j*nx + i).
 *
 * `stream` is the caller's HIP stream handle passed as an opaque pointer (the
 * reference takes a cudaStream_t; NULL = the default stream). The kernels are
 * gathers from interior cells (race-free), so every face, edge and corner gets
 * the value of the host reference's sequential x -> y -> z face order
 * (boundary_conditions_core_impl.h:41-186); the reference's device kernels
 * write all faces in one launch and leave edge cells to the race.
 * bc_apply_inlet_gpu is not provided (inlet profiles are outside the
 * projection path).
 */
#ifndef CFD_HIP_BOUNDARY_CONDITIONS_GPU_H
#define CFD_HIP_BOUNDARY_CONDITIONS_GPU_H

#include "cfd_hip/cfd_abi.h"

#ifdef __cplusplus
extern "C" {
#endif

CFD_HIP_EXPORT void bc_apply_neumann_gpu(double* d_field, size_t nx, size_t ny, void* stream);
CFD_HIP_EXPORT void bc_apply_scalar_gpu(double* d_field, size_t nx, size_t ny, bc_type_t type,
                                        void* stream);
CFD_HIP_EXPORT void bc_apply_velocity_gpu(double* d_u, double* d_v, size_t nx, size_t ny,
                                          bc_type_t type, void* stream);
CFD_HIP_EXPORT void bc_apply_dirichlet_scalar_gpu(double* d_field, size_t nx, size_t ny,
                                                  const bc_dirichlet_values_t* values,
                                                  void* stream);
CFD_HIP_EXPORT void bc_apply_dirichlet_velocity_gpu(double* d_u, double* d_v, size_t nx,
                                                    size_t ny,
                                                    const bc_dirichlet_values_t* u_values,
                                                    const bc_dirichlet_values_t* v_values,
                                                    void* stream);
CFD_HIP_EXPORT void bc_apply_scalar_3d_gpu(double* d_field, size_t nx, size_t ny, size_t nz,
                                           bc_type_t type, void* stream);
CFD_HIP_EXPORT void bc_apply_velocity_3d_gpu(double* d_u, double* d_v, double* d_w, size_t nx,
                                             size_t ny, size_t nz, bc_type_t type, void* stream);

#ifdef __cplusplus
}
#endif

#endif /* CFD_HIP_BOUNDARY_CONDITIONS_GPU_H */
