// bc_gpu.hip -- the reference's device-pointer BC entry points
// (boundary_conditions_gpu.cuh:32-151, impl boundary/gpu/boundary_conditions_gpu.cu)
// on caller-owned packed arrays: one k_bc_shell launch (pure gathers from
// interior cells, kernels.hpp) per field on the caller's stream.
#include "ctx.hpp"

#include "cfd_hip/boundary_conditions_gpu.h"

namespace {

Geo packed_geo(size_t nx, size_t ny, size_t nz) {
    Geo g{};
    g.nx = (int)nx;
    g.ny = (int)ny;
    g.nz = (int)nz;
    g.px = (long long)nx;
    g.ps = (long long)nx * (long long)ny;
    g.sz = nz > 1 ? g.ps : 0;
    g.k0 = nz > 1 ? 1 : 0;
    g.k1 = nz > 1 ? (int)nz - 1 : 1;
    g.lo_face = g.hi_face = 1;
    return g;
}

void shell(double* f, const Geo& g, int mode, const DirVals& dv, void* stream) {
    const long long ring = 2LL * g.nx + 2LL * (g.ny - 2);
    const long long total = ring * g.nz + (g.nz > 1 ? 2LL * g.nx * g.ny : 0);
    const unsigned blocks = (unsigned)std::max(1LL, std::min((total + 255) / 256, 65535LL));
    hipLaunchKernelGGL(k_bc_shell, dim3(blocks), dim3(256), 0, (hipStream_t)stream, g, f, mode,
                       dv);
}

// bc_type_t -> k_bc_shell mode; the reference's device switch treats every
// type other than PERIODIC as NEUMANN (boundary_conditions_gpu.cu:477-526)
int mode_of(bc_type_t t) { return t == BC_TYPE_PERIODIC ? 1 : 0; }

DirVals dirvals(const bc_dirichlet_values_t* v) {
    DirVals d{};
    d.left = v->left;
    d.right = v->right;
    d.top = v->top;
    d.bottom = v->bottom;
    d.front = v->front;
    d.back = v->back;
    return d;
}

}  // namespace

extern "C" {

void bc_apply_scalar_gpu(double* d_field, size_t nx, size_t ny, bc_type_t type, void* stream) {
    if (!d_field || nx < 3 || ny < 3) return;
    shell(d_field, packed_geo(nx, ny, 1), mode_of(type), DirVals{}, stream);
}

void bc_apply_neumann_gpu(double* d_field, size_t nx, size_t ny, void* stream) {
    bc_apply_scalar_gpu(d_field, nx, ny, BC_TYPE_NEUMANN, stream);
}

void bc_apply_velocity_gpu(double* d_u, double* d_v, size_t nx, size_t ny, bc_type_t type,
                           void* stream) {
    if (!d_u || !d_v || nx < 3 || ny < 3) return;
    const Geo g = packed_geo(nx, ny, 1);
    shell(d_u, g, mode_of(type), DirVals{}, stream);
    shell(d_v, g, mode_of(type), DirVals{}, stream);
}

void bc_apply_dirichlet_scalar_gpu(double* d_field, size_t nx, size_t ny,
                                   const bc_dirichlet_values_t* values, void* stream) {
    if (!d_field || !values || nx < 3 || ny < 3) return;
    shell(d_field, packed_geo(nx, ny, 1), 2, dirvals(values), stream);
}

void bc_apply_dirichlet_velocity_gpu(double* d_u, double* d_v, size_t nx, size_t ny,
                                     const bc_dirichlet_values_t* u_values,
                                     const bc_dirichlet_values_t* v_values, void* stream) {
    if (!d_u || !d_v || !u_values || !v_values || nx < 3 || ny < 3) return;
    const Geo g = packed_geo(nx, ny, 1);
    shell(d_u, g, 2, dirvals(u_values), stream);
    shell(d_v, g, 2, dirvals(v_values), stream);
}

void bc_apply_scalar_3d_gpu(double* d_field, size_t nx, size_t ny, size_t nz, bc_type_t type,
                            void* stream) {
    if (!d_field || nx < 3 || ny < 3) return;
    if (nz == 1) return bc_apply_scalar_gpu(d_field, nx, ny, type, stream);
    if (nz < 3) return;
    shell(d_field, packed_geo(nx, ny, nz), mode_of(type), DirVals{}, stream);
}

void bc_apply_velocity_3d_gpu(double* d_u, double* d_v, double* d_w, size_t nx, size_t ny,
                              size_t nz, bc_type_t type, void* stream) {
    if (!d_u || !d_v || nx < 3 || ny < 3) return;
    if (nz == 1) return bc_apply_velocity_gpu(d_u, d_v, nx, ny, type, stream);
    if (nz < 3) return;
    const Geo g = packed_geo(nx, ny, nz);
    shell(d_u, g, mode_of(type), DirVals{}, stream);
    shell(d_v, g, mode_of(type), DirVals{}, stream);
    if (d_w) shell(d_w, g, mode_of(type), DirVals{}, stream);
}

}  // extern "C"
