/*
 * vtk_hip_io.c -- VTK output of HBM-resident state:
 * the fields of a hip_proj context are downloaded into packed host arrays
 * and written as the reference's write_vtk_flow_field does
 * (lib/src/io/vtk_output.c:196-275), byte for byte.
 *
 * Density: the context keeps the per-cell rho only when RK4 uploaded it; the
 * projection reads rho[0] alone (solver_projection.c:195), so otherwise the
 * density written is that constant. Temperature: the resident T, or 0.0 when
 * the context holds none (the reference's flow_field always carries T).
 */
#include "cfd_hip/projection_hip.h"
#include "vtk_format.h"

#include <stdlib.h>

extern void cfd_set_error(cfd_status_t status, const char* message) __attribute__((weak));
__attribute__((visibility("hidden"))) int hip_proj_matches_internal(const hip_proj_ctx_t* ctx,
                                                                    size_t nx, size_t ny,
                                                                    size_t nz);

cfd_status_t hip_proj_write_vtk(hip_proj_ctx_t* ctx, const char* filename, const grid* g,
                                double rho0) {
    if (!ctx || !filename || !g) return CFD_ERROR_INVALID;
    const size_t nx = g->nx, ny = g->ny, nz = g->nz;
    if (!vtk_grid_ok(nx, ny, nz, g->xmin, g->xmax, g->ymin, g->ymax, g->zmin, g->zmax))
        return CFD_ERROR_INVALID;
    int rank = 0, size = 1;
    if (hip_proj_slab_info(ctx, NULL, NULL, &rank, &size) != CFD_SUCCESS || size != 1 ||
        !hip_proj_matches_internal(ctx, nx, ny, nz)) {
        if (cfd_set_error)
            cfd_set_error(CFD_ERROR_INVALID, "hip_proj_write_vtk: grid does not match the context "
                                             "(or the context is a Z-slab)");
        return CFD_ERROR_INVALID;
    }
    const size_t n = nx * ny * nz;
    double* buf = (double*)malloc(6 * n * sizeof(double));
    if (!buf) return CFD_ERROR_NOMEM;
    double *u = buf, *v = buf + n, *w = buf + 2 * n, *p = buf + 3 * n, *rho = buf + 4 * n,
           *T = buf + 5 * n;
    cfd_status_t s = CFD_SUCCESS;
    const int ids[4] = {HIP_FIELD_U, HIP_FIELD_V, HIP_FIELD_W, HIP_FIELD_P};
    double* dst[4] = {u, v, w, p};
    for (int q = 0; q < 4 && s == CFD_SUCCESS; q++) s = hip_proj_get_field(ctx, ids[q], dst[q]);
    if (s != CFD_SUCCESS) {
        free(buf);
        return s;
    }
    if (hip_proj_get_field(ctx, HIP_FIELD_RHO, rho) != CFD_SUCCESS)
        for (size_t q = 0; q < n; q++) rho[q] = rho0;
    if (hip_proj_get_field(ctx, HIP_FIELD_T, T) != CFD_SUCCESS)
        for (size_t q = 0; q < n; q++) T[q] = 0.0;
    if (vtk_write_flow_field_file(filename, u, v, w, p, rho, T, nx, ny, nz, g->xmin, g->xmax,
                                  g->ymin, g->ymax, g->zmin, g->zmax) != 0) {
        if (cfd_set_error) cfd_set_error(CFD_ERROR_IO, "Failed to open VTK flow field output file");
        s = CFD_ERROR_IO;
    }
    free(buf);
    return s;
}
