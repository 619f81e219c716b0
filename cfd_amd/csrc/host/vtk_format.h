/*
 * vtk_format.h -- legacy ASCII VTK (STRUCTURED_POINTS) text of the reference's
 * writers (lib/src/io/vtk_output.c:110-275), shared by the host mirror
 * (write_vtk_output / write_vtk_vector_output / write_vtk_flow_field in
 * libcfd_host.so) and the device-state writer of libcfd_hip.so
 * (hip_proj_write_vtk). Same header lines, "%f" values, k-j-i order.
 * Arrays are packed reference layout (k*nx*ny + j*nx + i).
 */
#ifndef CFD_HIP_VTK_FORMAT_H
#define CFD_HIP_VTK_FORMAT_H

#include <stddef.h>
#include <stdio.h>

/* vtk_output.c:112-115 (argument checks shared by the three writers) */
static inline int vtk_grid_ok(size_t nx, size_t ny, size_t nz, double xmin, double xmax,
                              double ymin, double ymax, double zmin, double zmax) {
    return !(nx < 2 || ny < 2 || nz < 1 || xmax <= xmin || ymax <= ymin ||
             (nz > 1 && zmax <= zmin));
}

static inline void vtk_header(FILE* fp, const char* title, size_t nx, size_t ny, size_t nz,
                              double xmin, double xmax, double ymin, double ymax, double zmin,
                              double zmax) {
    double dz = (nz > 1) ? (zmax - zmin) / (double)(nz - 1) : 1.0;
    fprintf(fp, "# vtk DataFile Version 3.0\n");
    fprintf(fp, "%s\n", title);
    fprintf(fp, "ASCII\n");
    fprintf(fp, "DATASET STRUCTURED_POINTS\n");
    fprintf(fp, "DIMENSIONS %zu %zu %zu\n", nx, ny, nz);
    fprintf(fp, "ORIGIN %f %f %f\n", xmin, ymin, zmin);
    fprintf(fp, "SPACING %f %f %f\n", (xmax - xmin) / (nx - 1), (ymax - ymin) / (ny - 1), dz);
}

static inline void vtk_scalars(FILE* fp, const char* name, const double* d, size_t n) {
    fprintf(fp, "SCALARS %s float 1\n", name);
    fprintf(fp, "LOOKUP_TABLE default\n");
    for (size_t q = 0; q < n; q++) fprintf(fp, "%f\n", d[q]);
}

static inline void vtk_vectors(FILE* fp, const char* name, const double* u, const double* v,
                               const double* w, size_t n) {
    fprintf(fp, "VECTORS %s float\n", name);
    for (size_t q = 0; q < n; q++) fprintf(fp, "%f %f %f\n", u[q], v[q], w ? w[q] : 0.0);
}

/* write_vtk_flow_field (vtk_output.c:196-275): velocity, pressure, density,
 * temperature. Returns 0 on success, -1 when the file cannot be opened. */
static inline int vtk_write_flow_field_file(const char* filename, const double* u,
                                            const double* v, const double* w, const double* p,
                                            const double* rho, const double* T, size_t nx,
                                            size_t ny, size_t nz, double xmin, double xmax,
                                            double ymin, double ymax, double zmin, double zmax) {
    FILE* fp = fopen(filename, "w");
    if (!fp) return -1;
    const size_t n = nx * ny * nz;
    vtk_header(fp, "CFD Framework Flow Field Output", nx, ny, nz, xmin, xmax, ymin, ymax, zmin,
               zmax);
    fprintf(fp, "\nPOINT_DATA %zu\n", n);
    vtk_vectors(fp, "velocity", u, v, w, n);
    fprintf(fp, "\n");
    vtk_scalars(fp, "pressure", p, n);
    fprintf(fp, "\n");
    vtk_scalars(fp, "density", rho, n);
    fprintf(fp, "\n");
    vtk_scalars(fp, "temperature", T, n);
    fclose(fp);
    return 0;
}

#endif /* CFD_HIP_VTK_FORMAT_H */
