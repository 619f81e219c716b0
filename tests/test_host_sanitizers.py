"""The host-side C code (libcfd_host's sources and the oracle) built with
AddressSanitizer + UndefinedBehaviorSanitizer into a C driver that walks the
host API: grids and fields, every BC, the registry without a HIP library,
restart-file round trip and corrupt-file rejection, VTK writers, the Poisson
factory surface, and oracle projection / CG / RB-SOR / RK4 steps. Sanitizers
run on host code only (there is no GPU sanitizer on this pool)."""
import os
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
HOST = ROOT / "cfd_amd" / "csrc" / "host"

DRIVER = r"""
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include "cfd_hip/cfd_host.h"
#include "oracle.h"

#define CHECK(c) do { if (!(c)) { fprintf(stderr, "FAIL %s:%d %s\n", __FILE__, __LINE__, #c); return 1; } } while (0)

int main(int argc, char** argv) {
    const char* dir = argv[1];
    char path[1024];
    size_t nx = 17, ny = 13, nz = 9;
    grid* g = grid_create(nx, ny, nz, 0, 1, 0, 1, 0, 1);
    CHECK(g);
    grid_initialize_uniform(g);
    flow_field* f = flow_field_create(nx, ny, nz);
    CHECK(f);
    initialize_flow_field(f, g);
    for (int t = 0; t < 3; t++) {
        bc_type_t ty = t == 0 ? BC_TYPE_NEUMANN : (t == 1 ? BC_TYPE_PERIODIC : BC_TYPE_NEUMANN);
        CHECK(bc_apply_scalar_3d(f->p, nx, ny, nz, nx * ny, ty) == CFD_SUCCESS);
        CHECK(bc_apply_velocity_3d(f->u, f->v, f->w, nx, ny, nz, nx * ny, ty) == CFD_SUCCESS);
    }
    bc_dirichlet_values_t lid = {0, 0, 1.0, 0, 0, 0}, zero = {0, 0, 0, 0, 0, 0};
    CHECK(bc_apply_dirichlet_velocity_3d(f->u, f->v, f->w, nx, ny, nz, nx * ny, &lid, &zero,
                                         &zero) == CFD_SUCCESS);
    /* registry without libcfd_hip.so: no HIP solvers, NOT_FOUND */
    ns_solver_registry_t* reg = cfd_registry_create();
    CHECK(reg);
    cfd_registry_register_defaults(reg);
    CHECK(cfd_solver_create(reg, "projection_hip") == NULL);
    cfd_registry_destroy(reg);
    /* restart files: round trip and a corrupted copy */
    ns_solver_params_t prm = ns_solver_params_default();
    snprintf(path, sizeof path, "%s/a.cfdchk", dir);
    CHECK(cfd_checkpoint_write(path, g, f, &prm, 1.5, "projection_hip", "run", "out") == CFD_SUCCESS);
    grid* g2 = NULL;
    flow_field* f2 = NULL;
    ns_solver_params_t p2;
    double t2 = 0;
    char name[64], pre[64], base[64];
    CHECK(cfd_checkpoint_read(path, &g2, &f2, &p2, &t2, name, sizeof name, pre, sizeof pre,
                              base, sizeof base) == CFD_SUCCESS);
    CHECK(t2 == 1.5 && memcmp(f2->u, f->u, nx * ny * nz * sizeof(double)) == 0);
    flow_field_destroy(f2);
    grid_destroy(g2);
    FILE* fp = fopen(path, "r+b");
    CHECK(fp);
    fseek(fp, 200, SEEK_SET);
    fputc(0x5a, fp);
    fclose(fp);
    g2 = NULL; f2 = NULL;
    CHECK(cfd_checkpoint_read(path, &g2, &f2, &p2, &t2, name, sizeof name, pre, sizeof pre,
                              base, sizeof base) != CFD_SUCCESS);
    /* VTK */
    snprintf(path, sizeof path, "%s/f.vtk", dir);
    write_vtk_flow_field(path, f, nx, ny, nz, 0, 1, 0, 1, 0, 1);
    write_vtk_output(path, "p", f->p, nx, ny, nz, 0, 1, 0, 1, 0, 1);
    write_vtk_vector_output(path, "vel", f->u, f->v, NULL, nx, ny, nz, 0, 1, 0, 1, 0, 1);
    write_vtk_output(NULL, "p", f->p, nx, ny, nz, 0, 1, 0, 1, 0, 1);
    /* Poisson factory surface without a device library */
    CHECK(poisson_solver_create(POISSON_METHOD_CG, POISSON_BACKEND_SCALAR) == NULL);
    CHECK(poisson_solver_create(POISSON_METHOD_CG, POISSON_BACKEND_GPU) == NULL);
    CHECK(!poisson_solver_backend_available(POISSON_BACKEND_GPU));
    /* oracle: projection (CG, RB-SOR), CG, RK4 */
    ns_solver_params_t vp = ns_solver_params_default();
    vp.dt = 1e-4; vp.mu = 0.01;
    ns_solver_stats_t st;
    int its = 0;
    CHECK(oracle_projection_step(f, g, &vp, &st, ORACLE_POISSON_CG, &its) == CFD_SUCCESS);
    cfd_status_t rs = oracle_projection_step(f, g, &vp, &st, ORACLE_POISSON_REDBLACK, &its);
    CHECK(rs == CFD_SUCCESS || rs == CFD_ERROR_MAX_ITER);
    CHECK(oracle_rk4_step(f, g, &vp, &st) == CFD_SUCCESS);
    CHECK(oracle_gpu_explicit_step(f, g, &vp) == CFD_SUCCESS);
    flow_field_destroy(f);
    grid_destroy(g);
    printf("ok\n");
    return 0;
}
"""


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not present")
def test_host_code_under_asan_ubsan(tmp_path):
    src = tmp_path / "drv.c"
    src.write_text(DRIVER)
    exe = tmp_path / "drv"
    cmd = ["gcc", "-std=c11", "-g", "-O1", "-fno-omit-frame-pointer",
           "-fsanitize=address,undefined", "-fno-sanitize-recover=undefined",
           f"-I{ROOT / 'include'}", f"-I{ROOT / 'oracle'}", f"-I{HOST}", str(src),
           str(HOST / "cfd_host.c"), str(HOST / "checkpoint_host.c"),
           str(ROOT / "oracle" / "cfd_oracle.c"), "-o", str(exe), "-ldl", "-lm", "-lz"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "-lz" in r.stderr:
        cmd.remove("-lz")
        r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    out = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, env=env,
                         timeout=300)
    assert out.returncode == 0 and out.stdout.strip() == "ok", (out.stdout + out.stderr)[-4000:]
