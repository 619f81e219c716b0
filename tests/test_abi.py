"""The C-ABI boundary on CPU: libraries load, every symbol the public headers
declare is exported, the ctypes mirrors have the C layouts, and the plugin
behaves like the reference's GPU factory when no device is present."""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

from cfd_amd import _abi as A
from cfd_amd import _native, api

ROOT = Path(__file__).resolve().parents[1]
INC = ROOT / "include" / "cfd_hip"


def _declared(header: Path):
    text = header.read_text()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return re.findall(r"CFD_HIP_EXPORT[^;(]*?\b(\w+)\s*\(", text)


def _exported(lib: Path):
    out = subprocess.run(["nm", "-D", "--defined-only", str(lib)], capture_output=True,
                         text=True, check=True).stdout
    return {line.split()[-1] for line in out.splitlines() if line.strip()}


def test_hip_library_exports_projection_abi():
    _native.hip()
    names = _declared(INC / "projection_hip.h")
    assert len(names) >= 25
    missing = set(names) - _exported(_native.HIP_LIB)
    assert not missing, missing


def test_hip_library_exports_gpu_device_api():
    """Every gpu_device.h entry point (reference gpu_device.h:91-247) is exported."""
    _native.hip()
    names = _declared(INC / "gpu_device.h")
    assert len(names) >= 15
    missing = set(names) - _exported(_native.HIP_LIB)
    assert not missing, missing


def test_hip_library_exports_device_bc_api():
    """boundary_conditions_gpu.cuh:32-151 entry points (inlet excepted)."""
    _native.hip()
    names = _declared(INC / "boundary_conditions_gpu.h")
    assert len(names) == 7
    missing = set(names) - _exported(_native.HIP_LIB)
    assert not missing, missing


def test_host_library_exports_host_api():
    _native.host()
    names = _declared(INC / "cfd_host.h")
    assert len(names) >= 30
    missing = set(names) - _exported(_native.HOST_LIB)
    assert not missing, missing


def test_hip_library_targets_gfx950_only(tmp_path):
    fat = tmp_path / "fat.bin"
    subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}",
                    str(_native.HIP_LIB)], check=True)
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/clang-offload-bundler", "--list", "--type=o",
                          f"--input={fat}"], capture_output=True, text=True, check=True)
    targets = [t for t in out.stdout.split() if "amdgcn" in t]
    assert targets and all(t.endswith("gfx950") for t in targets), targets


LAYOUT_PROBE = r"""
#include <stdio.h>
#include <stddef.h>
#include "cfd_hip/cfd_abi.h"
#include "cfd_hip/projection_hip.h"
#include "cfd_hip/cfd_host.h"
#include "cfd_hip/gpu_device.h"
int main(void) {
  printf("grid %zu %zu\n", sizeof(grid), offsetof(grid, k_end));
  printf("flow_field %zu %zu\n", sizeof(flow_field), offsetof(flow_field, nz));
  printf("params %zu %zu\n", sizeof(ns_solver_params_t), offsetof(ns_solver_params_t, thermal_bc));
  printf("stats %zu %zu\n", sizeof(ns_solver_stats_t), offsetof(ns_solver_stats_t, status));
  printf("solver %zu %zu\n", sizeof(ns_solver_t), offsetof(ns_solver_t, get_capabilities));
  printf("pparams %zu %zu\n", sizeof(poisson_solver_params_t), offsetof(poisson_solver_params_t, preconditioner));
  printf("pstats %zu\n", sizeof(poisson_solver_stats_t));
  printf("hipcfg %zu %zu\n", sizeof(hip_proj_config_t), offsetof(hip_proj_config_t, verbose));
  printf("sim %zu %zu\n", sizeof(simulation_data), offsetof(simulation_data, output_base_dir));
  printf("hipcfg2 %zu\n", offsetof(hip_proj_config_t, poisson_fail_fatal));
  printf("gpucfg %zu %zu\n", sizeof(gpu_config_t), offsetof(gpu_config_t, verbose));
  printf("gpuinfo %zu %zu\n", sizeof(gpu_device_info_t), offsetof(gpu_device_info_t, is_available));
  printf("gpustats %zu %zu\n", sizeof(gpu_solver_stats_t), offsetof(gpu_solver_stats_t, kernels_launched));
  printf("psolver %zu %zu\n", sizeof(poisson_solver_t), offsetof(poisson_solver_t, apply_bc));
  return 0;
}
"""


def test_ctypes_layouts_match_c(tmp_path):
    src = tmp_path / "probe.c"
    src.write_text(LAYOUT_PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c11", f"-I{ROOT / 'include'}", str(src), "-o", str(exe)],
                   check=True)
    got = {}
    for line in subprocess.run([str(exe)], capture_output=True, text=True,
                               check=True).stdout.splitlines():
        k, *v = line.split()
        got[k] = [int(x) for x in v]
    assert got["grid"] == [C.sizeof(A.Grid), A.Grid.k_end.offset]
    assert got["flow_field"] == [C.sizeof(A.FlowField), A.FlowField.nz.offset]
    assert got["params"] == [C.sizeof(A.SolverParams), A.SolverParams.thermal_bc.offset]
    assert got["stats"] == [C.sizeof(A.SolverStats), A.SolverStats.status.offset]
    assert got["solver"] == [C.sizeof(A.NSSolver), A.NSSolver.get_capabilities.offset]
    assert got["pparams"] == [C.sizeof(A.PoissonParams), A.PoissonParams.preconditioner.offset]
    assert got["pstats"] == [C.sizeof(A.PoissonStats)]
    assert got["hipcfg"] == [C.sizeof(A.HipProjConfig), A.HipProjConfig.verbose.offset]
    assert got["sim"] == [C.sizeof(A.SimulationData), A.SimulationData.output_base_dir.offset]
    assert got["hipcfg2"] == [A.HipProjConfig.poisson_fail_fatal.offset]
    assert got["gpucfg"] == [C.sizeof(A.GpuConfig), A.GpuConfig.verbose.offset]
    assert got["gpuinfo"] == [C.sizeof(A.GpuDeviceInfo), A.GpuDeviceInfo.is_available.offset]
    assert got["gpustats"] == [C.sizeof(A.GpuSolverStats), A.GpuSolverStats.kernels_launched.offset]
    assert got["psolver"] == [C.sizeof(A.PoissonSolver), A.PoissonSolver.apply_bc.offset]


def test_registry_lists_hip_solvers():
    reg = api.Registry()
    names = reg.names()
    for n in ("projection_hip", "projection_hip_rbsor", "projection_hip_jacobi", "rk4_hip",
              "projection_hip_cg1"):
        assert n in names


def test_factory_without_device_is_unsupported():
    """solver_registry.c:1155-1160: NULL + CFD_ERROR_UNSUPPORTED when no GPU."""
    if _native.hip().hip_projection_available():
        pytest.skip("a HIP device is present")
    reg = api.Registry()
    with pytest.raises(api.CfdError) as e:
        reg.create("projection_hip")
    assert e.value.status == A.CFD_ERROR_UNSUPPORTED


def test_unknown_solver_not_found():
    reg = api.Registry()
    with pytest.raises(api.CfdError) as e:
        reg.create("no_such_solver")
    assert e.value.status == A.CFD_ERROR_NOT_FOUND


def test_context_create_without_device_fails_loudly():
    if _native.hip().hip_projection_available():
        pytest.skip("a HIP device is present")
    with pytest.raises(api.CfdError):
        api.HipProjection(8, 8, 8)


def test_gpu_config_defaults():
    """test_solver_gpu_api.c:31-41 and solver_projection_gpu.cu:294-308."""
    c = _native.hip().gpu_config_default()
    assert c.enable_gpu == 1 and c.min_grid_size == 10000 and c.min_steps == 10
    assert c.block_size_x > 0 and c.block_size_y > 0
    assert c.poisson_max_iter == 1000 and c.poisson_tolerance == 1e-3


def test_gpu_api_without_device():
    """test_solver_gpu_api.c:467-495: no device -> should_use 0, create NULL."""
    lib = _native.hip()
    if lib.gpu_is_available():
        pytest.skip("a HIP device is present")
    c = lib.gpu_config_default()
    assert lib.gpu_should_use(C.byref(c), 1000, 1000, 1, 20) == 0
    assert lib.gpu_should_use(None, 100, 100, 1, 10) == 0
    assert not lib.gpu_solver_create(64, 64, 1, C.byref(c))
    info = (A.GpuDeviceInfo * 2)()
    assert lib.gpu_get_device_info(info, 2) == 0


def test_poisson_factory_surface():
    """poisson_solver_create (linear_solver.c:150-235): GPU factories by method,
    NULL for pairs with no GPU form; init reports UNSUPPORTED without a device
    (poisson_solver_cg_gpu.cu:61-65)."""
    host, hip = _native.host(), _native.hip()
    p = host.poisson_solver_params_default()
    assert (p.tolerance, p.absolute_tolerance, p.max_iterations, p.check_interval) == \
        (1e-6, 1e-10, 5000, 1)
    assert host.poisson_solver_stats_default().status == A.POISSON_ERROR
    for m, name in ((A.POISSON_METHOD_CG, b"cg_gpu"), (A.POISSON_METHOD_REDBLACK_SOR,
                    b"redblack_gpu"), (A.POISSON_METHOD_JACOBI, b"jacobi_gpu")):
        s = host.poisson_solver_create(m, A.POISSON_BACKEND_GPU)
        assert s and s.contents.name == name and s.contents.backend == A.POISSON_BACKEND_GPU
        assert s.contents.method == m
        if not hip.hip_projection_available():
            rc = host.poisson_solver_init(s, 17, 17, 1, 0.1, 0.1, 0.0, None)
            assert rc == A.CFD_ERROR_UNSUPPORTED
        host.poisson_solver_destroy(s)
    assert not host.poisson_solver_create(A.POISSON_METHOD_SOR, A.POISSON_BACKEND_GPU)
    assert not host.poisson_solver_create(A.POISSON_METHOD_CG, A.POISSON_BACKEND_SCALAR)
    assert not host.poisson_solver_create(A.POISSON_METHOD_BICGSTAB, A.POISSON_BACKEND_GPU)
    s = host.poisson_solver_create(A.POISSON_METHOD_CG, A.POISSON_BACKEND_GPU)
    assert host.poisson_solver_init(s, 17, 2, 1, 0.1, 0.1, 0.0, None) == A.CFD_ERROR_INVALID
    assert host.poisson_solver_iterate(s, None, None, None, None) == A.CFD_ERROR_INVALID
    host.poisson_solver_destroy(s)


REFERENCE_STYLE_DRIVER = r"""
/* Written the way a reference user calls the device API (cfd/core/gpu_device.h,
 * cfd/solvers/poisson_solver.h): it must compile and link against the MI355X
 * libraries unchanged. Without a device every entry reports "unavailable". */
#include <stdio.h>
#include "cfd_hip/cfd_host.h"
#include "cfd_hip/gpu_device.h"
#include "cfd_hip/projection_hip.h"
int main(void) {
  gpu_config_t cfg = gpu_config_default();
  int avail = gpu_is_available();
  gpu_solver_context_t* ctx = gpu_solver_create(32, 32, 1, &cfg);
  poisson_solver_t* ps = poisson_solver_create(POISSON_METHOD_CG, POISSON_BACKEND_GPU);
  cfd_status_t st = poisson_solver_init(ps, 33, 33, 1, 1.0 / 32, 1.0 / 32, 0.0, NULL);
  printf("%d %d %d %d\n", avail, ctx != NULL, ps != NULL, (int)st);
  if (ctx) gpu_solver_destroy(ctx);
  poisson_solver_destroy(ps);
  return 0;
}
"""


def test_reference_style_driver_links(tmp_path):
    lib = _native.hip()
    src = tmp_path / "driver.c"
    src.write_text(REFERENCE_STYLE_DRIVER)
    exe = tmp_path / "driver"
    libdir = _native.LIB_DIR
    subprocess.run(["gcc", "-std=c11", f"-I{ROOT / 'include'}", str(src), "-o", str(exe),
                    f"-L{libdir}", "-lcfd_host", "-lcfd_hip", f"-Wl,-rpath,{libdir}"], check=True)
    if lib.hip_projection_available():
        return  # the run is the GPU tests' business
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    assert out == ["0", "0", "1", str(A.CFD_ERROR_UNSUPPORTED)]
