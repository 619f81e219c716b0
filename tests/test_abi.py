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


def test_registry_lists_hip_solvers():
    reg = api.Registry()
    names = reg.names()
    for n in ("projection_hip", "projection_hip_rbsor", "projection_hip_jacobi"):
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
