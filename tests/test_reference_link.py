"""The reference-side binding, checked on CPU.

1. Link order. The reference always compiles its no-CUDA stub into
   libcfd_core.a (lib/CMakeLists.txt:182-185,247-251); the stub defines the
   same gpu_* / solve_*_gpu symbols libcfd_hip.so exports. A C driver is
   linked with a registry-like object (tests/link/registry_probe.c) in an
   archive, our restatement of the stub (tests/link/nocuda_stub.c) in a
   "core" archive, and libcfd_hip.so, in the orders INTEGRATION.md documents;
   dladdr tells which file each referenced symbol resolved to.
2. The registry's view of the new names, unpatched and patched
   (solver_registry.c:257-279,1638-1694; simulation_api.c:454-478), through
   the host mirror's switch cfd_host_set_hip_patch.
"""
import ctypes as C
import re
import subprocess
from pathlib import Path

import pytest

from cfd_amd import _abi as A
from cfd_amd import _native, api

ROOT = Path(__file__).resolve().parents[1]
LINK = ROOT / "tests" / "link"


@pytest.fixture(scope="module")
def objs(tmp_path_factory):
    _native.hip()  # built in-tree
    d = tmp_path_factory.mktemp("link")
    inc = f"-I{ROOT / 'include'}"
    for name in ("nocuda_stub", "registry_probe", "link_driver"):
        subprocess.run(["gcc", "-std=c11", "-fPIC", "-O1", inc, "-c", str(LINK / f"{name}.c"),
                        "-o", str(d / f"{name}.o")], check=True)
    subprocess.run(["ar", "rcs", str(d / "libcore_stub.a"), str(d / "nocuda_stub.o")], check=True)
    subprocess.run(["ar", "rcs", str(d / "libapi_probe.a"), str(d / "registry_probe.o")],
                   check=True)
    return d


def _link_and_run(d, name, libs):
    exe = d / name
    libdir = str(_native.LIB_DIR)
    subprocess.run(["gcc", "-pie", str(d / "link_driver.o"), *libs, "-o", str(exe), "-ldl",
                    f"-Wl,-rpath,{libdir}"], check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout
    return dict(line.split() for line in out.splitlines())


def test_stub_removed_from_core_resolves_to_hip(objs):
    """under CFD_HAS_HIP cfd_core is built without
    ${CFD_GPU_STUB_SOURCES}; every GPU symbol then comes from libcfd_hip.so."""
    hip = str(_native.HIP_LIB)
    got = _link_and_run(objs, "no_stub", ["-Wl,--start-group", str(objs / "libapi_probe.a"),
                                          "-Wl,--end-group", hip])
    assert got["gpu_is_available"] == "libcfd_hip.so"
    assert got["solve_projection_method_gpu"] == "libcfd_hip.so"
    assert got["solve_rk4_method_gpu"] == "libcfd_hip.so"
    assert got["enable_gpu"] == "1"


def test_hip_library_before_the_archive_group_wins(objs):
    """INTEGRATION.md §1 link rule: with the stub still in libcfd_core.a,
    naming libcfd_hip.so (kept with --no-as-needed) BEFORE the reference's
    static group (lib/CMakeLists.txt:524-536) defines every stub symbol
    first, so the stub object is never extracted."""
    hip = str(_native.HIP_LIB)
    got = _link_and_run(objs, "hip_first", ["-Wl,--no-as-needed", hip, "-Wl,--as-needed",
                                            "-Wl,--start-group",
                                            str(objs / "libapi_probe.a"),
                                            str(objs / "libcore_stub.a"), "-Wl,--end-group"])
    assert got["gpu_is_available"] == "libcfd_hip.so"
    assert got["solve_projection_method_gpu"] == "libcfd_hip.so"
    assert got["solve_rk4_method_gpu"] == "libcfd_hip.so"
    assert got["enable_gpu"] == "1"


def test_as_needed_hip_library_before_the_group_loses_to_the_stub(objs):
    """Why the rule says --no-as-needed: under --as-needed (the default of
    this gcc) a shared library that satisfies nothing yet when it is scanned
    is dropped with its definitions, so the stub is extracted after all."""
    hip = str(_native.HIP_LIB)
    got = _link_and_run(objs, "hip_first_as_needed", [
        "-Wl,--as-needed", hip, "-Wl,--start-group", str(objs / "libapi_probe.a"),
        str(objs / "libcore_stub.a"), "-Wl,--end-group"])
    assert got["gpu_is_available"] == "hip_first_as_needed"
    assert got["enable_gpu"] == "0"


def test_hip_library_after_the_group_loses_to_the_stub(objs):
    """The hazard the rule avoids: libcfd_hip.so after the group leaves
    gpu_is_available undefined while libcfd_core.a is scanned, the stub object
    is extracted, and the executable's copies shadow the HIP library."""
    hip = str(_native.HIP_LIB)
    got = _link_and_run(objs, "hip_last", ["-Wl,--start-group", str(objs / "libapi_probe.a"),
                                           str(objs / "libcore_stub.a"), "-Wl,--end-group", hip])
    assert got["gpu_is_available"] == "hip_last"
    assert got["solve_projection_method_gpu"] == "hip_last"
    assert got["enable_gpu"] == "0"


def test_hip_library_defines_every_stub_symbol():
    """libcfd_hip.so exports the full symbol set of solver_gpu_stub.c:15-161,
    the condition for the link rule above."""
    text = (LINK / "nocuda_stub.c").read_text()
    names = set(re.findall(r"^\w[\w\s\*]*?\b(gpu_\w+|solve_\w+)\(", text, flags=re.M))
    names |= set(re.findall(r"STUB_SOLVE\((\w+)\)", text))
    names -= {"gpu_solver_stats_t", "name"}
    assert len(names) == 17, sorted(names)
    out = subprocess.run(["nm", "-D", "--defined-only", str(_native.HIP_LIB)],
                         capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if line.strip()}
    assert not (names - exported), names - exported


def _names(fn, *args):
    n = fn(*args, None, 0)
    arr = (C.c_char_p * max(n, 1))()
    got = fn(*args, arr, n)
    return [arr[i].decode() for i in range(min(n, got))]


@pytest.fixture()
def host():
    h = _native.host()
    yield h
    h.cfd_host_set_hip_patch(0)


def test_unpatched_reference_classifies_hip_as_scalar(host):
    """Without the edits, infer_backend_from_type (solver_registry.c:257-279)
    stores projection_hip as SCALAR: the GPU listing omits it, the SCALAR
    listing holds it, create_checked checks the scalar backend (always
    available) and reaches the factory, and simulation_list_solvers'
    static table lacks the names."""
    host.cfd_host_set_hip_patch(0)
    reg = api.Registry()
    lb = host.cfd_registry_list_by_backend
    assert "projection_hip" not in _names(lb, reg._ptr, A.NS_SOLVER_BACKEND_CUDA)
    assert "projection_hip" in _names(lb, reg._ptr, A.NS_SOLVER_BACKEND_SCALAR)
    assert "projection_hip" not in _names(host.simulation_list_solvers)
    if not _native.hip().hip_projection_available():
        host.cfd_clear_error()
        assert not host.cfd_solver_create_checked(reg._ptr, b"projection_hip")
        # the factory's own check, not the backend gate
        assert host.cfd_get_last_error() == b"HIP GPU not available at runtime"


def test_patched_reference_classifies_hip_as_gpu(host):
    """With the INTEGRATION.md §1 edits: `_hip` names are GPU-backend entries,
    gated by gpu_is_available() (solver_registry.c:1615-1616, resolved into
    libcfd_hip.so), and listed by simulation_list_solvers."""
    host.cfd_host_set_hip_patch(1)
    reg = api.Registry()
    lb = host.cfd_registry_list_by_backend
    gpu = _names(lb, reg._ptr, A.NS_SOLVER_BACKEND_CUDA)
    for n in ("projection_hip", "projection_hip_rbsor", "projection_hip_jacobi", "rk4_hip",
              "projection_hip_cg1"):
        assert n in gpu
        assert n in _names(host.simulation_list_solvers)
    assert lb(reg._ptr, A.NS_SOLVER_BACKEND_SCALAR, None, 0) == 0
    if not _native.hip().hip_projection_available():
        host.cfd_clear_error()
        assert not host.cfd_solver_create_checked(reg._ptr, b"projection_hip")
        assert host.cfd_get_last_status() == A.CFD_ERROR_UNSUPPORTED
        assert host.cfd_get_last_error() == b"Backend 'cuda' is not available on this system"
