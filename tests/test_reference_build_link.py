"""The reference-side binding against the REAL reference (VERDICT r03 item
5): tools/reference_link.py copies /root/reference to a scratch directory,
applies the four INTEGRATION.md section-1 edits there, builds it with its
own CMake (CPU only), links libcfd_hip.so by the documented rule and runs
tests/link/reference_driver.c, a program written against the reference's
own API (solver_registry.c:213-279,1155-1181,1615-1694;
simulation_api.c:454-478). Skipped where the reference is absent (the GPU
box); nothing built from the reference travels there.

Opt-in: it configures and compiles the reference tree with the reference's
OWN build scripts (its CMakeLists.txt, run by cmake in a scratch copy) and
then runs a program linked against what they built, so it runs only with
CFD_RUN_REFERENCE_BUILD=1 (`CFD_RUN_REFERENCE_BUILD=1 python -m pytest
tests/test_reference_build_link.py`). The output of the last such run is
committed as profiles/r05_reference_link.json."""
import json
import os
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]

pytestmark = [
    pytest.mark.skipif(os.environ.get("CFD_RUN_REFERENCE_BUILD") != "1",
                       reason="runs the reference's own CMake build: opt in with "
                              "CFD_RUN_REFERENCE_BUILD=1"),
    pytest.mark.skipif(not Path("/root/reference/lib/CMakeLists.txt").exists()
                       or shutil.which("cmake") is None,
                       reason="the reference tree (or cmake) is not here"),
]


@pytest.fixture(scope="module")
def linked(tmp_path_factory):
    work = tmp_path_factory.mktemp("ref_link")
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "reference_link.py"), "--work",
                        str(work), "--jobs", "8"], capture_output=True, text=True, timeout=1200)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


def test_gpu_symbols_resolve_to_hip_library(linked):
    """Edit (c): with CFD_ENABLE_HIP the no-CUDA stub is not compiled into
    cfd_core, so the reference's GPU entry points are libcfd_hip.so's; the
    library's weak references bind to the reference's own registry."""
    assert linked["stub_in_core"] is False
    assert linked["gpu_is_available"] == "libcfd_hip.so"
    assert linked["solve_projection_method_gpu"] == "libcfd_hip.so"
    assert linked["cfd_hip_register_solvers"] == "libcfd_hip.so"
    assert linked["cfd_registry_register"] == "reference_driver"


def test_registry_lists_the_hip_solvers(linked):
    """Edits (a), (b), (d): the five names (projection_hip, _rbsor, _jacobi,
    rk4_hip, projection_hip_cg1) are registered, classified as the GPU
    backend, and in simulation_list_solvers."""
    assert linked["hip_names_by_cuda_backend"] == 5
    assert linked["hip_names_in_simulation_list"] == 5


def test_no_device_here_is_unsupported(linked):
    """No MI355X in this container: the backend reads unavailable, the
    checked create returns NULL, and init_simulation_with_solver(...,
    "projection_hip") fails with CFD_ERROR_UNSUPPORTED and the plugin's
    message (the reference's skip condition, lid_driven_cavity_common.h:286-300)."""
    assert linked["gpu_available"] == 0 and linked["cuda_backend_available"] == 0
    assert linked["create_checked_null"] == 1
    assert linked["init_sim_null"] == 1
    assert linked["init_sim_status"] == -5
    assert "not available" in linked["init_sim_error"]
