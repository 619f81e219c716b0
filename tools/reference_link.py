#!/usr/bin/env python3
"""Builds the REAL reference (shaia/CFD at /root/reference) with the four
INTEGRATION.md section-1 edits applied, links libcfd_hip.so by the documented
rule, and runs tests/link/reference_driver.c against it.

Nothing is written to /root/reference and no reference source enters this
repository: the tree is copied to a scratch directory (default
/tmp/cfd_ref_link), edited there, and built with the reference's own CMake
(CPU only: -DBUILD_TESTS=OFF -DBUILD_EXAMPLES=OFF, so no Unity fetch and no
CUDA). The edits are made by anchor: each one asserts the text it follows is
present, so a changed reference fails loudly instead of building unpatched.

  (a) solver_registry.c: register the HIP solvers after the CUDA block
      (:232-240) through cfd_hip_register_solvers;
  (b) solver_registry.c infer_backend_from_type (:257-279): "_hip" is a GPU
      (NS_SOLVER_BACKEND_CUDA) name;
  (c) lib/CMakeLists.txt: option CFD_ENABLE_HIP drops the no-CUDA stub from
      cfd_core (:182-185, :247-251) and gives cfd_api CFD_HAS_HIP, our
      include directory and libcfd_hip.so;
  (d) simulation_api.c s_solver_names (:454-465): the five HIP names.

The driver is linked with -rdynamic so that libcfd_hip.so's weak references
to cfd_registry_register / cfd_set_error bind to the reference's own.

usage: reference_link.py [--work DIR] [--jobs N]   (prints the driver's JSON line)
"""
import argparse
import json
import os
import shutil
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
REF = Path("/root/reference")


def edit(path: Path, anchor: str, insert: str, after: bool = True) -> None:
    s = path.read_text()
    if anchor not in s:
        raise SystemExit(f"reference_link: anchor not found in {path}: {anchor[:60]!r}")
    if s.count(anchor) != 1:
        raise SystemExit(f"reference_link: anchor not unique in {path}: {anchor[:60]!r}")
    s = s.replace(anchor, anchor + insert if after else insert + anchor)
    path.write_text(s)


def patch(src: Path) -> None:
    reg = src / "lib/src/api/solver_registry.c"
    # (a) includes + registration
    edit(reg, '#include "cfd/solvers/poisson_solver.h"\n',
         '#ifdef CFD_HAS_HIP\n#define CFD_HIP_REFERENCE_TYPES 1\n'
         '#include "cfd_hip/projection_hip.h"\n#endif\n')
    edit(reg, "    cfd_registry_register(registry, NS_SOLVER_TYPE_RK4_GPU, create_rk4_gpu_solver);\n"
              "#endif\n",
         "#ifdef CFD_HAS_HIP\n"
         "    /* projection_hip, projection_hip_rbsor, projection_hip_jacobi, rk4_hip,\n"
         "       projection_hip_cg1 */\n"
         "    cfd_hip_register_solvers(registry);\n#endif\n")
    # (b) backend classification
    edit(reg, '    if (strstr(type_name, "_gpu") != NULL) {\n'
              '        return NS_SOLVER_BACKEND_CUDA;\n    }\n',
         '    if (strstr(type_name, "_hip") != NULL) {\n'
         '        return NS_SOLVER_BACKEND_CUDA; /* the reference\'s only GPU backend id */\n'
         '    }\n')
    # (d) the static name list
    sim = src / "lib/src/api/simulation_api.c"
    edit(sim, '#include "cfd/solvers/navier_stokes_solver.h"\n',
         '#ifdef CFD_HAS_HIP\n#define CFD_HIP_REFERENCE_TYPES 1\n'
         '#include "cfd_hip/projection_hip.h"\n#endif\n')
    edit(sim, "    NS_SOLVER_TYPE_PROJECTION_GPU,\n#ifdef CFD_ENABLE_OPENMP\n",
         "#ifdef CFD_HAS_HIP\n"
         "    NS_SOLVER_TYPE_PROJECTION_HIP, NS_SOLVER_TYPE_PROJECTION_HIP_RBSOR,\n"
         "    NS_SOLVER_TYPE_PROJECTION_HIP_JACOBI, NS_SOLVER_TYPE_RK4_HIP,\n"
         "    NS_SOLVER_TYPE_PROJECTION_HIP_CG1,\n"
         "#endif\n", after=False)
    # (c) CMake: no stub under HIP, and cfd_api gets the library
    cm = src / "lib/CMakeLists.txt"
    edit(cm, "set(CFD_GPU_STUB_SOURCES\n    src/solvers/gpu/solver_gpu_stub.c\n)\n",
         'option(CFD_ENABLE_HIP "Link the MI355X projection library" OFF)\n'
         "if(CFD_ENABLE_HIP)\n    set(CFD_GPU_STUB_SOURCES \"\")\nendif()\n")
    edit(cm, "add_library(CFD::API ALIAS cfd_api)\n",
         "if(CFD_ENABLE_HIP)\n"
         "    target_compile_definitions(cfd_api PRIVATE CFD_HAS_HIP=1)\n"
         "    target_include_directories(cfd_api PRIVATE ${CFD_HIP_ROOT}/include)\n"
         "    target_link_libraries(cfd_api PUBLIC ${CFD_HIP_ROOT}/cfd_amd/lib/libcfd_hip.so)\n"
         "endif()\n", after=False)


def run(cmd, **kw):
    r = subprocess.run(cmd, capture_output=True, text=True, **kw)
    if r.returncode != 0:
        raise SystemExit(f"reference_link: {' '.join(map(str, cmd))} failed ({r.returncode}):\n"
                         + (r.stdout + r.stderr)[-4000:])
    return r.stdout


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--work", default="/tmp/cfd_ref_link")
    ap.add_argument("--jobs", type=int, default=8)
    a = ap.parse_args()
    if not REF.is_dir():
        raise SystemExit("reference_link: /root/reference is absent")
    hip = ROOT / "cfd_amd/lib/libcfd_hip.so"
    if not hip.exists():
        raise SystemExit("reference_link: build libcfd_hip.so first (make -C cfd_amd/csrc)")
    work = Path(a.work)
    src = work / "src"
    if src.exists():
        shutil.rmtree(src)
    shutil.copytree(REF, src, ignore=shutil.ignore_patterns(".git", "build*", "*.so", "*.a",
                                                           "ext_bin"))
    patch(src)
    bld = work / "build"
    gen = ["-G", "Ninja"] if shutil.which("ninja") else []
    run(["cmake", "-S", str(src), "-B", str(bld), *gen, "-DCMAKE_BUILD_TYPE=Release",
         "-DBUILD_TESTS=OFF", "-DBUILD_EXAMPLES=OFF", "-DBUILD_SHARED_LIBS=OFF",
         "-DCFD_ENABLE_HIP=ON", f"-DCFD_HIP_ROOT={ROOT}"])
    run(["cmake", "--build", str(bld), "--target", "cfd_api", "-j", str(a.jobs)])
    libs = {p.name: p for p in bld.rglob("libcfd_*.a")}
    need = ["libcfd_api.a", "libcfd_core.a", "libcfd_scalar.a", "libcfd_simd.a", "libcfd_omp.a"]
    missing = [n for n in need if n not in libs]
    if missing:
        raise SystemExit(f"reference_link: archives not built: {missing}")
    # the stub object must not be in cfd_core any more (edit (c))
    core_objs = run(["ar", "t", str(libs["libcfd_core.a"])])
    exe = work / "reference_driver"
    gen_inc = [str(p.parent.parent) for p in bld.rglob("cfd_export.h")]
    incs = [f"-I{src / 'lib/include'}", *[f"-I{d}" for d in gen_inc], f"-I{ROOT / 'include'}"]
    run(["gcc", "-std=c11", "-O1", "-DCFD_LIBRARY_STATIC_DEFINE", *incs,
         str(ROOT / "tests/link/reference_driver.c"), "-o", str(exe), "-rdynamic",
         "-Wl,--no-as-needed", str(hip), "-Wl,--as-needed",
         "-Wl,--start-group", *[str(libs[n]) for n in need], "-Wl,--end-group",
         "-fopenmp", "-lm", "-ldl", f"-Wl,-rpath,{hip.parent}"])
    env = dict(os.environ)
    out = run([str(exe)], env=env)
    d = json.loads(out.strip().splitlines()[-1])
    d["stub_in_core"] = "solver_gpu_stub.c.o" in core_objs
    d["reference_commit_tree"] = str(REF)
    print(json.dumps(d))


if __name__ == "__main__":
    sys.exit(main())
