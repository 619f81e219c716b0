"""include/cfd_hip/cfd_abi.h against the reference's own header TEXT.

Every struct, enum and function-pointer typedef that cfd_abi.h restates must
declare the same members (or enumerators, or parameter types) in the same
order with the same types as the reference declaration it cites:
navier_stokes_solver.h:54-277, poisson_solver.h:53-233, grid.h:18-40,
cfd_status.h:13-24, boundary_conditions.h:19-57. The reference is read as
data only (this build container has it; the GPU box does not, so the test
skips there).
"""
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
REF = Path("/root/reference/lib/include/cfd")
REF_HEADERS = ["core/cfd_status.h", "core/grid.h", "boundary/boundary_conditions.h",
               "solvers/navier_stokes_solver.h", "solvers/poisson_solver.h"]

pytestmark = pytest.mark.skipif(not REF.is_dir(), reason="reference headers not present")


def _clean(text: str) -> str:
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    text = re.sub(r"^\s*#[^\n]*", " ", text, flags=re.M)
    return re.sub(r"\s+", " ", text)


def _norm_decl(d: str) -> str:
    d = re.sub(r"\s*\*\s*", "* ", d.strip())
    d = re.sub(r"\s*\[\s*", "[", d)
    return re.sub(r"\s+", " ", d).strip()


def _param_types(params: str):
    out = []
    for p in params.split(","):
        p = _norm_decl(p)
        if p in ("void", ""):
            continue
        # drop the parameter name (last identifier) when a type precedes it
        m = re.match(r"^(.*?[\w\*])\s+(\w+)$", p)
        out.append(_norm_decl(m.group(1)) if m else p)
    return out


def _enum_values(body: str):
    vals, nxt = [], 0
    for e in [x.strip() for x in body.split(",") if x.strip()]:
        if "=" in e:
            name, expr = [s.strip() for s in e.split("=", 1)]
            nxt = int(eval(expr, {}, {}))  # integer literals, shifts, unary minus
        else:
            name = e
        vals.append((name, nxt))
        nxt += 1
    return vals


def parse(text: str):
    t = _clean(text)
    decls = {}
    for m in re.finditer(r"typedef struct (?:\w+ )?\{([^{}]*)\} (\w+);", t):
        decls[m.group(2)] = ("struct", [_norm_decl(x) for x in m.group(1).split(";") if x.strip()])
    for m in re.finditer(r"(?<!typedef )struct (\w+) \{([^{}]*)\};", t):
        decls["struct " + m.group(1)] = ("struct",
                                         [_norm_decl(x) for x in m.group(2).split(";") if x.strip()])
    for m in re.finditer(r"typedef enum (?:\w+ )?\{([^{}]*)\} (\w+);", t):
        decls[m.group(2)] = ("enum", _enum_values(m.group(1)))
    for m in re.finditer(r"typedef ([\w\s\*]+?) ?\(\*(\w+)\)\(([^()]*)\);", t):
        decls[m.group(2)] = ("fnptr", [_norm_decl(m.group(1))] + _param_types(m.group(3)))
    for m in re.finditer(r"typedef ([\w\s\*]+?) (\w+);", t):
        if m.group(2) not in decls and not m.group(1).startswith(("struct {", "enum {")):
            decls[m.group(2)] = ("alias", [_norm_decl(m.group(1))])
    return decls


@pytest.fixture(scope="module")
def both():
    ours = parse((ROOT / "include" / "cfd_hip" / "cfd_abi.h").read_text())
    ref = {}
    for h in REF_HEADERS:
        ref.update(parse((REF / h).read_text()))
    return ours, ref


# what cfd_abi.h must restate (the types that cross the plugin boundary)
REQUIRED = [
    "cfd_status_t", "grid", "bc_type_t", "bc_dirichlet_values_t", "flow_field",
    "ns_source_func_t", "ns_heat_source_func_t", "ns_thermal_bc_config_t",
    "ns_solver_params_t", "ns_solver_backend_t", "ns_solver_capabilities_t",
    "ns_solver_stats_t", "ns_solver_context_t", "ns_solver_init_func",
    "ns_solver_destroy_func", "ns_solver_step_func", "ns_solver_solve_func",
    "ns_solver_boundary_func", "ns_solver_compute_dt_func", "ns_solver_get_name_func",
    "ns_solver_get_description_func", "ns_solver_get_capabilities_func", "struct NSSolver",
    "poisson_solver_method_t", "poisson_solver_backend_t", "poisson_solver_status_t",
    "poisson_precond_type_t", "poisson_solver_params_t", "poisson_solver_stats_t",
    "poisson_solver_context_t", "poisson_solver_init_func", "poisson_solver_destroy_func",
    "poisson_solver_solve_func", "poisson_solver_iterate_func", "poisson_solver_apply_bc_func",
    "struct poisson_solver",
]


def test_parser_sees_the_reference_declarations(both):
    _, ref = both
    missing = [n for n in REQUIRED if n not in ref]
    assert not missing, missing
    assert ref["struct NSSolver"][1][0] == "const char* name"
    assert ref["ns_solver_backend_t"][1][-1] == ("NS_SOLVER_BACKEND_CUDA", 3)


@pytest.mark.parametrize("name", REQUIRED)
def test_declaration_matches_reference_text(both, name):
    ours, ref = both
    assert name in ours, f"cfd_abi.h does not declare {name}"
    kind_o, body_o = ours[name]
    kind_r, body_r = ref[name]
    assert kind_o == kind_r, (name, kind_o, kind_r)
    assert body_o == body_r, f"{name}:\n ours {body_o}\n ref  {body_r}"


def test_no_extra_members_anywhere(both):
    """Every declaration cfd_abi.h shares with the reference is identical, not
    only the required ones."""
    ours, ref = both
    shared = [n for n in ours if n in ref]
    assert len(shared) >= len(REQUIRED)
    bad = [n for n in shared if ours[n] != ref[n]]
    assert not bad, bad
