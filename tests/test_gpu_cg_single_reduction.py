"""Opt-in single-reduction (Chronopoulos-Gear) CG, hip_proj_config_t.cg_variant
= 1 (SURVEY.md:461-463, 635-639): the two dot products of
an iteration come out of one reduction, one all-reduce per iteration on
Z-slabs. It is the same Krylov method as the reference's textbook loop
(linear_solver_cg.c:367-439) with different rounding, so it is gated against
textbook CG on the oracle, not bitwise:

  - iteration count within +-2 of the oracle's textbook CG;
  - converged, and the final residual within 1e-8 relative of the oracle's
    final residual scale (|res_cc - res_tb| <= 1e-8 * res0, res0 the
    common initial residual);
  - the solution within 1e-6 relative of the oracle's (both stop at the
    1e-6 relative tolerance);
  - on Z-slabs (in-process group, 2-4 ranks) equal to the single-device
    variant within 1e-10 (only the dot summation order differs) with the
    same iteration counts +-1.
"""
import numpy as np
import pytest

from cfd_amd import _abi as A
from cfd_amd import api
from oracle import oracle
from tests import cases
from tests.test_gpu_slabs import FIELDS, Slabs, _cavity_bc_device, _run_steps, _slab_poisson

pytestmark = pytest.mark.gpu

CC = dict(cg_variant=1)


def _rel(a, b):
    return float(np.max(np.abs(a - b))) / max(1e-300, float(np.max(np.abs(b))))


@pytest.mark.parametrize("n,nz", [(33, 33), (65, 65), (48, 1), (40, 24)])
def test_poisson_vs_textbook_oracle(hip_lib, n, nz):
    """cos(pi x)cos(pi y)cos(pi z) (47 / 97 textbook
    iterations at 33^3 / 65^3)."""
    g, rhs = cases.cos_rhs(n, nz)
    xo = np.zeros_like(rhs)
    so, sto = oracle.cg_solve(xo, rhs, g.dx, g.dy, g.dz)
    ctx = api.HipProjection(n, n, nz, **CC)
    try:
        x = np.zeros_like(rhs)
        s, st = ctx.poisson_solve(A.HIP_POISSON_CG, x, rhs, g.dx, g.dy, g.dz)
    finally:
        ctx.close()
    assert so == s == A.CFD_SUCCESS
    assert st.status == A.POISSON_CONVERGED
    assert abs(st.iterations - sto.iterations) <= 2, (st.iterations, sto.iterations)
    assert st.initial_residual == pytest.approx(sto.initial_residual, rel=1e-12)
    assert abs(st.final_residual - sto.final_residual) <= 1e-8 * sto.initial_residual
    d = (x - x.mean()) - (xo - xo.mean())
    assert float(np.max(np.abs(d))) / float(np.max(np.abs(xo))) <= 1e-6


def test_projection_steps_vs_textbook_oracle(hip_lib):
    """Cavity steps through the whole projection (CG on the fused divergence
    RHS), cg_variant 1 vs the oracle's textbook CG."""
    g, f, p = cases.cavity(33, 29, 21, Re=100.0, dt=5e-4)
    fo = api.FlowField(g.nx, g.ny, g.nz)
    fo.copy_from(f)
    ctx = api.HipProjection(g.nx, g.ny, g.nz, **CC)
    try:
        for _ in range(4):
            api.cavity_bc(f, 1.0)
            api.cavity_bc(fo, 1.0)
            assert ctx.step(f, g, p) == A.CFD_SUCCESS, api._native.last_error()
            ih = ctx.poisson_stats().iterations
            so, _, io = oracle.projection_step(fo, g, p)
            assert so == A.CFD_SUCCESS
            assert abs(ih - io) <= 2, (ih, io)
    finally:
        ctx.close()
    for k in ("u", "v", "w"):
        assert _rel(getattr(f, k), getattr(fo, k)) <= 1e-6, k
    dp = (f.p - f.p.mean()) - (fo.p - fo.p.mean())
    assert float(np.max(np.abs(dp))) / float(np.max(np.abs(fo.p))) <= 1e-5


def test_trivial_and_capped(hip_lib):
    """Zero RHS: converged at iteration 0 (x untouched); a cap below the
    needed count: MAX_ITER after exactly max_iterations iterations."""
    g, rhs = cases.cos_rhs(17)
    ctx = api.HipProjection(17, 17, 17, **CC)
    try:
        x = np.zeros_like(rhs)
        s, st = ctx.poisson_solve(A.HIP_POISSON_CG, x, np.zeros_like(rhs), g.dx, g.dy, g.dz)
        assert s == A.CFD_SUCCESS and st.iterations == 0 and not x.any()
        prm = oracle.poisson_params(max_iterations=5, tolerance=1e-14, absolute_tolerance=0.0)
        x = np.zeros_like(rhs)
        s, st = ctx.poisson_solve(A.HIP_POISSON_CG, x, rhs, g.dx, g.dy, g.dz, prm)
        assert s == A.CFD_ERROR_MAX_ITER and st.iterations == 5
        xo = np.zeros_like(rhs)
        so, sto = oracle.cg_solve(xo, rhs, g.dx, g.dy, g.dz, prm)
        assert sto.iterations == 5
        # after 5 iterations the Krylov iterates agree to rounding
        assert _rel(x, xo) <= 1e-10
    finally:
        ctx.close()


@pytest.mark.parametrize("nranks,n", [(2, 33), (4, 33), (4, 13), (8, 17), (4, 9)])
def test_slab_poisson_matches_single_device(hip_lib, nranks, n):
    """33^3: every slab >= 3 planes (the edge-plane launch, the r halo on the
    side stream over the interior launch); 13^3 on 4 ranks mixes 3- and
    2-plane slabs, 17^3 on 8 ranks 2- and 1-plane ones, 9^3 on 4 ranks 2 and
    1: slabs of < 3 planes run the whole march, then a blocking r halo
    (projection_hip.hip iterate_cc), beside neighbours that split."""
    spans = [api.slab_layout(n, r, nranks)[1] - 2 for r in range(nranks)]
    if n == 13:
        assert sorted(set(spans)) == [2, 3]
    elif n != 33:
        assert min(spans) < 3
    g, rhs = cases.cos_rhs(n)
    ctx = api.HipProjection(n, n, n, **CC)
    try:
        x1 = np.zeros_like(rhs)
        s1, st1 = ctx.poisson_solve(A.HIP_POISSON_CG, x1, rhs, g.dx, g.dy, g.dz)
    finally:
        ctx.close()
    stat, its, x = _slab_poisson(g, rhs, nranks, A.HIP_POISSON_CG, **CC)
    assert s1 == A.CFD_SUCCESS and all(s == A.CFD_SUCCESS for s in stat)
    assert len(set(its)) == 1 and abs(its[0] - st1.iterations) <= 1
    assert _rel(x, x1) <= 1e-10


def test_slab_cavity_steps(hip_lib):
    g, f, p = cases.cavity(33, 33, 33, Re=100.0, dt=5e-4)
    ref = api.HipProjection(g.nx, g.ny, g.nz, **CC)
    S = Slabs(g, 3, **CC)
    try:
        ref.upload(f)
        S.scatter(f)
        hist = _run_steps(S, g, p, 3, _cavity_bc_device)
        its1 = []
        for _ in range(3):
            _cavity_bc_device(ref)
            assert ref.step_device(g, p) == A.CFD_SUCCESS
            its1.append(ref.poisson_stats().iterations)
        got = {k: S.gather(k) for k in FIELDS}
        want = {k: ref.get_field(fid) for k, fid in FIELDS.items()}
    finally:
        S.close()
        ref.close()
    for r in range(3):
        assert hist[r] == hist[0]
    assert all(abs(h[0] - i) <= 1 for h, i in zip(hist[0], its1)), (hist[0], its1)
    for k in FIELDS:
        assert _rel(got[k], want[k]) <= 1e-10, k


@pytest.mark.parametrize("tail,kc2", [("1", "12"), ("2", "5")])
def test_ccf_tail_layout_vs_textbook_oracle(hip_lib, monkeypatch, tail, kc2):
    """k_ccf's optional tail layers of shorter z runs (ccf_layout,
    CFD_HIP_CCF_TAIL / _KC2, read at context creation; off by default, r06):
    the march's z decomposition changes only the per-tile dot grouping, so
    the solve stays within the single-reduction gates against the oracle's
    textbook CG. 65^3 (63 planes: 24-plane bulk runs + the tail) and a
    fixed-iteration run, bitwise equal iterates between two contexts of the
    same layout."""
    monkeypatch.setenv("CFD_HIP_CCF_TAIL", tail)
    monkeypatch.setenv("CFD_HIP_CCF_KC2", kc2)
    monkeypatch.setenv("CFD_HIP_CCF_KC", "24")
    monkeypatch.setenv("CFD_HIP_CCF_KC_FIXED", "1")
    n = 65
    g, rhs = cases.cos_rhs(n, n)
    xo = np.zeros_like(rhs)
    so, sto = oracle.cg_solve(xo, rhs, g.dx, g.dy, g.dz)
    ctx = api.HipProjection(n, n, n, **CC)
    try:
        x = np.zeros_like(rhs)
        s, st = ctx.poisson_solve(A.HIP_POISSON_CG, x, rhs, g.dx, g.dy, g.dz)
    finally:
        ctx.close()
    assert so == s == A.CFD_SUCCESS and st.status == A.POISSON_CONVERGED
    assert abs(st.iterations - sto.iterations) <= 2, (st.iterations, sto.iterations)
    assert abs(st.final_residual - sto.final_residual) <= 1e-8 * sto.initial_residual
    d = (x - x.mean()) - (xo - xo.mean())
    assert float(np.max(np.abs(d))) / float(np.max(np.abs(xo))) <= 1e-6


def test_field_stagger_is_bitwise_neutral(hip_lib, monkeypatch):
    """The default 4 KiB field stagger (r06) moves where fields sit in their
    allocations, never what is computed: cavity steps with both CG forms
    are bitwise equal to the unstaggered fields (CFD_HIP_FIELD_STAGGER=0)."""
    n = 33
    out = {}
    for stagger in ("0", None):
        if stagger is None:
            monkeypatch.delenv("CFD_HIP_FIELD_STAGGER", raising=False)
        else:
            monkeypatch.setenv("CFD_HIP_FIELD_STAGGER", stagger)
        for cgv in (0, 1):
            g, f, p = cases.cavity(n, n, n, Re=400.0, dt=2e-3)
            ctx = api.HipProjection(n, n, n, cg_variant=cgv)
            try:
                api.cavity_bc(f, 1.0)
                ctx.upload(f)
                for _ in range(3):
                    assert ctx.step_device(g, p) == A.CFD_SUCCESS, api._native.last_error()
                out[(stagger, cgv)] = {k: ctx.get_field(fid).copy() for k, fid in
                                       (("u", A.HIP_FIELD_U), ("v", A.HIP_FIELD_V),
                                        ("w", A.HIP_FIELD_W), ("p", A.HIP_FIELD_P))}
            finally:
                ctx.close()
    for cgv in (0, 1):
        for k in ("u", "v", "w", "p"):
            a, b = out[("0", cgv)][k], out[(None, cgv)][k]
            assert np.array_equal(a.view(np.uint64), b.view(np.uint64)), (cgv, k)


def test_placement_draws_are_bitwise_neutral(hip_lib, monkeypatch):
    """The placement draws (r06; a single-reduction context of >= 2^24 cells
    allocates its CG fields six times and times 40 assignments of them to the
    seven roles) choose where the fields sit, never what is computed: the
    probe records 40 positive times and keeps the fastest, and cavity steps
    are bitwise those of a context without draws (CFD_HIP_PLACEMENT_DRAWS=1)."""
    n, nz = 256, 257  # 16.84 M cells, just above 2^24
    out, place = {}, {}
    for draws in ("1", None):
        if draws is None:
            monkeypatch.delenv("CFD_HIP_PLACEMENT_DRAWS", raising=False)
        else:
            monkeypatch.setenv("CFD_HIP_PLACEMENT_DRAWS", draws)
        g, f, p = cases.cavity(n, n, nz, Re=400.0, dt=2e-4)
        ctx = api.HipProjection(n, n, nz, cg_variant=1)
        try:
            place[draws] = ctx.placement()
            api.cavity_bc(f, 1.0)
            ctx.upload(f)
            for _ in range(2):
                assert ctx.step_device(g, p) == A.CFD_SUCCESS, api._native.last_error()
            out[draws] = {k: ctx.get_field(fid).copy() for k, fid in
                          (("u", A.HIP_FIELD_U), ("p", A.HIP_FIELD_P))}
        finally:
            ctx.close()
    assert place["1"] == ([], -1)
    ms, pick = place[None]
    assert len(ms) == 40 and all(v > 0 for v in ms)
    assert 0 <= pick < 40 and ms[pick] == min(ms)  # (times rounded to 0.1 us)
    for k in ("u", "p"):
        assert np.array_equal(out["1"][k].view(np.uint64), out[None][k].view(np.uint64)), k
