"""The CPU oracle against the reference's own golden vectors and against
reference outputs recorded in SURVEY.md App. B (CPU only)."""
import math

import numpy as np
import pytest

from cfd_amd import _abi as A
from oracle import oracle
from tests import cases


def test_projection_kat_bitexact():
    """test_ns_solver_3d.c:345-348, reproduced bit for bit (reference gate 1e-12)."""
    g, f, p = cases.kat_2d()
    s, st, iters = oracle.projection_step(f, g, p)
    assert s == A.CFD_SUCCESS
    l2 = (cases.l2_rms(f.u), cases.l2_rms(f.v), cases.l2_rms(f.p))
    assert l2 == cases.KAT_PROJECTION_L2
    assert np.all(f.w == 0.0)
    assert st.iterations == 1 and iters > 0


def test_rk4_kat_bitexact():
    """test_ns_solver_3d.c:363-366 RK4 golden L2 triple, bit for bit."""
    g, f, p = cases.kat_2d()
    s, st = oracle.rk4_step(f, g, p)
    assert s == A.CFD_SUCCESS and st.iterations == 1
    l2 = (cases.l2_rms(f.u), cases.l2_rms(f.v), cases.l2_rms(f.p))
    assert l2 == cases.KAT_RK4_L2
    assert np.all(f.w == 0.0)


@pytest.mark.parametrize("n,expected", [(33, 47), (65, 97)])
def test_cg_iteration_counts(n, expected):
    """CG cold solve on the cos*cos*cos rhs: 47 / 97 iterations at 33^3 / 65^3
    (measured on the reference build)."""
    g, rhs = cases.cos_rhs(n)
    x = np.zeros_like(rhs)
    s, st = oracle.cg_solve(x, rhs, g.dx, g.dy, g.dz)
    assert s == A.CFD_SUCCESS and st.status == A.POISSON_CONVERGED
    assert st.iterations == expected


def test_tg3d_16_l2():
    """3-D Taylor-Green 16^3, 100 steps: rel. L2(u) = L2(v) = 5.336557e-02
    (reference gate 0.25 in taylor_green_3d_reference.h:58)."""
    g, f, p = cases.tg3(16)
    for _ in range(100):
        cases.tg3_bc(f)
        s, _, _ = oracle.projection_step(f, g, p)
        assert s == A.CFD_SUCCESS
    eu, ev = cases.tg3_l2_errors(g, f, 100 * 1e-3)
    assert eu == pytest.approx(5.336557e-02, rel=2e-6)
    assert ev == pytest.approx(5.336557e-02, rel=2e-6)


@pytest.mark.slow
def test_ghia_33_re100_rms():
    """33x33 cavity Re=100, 5000 steps, dt=5e-4: RMS_u = 0.0382 vs Ghia
    (docs/validation/cavity-backends-validation.md:115)."""
    from tests import ghia
    g, f, p = cases.cavity(33, 33, 1, Re=100.0, dt=5e-4)
    for _ in range(5000):
        ghia_bc(f)
        s, _, _ = oracle.projection_step(f, g, p)
        assert s == A.CFD_SUCCESS
    rms_u, rms_v = ghia.rms_re100(f, g)
    assert round(rms_u, 4) == 0.0382


def ghia_bc(f):
    from cfd_amd import api
    api.cavity_bc(f, 1.0)
