"""Z-slab decomposition on the GPU, run as an in-process group
of slab contexts on one device: the same driver code, halo exchanges and
all-reduces the RCCL backend runs one process per GPU, with the transport
replaced by device copies (RCCL refuses two ranks on one GPU).

Parity bars: the relaxation methods have no summation, so a slab run is
bitwise the single-domain oracle; CG dot products are summed per slab and
then across slabs, so CG runs agree to rounding (same bar as the 1-GPU CG)."""
import numpy as np
import pytest

from cfd_amd import _abi as A
from cfd_amd import api
from oracle import oracle
from tests import cases

pytestmark = pytest.mark.gpu

FIELDS = {"u": A.HIP_FIELD_U, "v": A.HIP_FIELD_V, "w": A.HIP_FIELD_W, "p": A.HIP_FIELD_P}


@pytest.fixture(autouse=True)
def _short_group_timeout(monkeypatch):
    monkeypatch.setenv("CFD_HIP_GROUP_TIMEOUT_S", "60")


class Slabs:
    def __init__(self, g, nranks, **cfg):
        self.g = g
        self.group = api.LocalGroup(nranks)
        self.ctx = [api.HipProjection(g.nx, g.ny, g.nz, comm=self.group.comm(r, 0), **cfg)
                    for r in range(nranks)]
        self.n = nranks

    def scatter(self, f):
        for c in self.ctx:
            sl = slice(c.k_offset, c.k_offset + c.nz_local)
            for k, fid in FIELDS.items():
                c.set_field(fid, getattr(f, k)[sl])
            c.set_density(float(f.rho.flat[0]))

    def gather(self, name):
        out = np.full((self.g.nz, self.g.ny, self.g.nx), np.nan)
        for c in self.ctx:
            loc, glob = c.owned()
            out[glob] = c.get_field(FIELDS[name])[loc]
        assert not np.isnan(out).any()
        return out

    def run(self, fn):
        return api.run_ranks(lambda r: fn(r, self.ctx[r]), self.n)

    def close(self):
        for c in self.ctx:
            c.close()
        self.group.close()


def _cavity_bc_device(c):
    c.apply_dirichlet(A.HIP_FIELD_U, api.dirichlet(top=1.0))
    c.apply_dirichlet(A.HIP_FIELD_V, api.dirichlet())
    c.apply_dirichlet(A.HIP_FIELD_W, api.dirichlet())
    c.apply_scalar_bc(A.HIP_FIELD_P, A.BC_TYPE_NEUMANN)


def _tg_bc_device(c):
    for fid in FIELDS.values():
        c.apply_scalar_bc(fid, A.BC_TYPE_PERIODIC)


def _run_steps(S, g, p, n_steps, bc_dev):
    def body(r, c):
        out = []
        for _ in range(n_steps):
            bc_dev(c)
            st = A.SolverStats()
            s = c.step_device(g, p, st)
            assert s == A.CFD_SUCCESS, (r, s, api._native.last_error())
            out.append((c.poisson_stats().iterations, st.max_velocity, st.max_pressure))
        return out
    return S.run(body)


def _oracle_steps(g, f, p, n_steps, bc_host, kind):
    hist = []
    for _ in range(n_steps):
        bc_host(f)
        s, st, it = oracle.projection_step(f, g, p, kind)
        assert s == A.CFD_SUCCESS
        hist.append((it, st.max_velocity, st.max_pressure))
    return hist


@pytest.mark.parametrize("nranks", [2, 3, 4])
def test_slab_layout_covers_interior(hip_lib, nranks):
    nz = 17
    spans = [api.slab_layout(nz, r, nranks) for r in range(nranks)]
    owned = []
    for ko, nl in spans:
        owned += list(range(ko + 1, ko + nl - 1))
    assert owned == list(range(1, nz - 1))
    assert max(nl for _, nl in spans) - min(nl for _, nl in spans) <= 1


@pytest.mark.parametrize("nranks", [2, 3])
@pytest.mark.parametrize("bc", ["neumann", "periodic"])
def test_slab_scalar_bc_bitwise(hip_lib, nranks, bc):
    """Device BCs on slabs (z faces on the edge ranks; periodic z as the
    wrap-around exchange) equal the reference's host BC on the whole field."""
    nx, ny, nz = 17, 13, 11
    rng = np.random.default_rng(11)
    ref = rng.standard_normal((nz, ny, nx))
    g = api.Grid(nx, ny, nz, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0)
    f = api.FlowField(nx, ny, nz)
    f.p[...] = ref
    f.u[...] = f.v[...] = f.w[...] = 0.0
    f.rho[...] = 1.0
    S = Slabs(g, nranks)
    try:
        S.scatter(f)
        t = A.BC_TYPE_NEUMANN if bc == "neumann" else A.BC_TYPE_PERIODIC
        S.run(lambda r, c: c.apply_scalar_bc(A.HIP_FIELD_P, t))
        got = S.gather("p")
    finally:
        S.close()
    want = ref.copy()
    api.bc_apply_scalar_3d(want, t)
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("method,nranks", [(A.HIP_POISSON_REDBLACK, 2),
                                           (A.HIP_POISSON_REDBLACK, 4),
                                           (A.HIP_POISSON_JACOBI, 3)])
def test_slab_relaxation_projection_bitwise(hip_lib, method, nranks):
    """RB-SOR (global colour parity, halo after each colour) and Jacobi on
    slabs: bitwise the single-domain oracle, iteration counts included."""
    g, f, p = cases.cavity(17, 17, 17, Re=100.0, dt=5e-4)
    maxit = 2000 if method == A.HIP_POISSON_JACOBI else 5000
    okind = (A.ORACLE_POISSON_REDBLACK if method == A.HIP_POISSON_REDBLACK
             else A.ORACLE_POISSON_JACOBI)
    S = Slabs(g, nranks, poisson_method=method, poisson_tolerance=1e-2, poisson_max_iter=maxit)
    try:
        S.scatter(f)
        hist = _run_steps(S, g, p, 3, _cavity_bc_device)
        got = {k: S.gather(k) for k in FIELDS}
    finally:
        S.close()
    oracle.set_projection_poisson_params(
        oracle.poisson_params(tolerance=1e-2, max_iterations=maxit))
    try:
        ohist = _oracle_steps(g, f, p, 3, lambda ff: api.cavity_bc(ff, 1.0), okind)
    finally:
        oracle.set_projection_poisson_params(None)
    for r in range(nranks):
        assert hist[r] == ohist, (r, hist[r], ohist)
    for k in FIELDS:
        np.testing.assert_array_equal(got[k], getattr(f, k), err_msg=k)


@pytest.mark.parametrize("nranks", [2, 4])
def test_slab_cg_cavity_vs_oracle(hip_lib, nranks):
    g, f, p = cases.cavity(33, 33, 33, Re=100.0, dt=5e-4)
    S = Slabs(g, nranks)
    try:
        S.scatter(f)
        hist = _run_steps(S, g, p, 4, _cavity_bc_device)
        got = {k: S.gather(k) for k in FIELDS}
    finally:
        S.close()
    ohist = _oracle_steps(g, f, p, 4, lambda ff: api.cavity_bc(ff, 1.0), A.ORACLE_POISSON_CG)
    for r in range(nranks):
        assert hist[r] == hist[0]  # every rank holds the same all-reduced state
    for (ih, vh, ph), (io, vo, po) in zip(hist[0], ohist):
        assert abs(ih - io) <= 1
        assert vh == pytest.approx(vo, rel=1e-9)
        assert ph == pytest.approx(po, rel=1e-9)
    for k in FIELDS:
        ref = getattr(f, k)
        scale = max(1.0, float(np.max(np.abs(ref))))
        assert float(np.max(np.abs(got[k] - ref))) / scale <= 1e-10, k


@pytest.mark.parametrize("nranks,n", [(2, 17), (3, 17), (8, 33)])
def test_slab_taylor_green_vs_oracle(hip_lib, nranks, n):
    """Config 4 at test size: periodic BCs across the slab boundary every step
    (with 2 ranks both neighbours of each rank are the same peer; 8 ranks is
    the configs[3] decomposition)."""
    g, f, p = cases.tg3(n)
    S = Slabs(g, nranks)
    try:
        S.scatter(f)
        _run_steps(S, g, p, 5, _tg_bc_device)
        got = {k: S.gather(k) for k in FIELDS}
    finally:
        S.close()
    _oracle_steps(g, f, p, 5, cases.tg3_bc, A.ORACLE_POISSON_CG)
    for k in FIELDS:
        ref = getattr(f, k)
        scale = max(1.0, float(np.max(np.abs(ref))))
        assert float(np.max(np.abs(got[k] - ref))) / scale <= 1e-10, k


def _slab_poisson(g, rhs, nranks, method, prm=None, check_halo=False, **cfg):
    S = Slabs(g, nranks, **cfg)
    try:
        def body(r, c):
            sl = slice(c.k_offset, c.k_offset + c.nz_local)
            x = np.zeros(c.shape)
            s, st = c.poisson_solve(method, x, rhs[sl], g.dx, g.dy, g.dz, prm)
            return s, st.iterations, x
        res = S.run(body)
        x = np.full(rhs.shape, np.nan)
        for c, (s, it, xl) in zip(S.ctx, res):
            loc, glob = c.owned()
            x[glob] = xl[loc]
        if check_halo:  # halo planes hold the neighbours' final owned planes
            for c, (s, it, xl) in zip(S.ctx, res):
                np.testing.assert_array_equal(xl, x[c.k_offset:c.k_offset + c.nz_local])
    finally:
        S.close()
    assert not np.isnan(x).any()
    return [r[0] for r in res], [r[1] for r in res], x


def test_slab_poisson_cg_vs_oracle(hip_lib):
    """Standalone slab CG: the reference's iteration count and demeaned gate."""
    g, rhs = cases.cos_rhs(33)
    xo = np.zeros_like(rhs)
    so, sto = oracle.cg_solve(xo, rhs, g.dx, g.dy, g.dz)
    stat, its, x = _slab_poisson(g, rhs, 3, A.HIP_POISSON_CG)
    assert so == A.CFD_SUCCESS and all(s == A.CFD_SUCCESS for s in stat)
    assert len(set(its)) == 1 and abs(its[0] - sto.iterations) <= 1
    d = (x - x.mean()) - (xo - xo.mean())
    assert np.max(np.abs(d)) / np.max(np.abs(xo)) < 1e-9


@pytest.mark.parametrize("method", [A.HIP_POISSON_REDBLACK, A.HIP_POISSON_JACOBI])
@pytest.mark.parametrize("nranks,two_pass,maxit,split", [
    (4, 0, None, "1"), (4, 1, None, "1"), (4, 2, None, "1"), (2, 0, None, "1"),
    (3, 0, 11, "1"), (2, 0, None, "0"), (3, 0, 11, "0")])
def test_slab_poisson_relax_bitwise(hip_lib, monkeypatch, method, nranks, two_pass, maxit,
                                    split):
    """Slab RB-SOR / Jacobi, fused device loop (residual max across ranks) and
    two-pass form: bitwise the oracle, iteration counts and status included;
    every rank's halo planes end equal to the neighbours' owned planes.
    RB-SOR: relax_two_pass 0 = one pass per iteration (k_rb_edge_r, R halo,
    k_rb1<DIST>), 2 = the two colour sweeps of k_rx, 1 = the unfused form.
    The one-pass form on a slab of >= 4 planes runs as three launches (the
    interior halves overlap the R and Y exchanges on the side stream, the
    edge planes in between; CFD_HIP_RB_SPLIT=0: one launch between blocking
    exchanges); 17^3 over 4 ranks mixes 4- and 3-plane slabs."""
    monkeypatch.setenv("CFD_HIP_RB_SPLIT", split)
    g, rhs = cases.cos_rhs(17)
    xo = np.zeros_like(rhs)
    if maxit is None:
        maxit = 3000 if method == A.HIP_POISSON_JACOBI else 5000
    prm = oracle.poisson_params(max_iterations=maxit)
    if method == A.HIP_POISSON_REDBLACK:
        so, sto = oracle.redblack_solve(xo, rhs, g.dx, g.dy, g.dz, prm)
    else:
        so, sto = oracle.jacobi_solve(xo, rhs, g.dx, g.dy, g.dz, prm)
    stat, its, x = _slab_poisson(g, rhs, nranks, method, prm, check_halo=True,
                                 relax_two_pass=two_pass)
    assert all(s == so for s in stat)
    assert all(i == sto.iterations for i in its)
    np.testing.assert_array_equal(x, xo)


@pytest.fixture()
def omp_oracle():
    import os
    n = len(os.sched_getaffinity(0))
    env = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    oracle.set_threads(max(1, min(n, env) if env > 0 else n))
    yield
    oracle.set_threads(1)


DEPTH_N = 130  # 128 interior planes: 16 per rank at 8 ranks


def test_slab8_taylor_green_depth_vs_oracle(hip_lib, omp_oracle):
    """8 ranks at a realistic slab depth (130^3: 16 planes each), so the CG's
    split sweep B (edge planes + interior), the r halo on the side stream and
    the x fold run on real slab interiors: fields within 1e-10 of the oracle,
    CG iterations within 1 per step."""
    g, f, p = cases.tg3(DEPTH_N)
    S = Slabs(g, 8)
    try:
        S.scatter(f)
        hist = _run_steps(S, g, p, 2, _tg_bc_device)
        got = {k: S.gather(k) for k in FIELDS}
    finally:
        S.close()
    ohist = _oracle_steps(g, f, p, 2, cases.tg3_bc, A.ORACLE_POISSON_CG)
    for r in range(8):
        assert hist[r] == hist[0]
    for (ih, _, _), (io, _, _) in zip(hist[0], ohist):
        assert ih > 50 and abs(ih - io) <= 1, (ih, io)
    for k in FIELDS:
        ref = getattr(f, k)
        scale = max(1.0, float(np.max(np.abs(ref))))
        assert float(np.max(np.abs(got[k] - ref))) / scale <= 1e-10, k


@pytest.mark.parametrize("split", ["1", "0"])
def test_slab8_cavity_rbsor_depth_bitwise(hip_lib, omp_oracle, monkeypatch, split):
    """8 ranks at 130^3 with the one-pass RB-SOR: the three-launch iteration
    (interior halves overlapping the R / Y exchanges) on 16-plane slabs,
    bitwise the oracle's red-black SOR step, iteration counts included."""
    monkeypatch.setenv("CFD_HIP_RB_SPLIT", split)
    g, f, p = cases.cavity(DEPTH_N, DEPTH_N, DEPTH_N, Re=100.0, dt=5e-4)
    tol = 1e-3
    S = Slabs(g, 8, poisson_method=A.HIP_POISSON_REDBLACK, poisson_tolerance=tol,
              poisson_max_iter=5000)
    try:
        S.scatter(f)
        hist = _run_steps(S, g, p, 2, _cavity_bc_device)
        got = {k: S.gather(k) for k in FIELDS}
    finally:
        S.close()
    oracle.set_projection_poisson_params(oracle.poisson_params(tolerance=tol,
                                                               max_iterations=5000))
    try:
        ohist = _oracle_steps(g, f, p, 2, lambda ff: api.cavity_bc(ff, 1.0),
                              A.ORACLE_POISSON_REDBLACK)
    finally:
        oracle.set_projection_poisson_params(None)
    for r in range(8):
        assert hist[r] == ohist, (r, hist[r], ohist)
    assert all(it > 10 for it, _, _ in ohist)
    for k in FIELDS:
        np.testing.assert_array_equal(got[k], getattr(f, k), err_msg=k)


@pytest.mark.timeout(600)
def test_slab8_taylor_green_512_vs_single_device(hip_lib, monkeypatch):
    """BASELINE configs[3] at its own size: 512^3 Taylor-Green on 8
    in-process Z-slabs (6 x 64 + 2 x 63 interior planes, the periodic z wrap
    as the exchange between ranks 0 and 7) against one context on the same
    device, 2 steps with the periodic BCs before each step
    (taylor_green_3d_reference.h:177-404). Gates:
    identical CG iteration counts, the relative L2 errors of u and v against
    the analytic decay equal within 1e-10 relative, and the fields within
    1e-10 of their scale."""
    monkeypatch.setenv("CFD_HIP_GROUP_TIMEOUT_S", "120")
    n, steps = 512, 2
    g, f, p = cases.tg3(n)
    one = api.HipProjection(n, n, n)
    try:
        for k, fid in FIELDS.items():
            one.set_field(fid, getattr(f, k))
        one.set_density(1.0)
        its1 = []
        for _ in range(steps):
            _tg_bc_device(one)
            assert one.step_device(g, p) == A.CFD_SUCCESS, api._native.last_error()
            its1.append(one.poisson_stats().iterations)
        ref = {k: one.get_field(fid) for k, fid in FIELDS.items()}
    finally:
        one.close()
    S = Slabs(g, 8)
    try:
        assert [c.nz_local - 2 for c in S.ctx] == [64] * 6 + [63] * 2
        S.scatter(f)
        hist = _run_steps(S, g, p, steps, _tg_bc_device)
        got = {k: S.gather(k) for k in FIELDS}
    finally:
        S.close()
    for r in range(8):
        assert [h[0] for h in hist[r]] == its1, (r, hist[r], its1)
    assert all(i > 100 for i in its1)
    t = steps * p.dt
    for k in FIELDS:
        f_k = getattr(f, k)
        f_k[...] = ref[k]
    e1 = cases.tg3_l2_errors(g, f, t)
    for k in FIELDS:
        getattr(f, k)[...] = got[k]
    eN = cases.tg3_l2_errors(g, f, t)
    for a, b in zip(e1, eN):
        assert b == pytest.approx(a, rel=1e-10), (e1, eN)
    for k in FIELDS:
        scale = max(1.0, float(np.max(np.abs(ref[k]))))
        assert float(np.max(np.abs(got[k] - ref[k]))) / scale <= 1e-10, k
    print("tg512 on 8 slabs: CG iterations", its1, "L2 errors (1 device, 8 slabs)", e1, eN)
