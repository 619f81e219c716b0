"""Resident mode of the host-buffer step (hip_proj_config_t.dirty_faces,
SURVEY.md:449-455): the interior stays in HBM, a step
uploads the boundary shell the caller's BC routine wrote and downloads the
two outer layers it reads. Against the full-transfer step on the reference's
drivers, the caller re-applying its BCs on the host before every step:

  - 3-D lid-driven cavity (lid_driven_cavity_common.h:306-308),
  - Taylor-Green with periodic BCs (taylor_green_3d_reference.h:297-313),
  - buoyancy + energy with device thermal BCs (T in the shell too),

bit for bit: every step's stats and the depth-2 shell of every field, and all
cells after hip_proj_sync_host / at the sync interval. Also: the interior
really is left stale between syncs, a new host array or a device-side entry
in between falls back to a full upload, a failed step hands back the whole
field, and the plugin's CFD_HIP_DIRTY_FACES switch.
"""
import numpy as np
import pytest

from cfd_amd import _abi as A
from cfd_amd import api
from tests import cases
from tests.test_gpu_energy import _convection_case

pytestmark = pytest.mark.gpu

FIELDS = ("u", "v", "w", "p", "T")


def _shell_mask(shape, depth=2):
    nz, ny, nx = shape
    m = np.zeros(shape, bool)
    m[:, :, :depth] = m[:, :, nx - depth:] = True
    m[:, :depth, :] = m[:, ny - depth:, :] = True
    if nz > 1:
        m[:depth] = m[nz - depth:] = True
    return m


def _clone(g, f):
    f2 = api.FlowField(g.nx, g.ny, g.nz)
    f2.copy_from(f)
    return f2


def _run(g, f, p, n, bc, **cfg):
    """n host-buffer steps with bc(f) on the host before each; returns the
    per-step (status, stats, field copies) and the context (open)."""
    ctx = api.HipProjection(g.nx, g.ny, g.nz, **cfg)
    out = []
    for _ in range(n):
        bc(f)
        st = A.SolverStats()
        s = ctx.step(f, g, p, st)
        out.append((s, (st.max_velocity, st.max_pressure, st.max_temperature),
                    {k: getattr(f, k).copy() for k in FIELDS}))
    return out, ctx


def _cavity_bc(f):
    api.cavity_bc(f, 1.0)


CASES = {
    "cavity": (lambda: cases.cavity(33, 29, 21, Re=100.0, dt=5e-4), _cavity_bc),
    "taylor_green": (lambda: cases.tg3(24), cases.tg3_bc),
    "convection": (lambda: _convection_case(19, 17, 13), lambda f: None),
}


@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("method", [A.HIP_POISSON_CG, A.HIP_POISSON_REDBLACK])
def test_resident_steps_bitwise(hip_lib, name, method):
    build, bc = CASES[name]
    g, f, p = build()
    fr = _clone(g, f)
    # RB-SOR: a capped solve that continues (the Neumann problems stall above 1e-6)
    tol = {} if method == A.HIP_POISSON_CG else dict(poisson_max_iter=300, poisson_fail_fatal=0)
    full, cf = _run(g, f, p, 5, bc, poisson_method=method, **tol)
    res, cr = _run(g, fr, p, 5, bc, poisson_method=method, dirty_faces=1, **tol)
    m = _shell_mask(f.u.shape)
    stale = False
    for (sf, stf, ff), (sr, str_, fr_) in zip(full, res):
        assert sf == sr == A.CFD_SUCCESS
        assert stf == str_
        for k in FIELDS:
            np.testing.assert_array_equal(fr_[k][m], ff[k][m], err_msg=k)
        stale = stale or not np.array_equal(fr_["u"], ff["u"])
    assert stale, "the interior was transferred: resident mode not active"
    cr.sync_host(fr)
    for k in FIELDS:
        np.testing.assert_array_equal(getattr(fr, k), getattr(f, k), err_msg=k)
    cf.close()
    cr.close()


def test_sync_interval(hip_lib):
    g, f, p = cases.cavity(25, 23, 19)
    fr = _clone(g, f)
    full, cf = _run(g, f, p, 6, _cavity_bc)
    res, cr = _run(g, fr, p, 6, _cavity_bc, dirty_faces=1, dirty_sync_interval=3)
    for step in (2, 5):  # the 3rd and 6th steps download in full
        for k in FIELDS:
            np.testing.assert_array_equal(res[step][2][k], full[step][2][k], err_msg=k)
    assert not np.array_equal(res[3][2]["u"], full[3][2]["u"])
    cf.close()
    cr.close()


def test_new_host_arrays_and_device_entries_fall_back(hip_lib):
    """Handing over a different flow_field, or a device-side entry between
    two steps (here hip_proj_set_field overwriting u), makes the next step
    upload in full: results stay equal to the full-transfer path."""
    g, f, p = cases.cavity(21, 19, 17)
    ff, f1 = _clone(g, f), _clone(g, f)
    cf = api.HipProjection(g.nx, g.ny, g.nz)
    cr = api.HipProjection(g.nx, g.ny, g.nz, dirty_faces=1)
    bump = 1e-3 * np.random.default_rng(5).standard_normal(f.u.shape)
    for step in range(5):
        if step == 2:
            # both sides continue on new host arrays with a changed interior
            cr.sync_host(f1)
            ff, f1 = _clone(g, ff), _clone(g, f1)
            ff.u[...] += bump
            f1.u[...] += bump
        if step == 3:
            # the documented order: make the host current, then a device entry
            cr.sync_host(f1)
            cr.set_field(A.HIP_FIELD_U, np.zeros(f.u.shape))
        _cavity_bc(ff)
        assert cf.step(ff, g, p) == A.CFD_SUCCESS
        _cavity_bc(f1)
        assert cr.step(f1, g, p) == A.CFD_SUCCESS, api._native.last_error()
    cr.sync_host(f1)
    for k in FIELDS:
        np.testing.assert_array_equal(getattr(f1, k), getattr(ff, k), err_msg=k)
    cf.close()
    cr.close()


def test_failed_step_returns_whole_field(hip_lib):
    """An unconverged pressure solve (fail-fatal) leaves the host field whole
    and equal to the full-transfer path's."""
    g, f, p = cases.cavity(21, 19, 17)
    fr = _clone(g, f)
    cfg = dict(poisson_max_iter=2, poisson_tolerance=1e-14, poisson_abs_tolerance=0.0)
    full, cf = _run(g, f, p, 2, _cavity_bc, **cfg)
    res, cr = _run(g, fr, p, 2, _cavity_bc, dirty_faces=1, **cfg)
    for (sf, _, ff), (sr, _, fr_) in zip(full, res):
        assert sf == sr == A.CFD_ERROR_MAX_ITER
        for k in FIELDS:
            np.testing.assert_array_equal(fr_[k], ff[k], err_msg=k)
    cf.close()
    cr.close()


@pytest.mark.parametrize("name", ["projection_hip", "projection_hip_cg1"])
def test_plugin_env_switch(hip_lib, monkeypatch, name):
    """CFD_HIP_DIRTY_FACES=N through the registry's `step` (the textbook-CG
    plugin and the single-reduction one): a full download every N steps,
    equal to the same plugin's field without the resident mode."""
    monkeypatch.setenv("CFD_HIP_DIRTY_FACES", "2")
    g, f, p = cases.cavity(21, 19, 17)
    fr = _clone(g, f)
    reg = api.Registry()
    s_res = reg.create(name)
    assert s_res.init(g, p) == A.CFD_SUCCESS
    monkeypatch.delenv("CFD_HIP_DIRTY_FACES")
    s_full = reg.create(name)
    assert s_full.init(g, p) == A.CFD_SUCCESS
    for step in range(4):
        _cavity_bc(f)
        _cavity_bc(fr)
        assert s_full.step(f, g, p) == A.CFD_SUCCESS
        assert s_res.step(fr, g, p) == A.CFD_SUCCESS
        same = all(np.array_equal(getattr(fr, k), getattr(f, k)) for k in FIELDS)
        assert same == (step % 2 == 1), step
    s_res.close()
    s_full.close()


@pytest.mark.parametrize("verify,cell", [(1, (10, 10, 10)), (1, (1, 7, 9)), (2, (10, 10, 10))])
def test_verify_guard_and_mark_host_dirty(hip_lib, verify, cell):
    """dirty_verify_interval: a caller that writes an interior cell of its
    host arrays between resident steps (which the shell upload would ignore)
    gets CFD_ERROR_INVALID from the next verified step, nothing run. The
    supported way -- hip_proj_sync_host, write, hip_proj_mark_host_dirty --
    then gives bitwise the full-transfer run with the same write. Deep cells
    are caught at the next verified step whatever the interval; cell (1, 7, 9)
    is in the layer next to the boundary, which every step's download
    rewrites, caught with interval 1."""
    g, f, p = cases.cavity(33, 29, 21, Re=100.0, dt=5e-4)
    fr = _clone(g, f)
    full = api.HipProjection(g.nx, g.ny, g.nz)
    res = api.HipProjection(g.nx, g.ny, g.nz, dirty_faces=1, dirty_verify_interval=verify)
    try:
        for _ in range(3):
            _cavity_bc(f)
            _cavity_bc(fr)
            assert full.step(f, g, p) == A.CFD_SUCCESS
            assert res.step(fr, g, p) == A.CFD_SUCCESS
        before = fr.u.copy()
        fr.u[cell] += 0.25
        statuses = []
        for _ in range(verify):  # the write is caught within `verify` steps
            _cavity_bc(fr)
            s = res.step(fr, g, p)
            statuses.append(s)
            if s != A.CFD_SUCCESS:
                break
        assert statuses[-1] == A.CFD_ERROR_INVALID, statuses
        assert "interior" in api._native.last_error()
        n_ok = len(statuses) - 1  # verified-free steps that ran before the check
        for _ in range(n_ok):
            _cavity_bc(f)
            assert full.step(f, g, p) == A.CFD_SUCCESS
        # the supported path: sync, write, mark dirty
        res.sync_host(fr)
        for k in FIELDS[:4]:
            np.testing.assert_array_equal(getattr(fr, k), getattr(f, k), err_msg=k)
        f.u[cell] += 0.25
        fr.u[cell] += 0.25
        res.mark_host_dirty()
        for _ in range(2):
            _cavity_bc(f)
            _cavity_bc(fr)
            assert full.step(f, g, p) == A.CFD_SUCCESS
            assert res.step(fr, g, p) == A.CFD_SUCCESS
        res.sync_host(fr)
        for k in FIELDS[:4]:
            np.testing.assert_array_equal(getattr(fr, k), getattr(f, k), err_msg=k)
        assert not np.array_equal(before, fr.u)
    finally:
        full.close()
        res.close()
