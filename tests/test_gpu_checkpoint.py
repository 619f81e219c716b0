"""Restart files of the device-resident state (hip_proj_checkpoint_write/read,
hip_proj_field_crc32) against the format oracle
(oracle/checkpoint_format.py: struct + zlib) and the reference's restart
contract (tests/io/test_checkpoint.c:169-233: N steps + checkpoint + M steps
equals N + M steps bit for bit). Runs on an MI355X."""
import ctypes as C
import zlib

import numpy as np
import pytest

from cfd_amd import _abi as A
from cfd_amd import _native, api
from oracle import checkpoint_format as fmt
from tests import cases
from tests.test_checkpoint import grid_dict, nondefault_params, params_dict

pytestmark = pytest.mark.gpu

F = {"u": A.HIP_FIELD_U, "v": A.HIP_FIELD_V, "w": A.HIP_FIELD_W, "p": A.HIP_FIELD_P,
     "T": A.HIP_FIELD_T}


def _loaded(g, f, **cfg):
    ctx = api.HipProjection(g.nx, g.ny, g.nz, **cfg)
    for k, fid in F.items():
        ctx.set_field(fid, getattr(f, k))
    ctx.set_density(float(f.rho.flat[0]))
    return ctx


@pytest.mark.parametrize("shape", [(33, 33, 33), (17, 9, 5), (130, 70, 3), (64, 64, 1)])
def test_device_crc32_matches_zlib(hip_lib, shape):
    """GPU CRC of the packed field (wave-strided registers, lane/chunk shifts,
    XOR combine) equals zlib.crc32 of the same bytes, for rows shorter and
    longer than a wavefront and chunk tails."""
    nx, ny, nz = shape
    rng = np.random.default_rng(nx * ny * nz)
    ctx = api.HipProjection(nx, ny, nz)
    a = rng.standard_normal((nz, ny, nx))
    ctx.set_field(A.HIP_FIELD_U, a)
    assert ctx.field_crc32(A.HIP_FIELD_U) == zlib.crc32(np.ascontiguousarray(a).tobytes())
    ctx.close()


def test_device_crc32_large_multichunk(hip_lib):
    """256^3: 2048 chunks of 8192 values joined by x^(8d) shifts and an XOR."""
    n = 256
    ctx = api.HipProjection(n, n, n)
    a = np.random.default_rng(1).standard_normal((n, n, n))
    ctx.set_field(A.HIP_FIELD_P, a)
    assert ctx.field_crc32(A.HIP_FIELD_P) == zlib.crc32(a.tobytes())
    ctx.close()


def test_device_write_matches_format_and_host_writer(hip_lib, tmp_path):
    g, f, _ = cases.tg3(17)
    f.T[...] = np.random.default_rng(3).standard_normal(f.T.shape) + 300.0
    ctx = _loaded(g, f)
    p = nondefault_params()
    dev = str(tmp_path / "dev.cfdchk")
    host = str(tmp_path / "host.cfdchk")
    assert ctx.checkpoint_write(dev, g, p, 3.5, "projection_hip", "run7", "/out") == A.CFD_SUCCESS
    data = open(dev, "rb").read()
    d = fmt.decode(data)
    assert d["crc_ok"] is True
    for k, fid in F.items():
        assert np.array_equal(d["fields"][k], ctx.get_field(fid)), k
    assert np.all(d["fields"]["rho"] == 1.0)
    assert (d["solver"], d["prefix"], d["base"], d["time"]) == (b"projection_hip", b"run7", b"/out", 3.5)
    # the host writer, given the same arrays, produces the identical file
    assert api.checkpoint_write(host, g, f, p, 3.5, "projection_hip", "run7", "/out") == 0
    assert open(host, "rb").read() == data
    ctx.close()


def test_device_read_and_reject_corruption(hip_lib, tmp_path):
    g, f, _ = cases.tg3(17)
    f.T[...] = 290.0 + np.arange(f.T.size).reshape(f.T.shape) * 1e-3
    p = nondefault_params()
    path = str(tmp_path / "h.cfdchk")
    assert api.checkpoint_write(path, g, f, p, 9.0, "projection_hip", None, "/b") == 0
    ctx = api.HipProjection(17, 17, 17)
    st, g2, p2, t2, name, prefix, base = ctx.checkpoint_read(path)
    assert st == A.CFD_SUCCESS and (t2, name, prefix, base) == (9.0, "projection_hip", "", "/b")
    for k, fid in F.items():
        assert np.array_equal(ctx.get_field(fid), getattr(f, k)), k
    for k, v in grid_dict(g).items():
        assert np.array_equal(np.asarray(grid_dict(g2)[k]), np.asarray(v)), k
    assert params_dict(p2) == params_dict(p)
    before = {k: ctx.get_field(fid) for k, fid in F.items()}
    data = open(path, "rb").read()
    for name, off in fmt.field_offsets(data).items():
        bad = bytearray(data)
        bad[off + 8 * 100 + 3] ^= 0x10
        open(path, "wb").write(bytes(bad))
        assert ctx.checkpoint_read(path)[0] == A.CFD_ERROR_IO, name
        for k, fid in F.items():  # a rejected file leaves the device state alone
            assert np.array_equal(ctx.get_field(fid), before[k]), (name, k)
    open(path, "wb").write(data[: len(data) // 3])
    assert ctx.checkpoint_read(path)[0] == A.CFD_ERROR_IO
    other = str(tmp_path / "o.cfdchk")
    g9, f9, _ = cases.tg3(9)
    assert api.checkpoint_write(other, g9, f9, p, 0.0, "projection_hip") == 0
    assert ctx.checkpoint_read(other)[0] == A.CFD_ERROR_INVALID  # dimensions are the context's
    ctx.close()


@pytest.mark.parametrize("case", ["tg", "cavity"])
def test_restart_continuity_device(hip_lib, tmp_path, case):
    """test_checkpoint.c:169-222 on the device path: N steps, checkpoint, M
    steps in a fresh context from the file == N + M steps, bit for bit."""
    if case == "tg":
        g, f, p = cases.tg3(17)
        bc = lambda c: [c.apply_scalar_bc(fid, A.BC_TYPE_PERIODIC) for fid in  # noqa: E731
                        (A.HIP_FIELD_U, A.HIP_FIELD_V, A.HIP_FIELD_W, A.HIP_FIELD_P)]
    else:
        g, f, p = cases.cavity(17, 17, 17, Re=100.0, dt=5e-4)

        def bc(c):
            c.apply_dirichlet(A.HIP_FIELD_U, api.dirichlet(top=1.0))
            c.apply_dirichlet(A.HIP_FIELD_V, api.dirichlet())
            c.apply_dirichlet(A.HIP_FIELD_W, api.dirichlet())
            c.apply_scalar_bc(A.HIP_FIELD_P, A.BC_TYPE_NEUMANN)
    N, M = 3, 4
    path = str(tmp_path / "r.cfdchk")
    a = _loaded(g, f)
    for i in range(N + M):
        if i == N:
            assert a.checkpoint_write(path, g, p, N * p.dt, "projection_hip") == A.CFD_SUCCESS
        bc(a)
        assert a.step_device(g, p) == A.CFD_SUCCESS
    b = api.HipProjection(g.nx, g.ny, g.nz)
    st, _, p2, t2, *_ = b.checkpoint_read(path)
    assert st == A.CFD_SUCCESS and t2 == N * p.dt
    for _ in range(M):
        bc(b)
        assert b.step_device(g, p2) == A.CFD_SUCCESS
    for k, fid in F.items():
        if k == "T":
            continue
        assert np.array_equal(a.get_field(fid), b.get_field(fid)), k
    a.close()
    b.close()


def test_simulation_save_load_restart_projection_hip(hip_lib, tmp_path):
    """save_simulation_checkpoint / load_simulation_from_checkpoint /
    restore_simulation_checkpoint (simulation_api.c:257-440) with the
    projection_hip plugin driving run_simulation_step: bitwise continuation."""
    h = _native.host()
    _native.hip()
    path = str(tmp_path / "sim.cfdchk").encode()

    def new_sim():
        s = h.init_simulation_with_solver(17, 17, 17, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0,
                                          b"projection_hip")
        assert s, _native.last_error()
        return s

    def arrays(s):
        c = s.contents.field.contents
        n = c.nx * c.ny * c.nz
        return {k: np.ctypeslib.as_array(getattr(c, k), (n,)).copy() for k in ("u", "v", "w", "p")}

    a = new_sim()
    for _ in range(2):
        assert h.run_simulation_step(a) == A.CFD_SUCCESS
    assert h.save_simulation_checkpoint(a, path) == A.CFD_SUCCESS
    for _ in range(3):
        assert h.run_simulation_step(a) == A.CFD_SUCCESS
    b = h.load_simulation_from_checkpoint(path)
    assert b, _native.last_error()
    assert b.contents.solver.contents.name == b"projection_hip"
    assert b.contents.current_time == pytest.approx(2 * 0.005)
    for _ in range(3):
        assert h.run_simulation_step(b) == A.CFD_SUCCESS
    fa, fb = arrays(a), arrays(b)
    for k in fa:
        assert np.array_equal(fa[k], fb[k]), k
    c = new_sim()
    assert h.restore_simulation_checkpoint(c, path) == A.CFD_SUCCESS
    for _ in range(3):
        assert h.run_simulation_step(c) == A.CFD_SUCCESS
    fc = arrays(c)
    for k in fa:
        assert np.array_equal(fa[k], fc[k]), k
    for s in (a, b, c):
        h.free_simulation(s)
