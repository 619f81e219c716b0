"""Legacy VTK output: the host mirror's writers restate
lib/src/io/vtk_output.c:110-275 and are checked against an independent Python
rendering of the same text, plus the assertions of the reference's
tests/io/test_vtk_output.c (headers, field names, NULL safety). The GPU test
writes the HBM-resident state with hip_proj_write_vtk and compares bytes."""
import ctypes as C

import numpy as np
import pytest

from cfd_amd import _abi as A
from cfd_amd import _native, api


def _header(title, nx, ny, nz, xmin, xmax, ymin, ymax, zmin, zmax):
    dz = (zmax - zmin) / (nz - 1) if nz > 1 else 1.0
    return ("# vtk DataFile Version 3.0\n%s\nASCII\nDATASET STRUCTURED_POINTS\n"
            "DIMENSIONS %d %d %d\nORIGIN %f %f %f\nSPACING %f %f %f\n"
            % (title, nx, ny, nz, xmin, ymin, zmin, (xmax - xmin) / (nx - 1),
               (ymax - ymin) / (ny - 1), dz))


def _scalars(name, a):
    return "SCALARS %s float 1\nLOOKUP_TABLE default\n" % name + \
        "".join("%f\n" % v for v in a.ravel())


def expected_flow_field(f, nx, ny, nz, box):
    n = nx * ny * nz
    t = _header("CFD Framework Flow Field Output", nx, ny, nz, *box)
    t += "\nPOINT_DATA %d\nVECTORS velocity float\n" % n
    t += "".join("%f %f %f\n" % q for q in zip(f.u.ravel(), f.v.ravel(), f.w.ravel()))
    for name, a in (("pressure", f.p), ("density", f.rho), ("temperature", f.T)):
        t += "\n" + _scalars(name, a)
    return t


def _field(nx, ny, nz, seed=3):
    rng = np.random.default_rng(seed)
    f = api.FlowField(nx, ny, nz)
    for k in ("u", "v", "w", "p", "rho", "T"):
        getattr(f, k)[...] = rng.standard_normal((nz, ny, nx)) * 10.0 ** rng.integers(-3, 4)
    return f


def test_write_vtk_flow_field_text(tmp_path):
    """write_vtk_flow_field (vtk_output.c:196-275) byte for byte."""
    host = _native.host()
    nx, ny, nz, box = 7, 5, 4, (0.0, 2.0, -1.0, 1.0, 0.5, 3.5)
    f = _field(nx, ny, nz)
    path = tmp_path / "flow.vtk"
    host.write_vtk_flow_field(str(path).encode(), f.ptr, nx, ny, nz, *box)
    text = path.read_text()
    assert text == expected_flow_field(f, nx, ny, nz, box)
    for tag in ("VECTORS velocity", "SCALARS pressure", "SCALARS density",
                "SCALARS temperature"):  # test_vtk_output.c:197-210
        assert tag in text


def test_write_vtk_scalar_and_vector_text(tmp_path):
    """write_vtk_output / write_vtk_vector_output (vtk_output.c:110-190), 2-D
    (nz = 1: SPACING z = 1) and with w = NULL."""
    host = _native.host()
    nx, ny, nz, box = 6, 4, 1, (0.0, 1.0, 0.0, 1.0, 0.0, 0.0)
    f = _field(nx, ny, nz, seed=5)
    p1 = tmp_path / "s.vtk"
    host.write_vtk_output(str(p1).encode(), b"velocity_u", f.u.ctypes.data_as(A.c_double_p),
                          nx, ny, nz, *box)
    exp = _header("CFD Framework Output", nx, ny, nz, *box) + \
        "\nPOINT_DATA %d\n" % (nx * ny) + _scalars("velocity_u", f.u)
    assert p1.read_text() == exp
    p2 = tmp_path / "v.vtk"
    host.write_vtk_vector_output(str(p2).encode(), b"velocity", f.u.ctypes.data_as(A.c_double_p),
                                 f.v.ctypes.data_as(A.c_double_p), None, nx, ny, nz, *box)
    exp = _header("CFD Framework Vector Output", nx, ny, nz, *box) + \
        "\nPOINT_DATA %d\nVECTORS velocity float\n" % (nx * ny) + \
        "".join("%f %f %f\n" % (a, b, 0.0) for a, b in zip(f.u.ravel(), f.v.ravel()))
    assert p2.read_text() == exp


def test_write_vtk_null_safety(tmp_path):
    """test_vtk_output.c:219-256: invalid arguments write no file."""
    host = _native.host()
    f = _field(10, 10, 1)
    path = tmp_path / "none.vtk"
    b = str(path).encode()
    u = f.u.ctypes.data_as(A.c_double_p)
    host.write_vtk_output(None, b"t", u, 10, 10, 1, 0, 1, 0, 1, 0.0, 0.0)
    host.write_vtk_output(b, None, u, 10, 10, 1, 0, 1, 0, 1, 0.0, 0.0)
    host.write_vtk_output(b, b"t", None, 10, 10, 1, 0, 1, 0, 1, 0.0, 0.0)
    host.write_vtk_output(b, b"t", u, 10, 10, 1, 1, 0, 0, 1, 0.0, 0.0)   # xmax <= xmin
    host.write_vtk_vector_output(b, b"v", u, None, None, 10, 10, 1, 0, 1, 0, 1, 0.0, 0.0)
    host.write_vtk_flow_field(b, None, 10, 10, 1, 0, 1, 0, 1, 0.0, 0.0)
    host.write_vtk_flow_field(b, f.ptr, 10, 10, 3, 0, 1, 0, 1, 0.0, 0.0)  # nz > 1, zmax <= zmin
    assert not path.exists()


@pytest.mark.gpu
def test_hip_proj_write_vtk_matches_host_writer(hip_lib, tmp_path):
    """The resident state written from HBM == write_vtk_flow_field of the same
    fields on the host (rho: the constant rho0, T resident)."""
    host = _native.host()
    nx, ny, nz = 9, 7, 5
    g = api.Grid(nx, ny, nz, 0.0, 1.0, 0.0, 2.0, 0.0, 0.5)
    f = _field(nx, ny, nz, seed=11)
    f.rho[...] = 1.25
    ctx = api.HipProjection(nx, ny, nz)
    assert hip_lib.hip_proj_upload(ctx.ctx, f.ptr) == A.CFD_SUCCESS
    p_dev = tmp_path / "dev.vtk"
    assert hip_lib.hip_proj_write_vtk(ctx.ctx, str(p_dev).encode(), g.ptr, 1.25) == A.CFD_SUCCESS
    g2 = api.Grid(nx + 1, ny, nz, 0.0, 1.0, 0.0, 2.0, 0.0, 0.5)
    assert hip_lib.hip_proj_write_vtk(ctx.ctx, str(tmp_path / "x.vtk").encode(), g2.ptr,
                                      1.0) == A.CFD_ERROR_INVALID
    ctx.close()
    p_host = tmp_path / "host.vtk"
    host.write_vtk_flow_field(str(p_host).encode(), f.ptr, nx, ny, nz, 0.0, 1.0, 0.0, 2.0, 0.0, 0.5)
    assert p_dev.read_bytes() == p_host.read_bytes()
