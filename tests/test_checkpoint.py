"""Restart files on the host (libcfd_host.so cfd_checkpoint_write/read), checked
against the independent format restatement in oracle/checkpoint_format.py
(struct + zlib, citing lib/src/io/checkpoint.c) and against the reference's
own test cases (tests/io/test_checkpoint.c: round trips, bad version, bad
magic, truncation, CRC corruption, caller buffers). CPU only."""
import ctypes as C
import zlib

import numpy as np
import pytest

from cfd_amd import _abi as A
from cfd_amd import api
from oracle import checkpoint_format as fmt


def nondefault_params():
    """Every scalar field away from its default (test_checkpoint.c make_nondefault_params)."""
    p = api.params_default()
    p.dt, p.cfl, p.gamma, p.mu, p.k = 2.5e-4, 0.33, 1.31, 7.5e-3, 0.021
    p.max_iter = 37
    p.tolerance = 3e-7
    p.source_amplitude_u, p.source_amplitude_v, p.source_decay_rate = 0.2, -0.07, 0.45
    p.pressure_coupling = 0.17
    p.alpha, p.beta, p.T_ref = 1.4e-4, 3.3e-3, 301.5
    p.gravity[0], p.gravity[1], p.gravity[2] = 0.0, -9.81, 0.5
    t = p.thermal_bc
    t.left, t.right = A.BC_TYPE_DIRICHLET, A.BC_TYPE_DIRICHLET
    t.bottom, t.top, t.front, t.back = (A.BC_TYPE_NEUMANN, A.BC_TYPE_NEUMANN,
                                        A.BC_TYPE_PERIODIC, A.BC_TYPE_PERIODIC)
    d = t.dirichlet_values
    d.left, d.right, d.top, d.bottom, d.front, d.back = 310.0, 290.0, 1.0, 2.0, 3.0, 4.0
    return p


def params_dict(p):
    t, d = p.thermal_bc, p.thermal_bc.dirichlet_values
    return {"dt": p.dt, "cfl": p.cfl, "gamma": p.gamma, "mu": p.mu, "k": p.k,
            "max_iter": p.max_iter, "tolerance": p.tolerance,
            "source_amplitude_u": p.source_amplitude_u,
            "source_amplitude_v": p.source_amplitude_v,
            "source_decay_rate": p.source_decay_rate, "pressure_coupling": p.pressure_coupling,
            "alpha": p.alpha, "beta": p.beta, "T_ref": p.T_ref, "g0": p.gravity[0],
            "g1": p.gravity[1], "g2": p.gravity[2],
            "bc_types": (t.left, t.right, t.bottom, t.top, t.front, t.back),
            "bc_values": (d.left, d.right, d.top, d.bottom, d.front, d.back)}


def grid_dict(g):
    c = g.c
    d = {"nx": g.nx, "ny": g.ny, "nz": g.nz,
         "bounds": (c.xmin, c.xmax, c.ymin, c.ymax, c.zmin, c.zmax),
         "x": np.ctypeslib.as_array(c.x, (g.nx,)).copy(),
         "y": np.ctypeslib.as_array(c.y, (g.ny,)).copy(),
         "dx": np.ctypeslib.as_array(c.dx, (g.nx - 1,)).copy(),
         "dy": np.ctypeslib.as_array(c.dy, (g.ny - 1,)).copy()}
    if g.nz > 1:
        d["z"] = np.ctypeslib.as_array(c.z, (g.nz,)).copy()
        d["dz"] = np.ctypeslib.as_array(c.dz, (g.nz - 1,)).copy()
        d["inv_dz2"] = c.inv_dz2
    return d


def stretch(g, beta=2.0):
    """tanh-stretched coordinates (grid_initialize_stretched's shape), written
    straight into the C arrays: exercises non-uniform x/y/z/dz in the file."""
    c = g.c
    for n, arr, darr, lo, hi in ((g.nx, c.x, c.dx, c.xmin, c.xmax), (g.ny, c.y, c.dy, c.ymin, c.ymax),
                                 (g.nz, c.z, c.dz, c.zmin, c.zmax)):
        s = np.linspace(-1.0, 1.0, n)
        v = lo + (hi - lo) * 0.5 * (1.0 + np.tanh(beta * s) / np.tanh(beta))
        for i in range(n):
            arr[i] = v[i]
        for i in range(n - 1):
            darr[i] = v[i + 1] - v[i]
    c.inv_dz2 = 1.0 / min(c.dz[i] for i in range(g.nz - 1)) ** 2


def known_field(f, seed):
    rng = np.random.default_rng(int(seed * 10))
    for k in api.FlowField.NAMES:
        getattr(f, k)[...] = rng.standard_normal(getattr(f, k).shape) * seed


def assert_params_equal(a, b):
    da, db = params_dict(a), params_dict(b)
    for k in da:
        assert np.array_equal(np.asarray(da[k]), np.asarray(db[k])), k
    assert not b.source_func and not b.heat_source_func


def test_roundtrip_2d_uniform_matches_format(tmp_path):
    """test_checkpoint.c:192-226, plus the oracle's independent parse."""
    path = str(tmp_path / "a.cfdchk")
    g = api.Grid(12, 8, 1, 0.0, 1.0, 0.0, 2.0)
    f = api.FlowField(12, 8, 1)
    known_field(f, 3.0)
    p = nondefault_params()
    assert api.checkpoint_write(path, g, f, p, 1.25, "rk2", "myrun", "/base/dir") == A.CFD_SUCCESS
    data = open(path, "rb").read()
    d = fmt.decode(data)
    assert d["crc_ok"] is True
    assert (d["version"], d["endian"], d["lib_version"], d["flags"]) == (1, 0x01020304, (0, 3, 0), 1)
    assert (d["solver"], d["prefix"], d["base"], d["time"]) == (b"rk2", b"myrun", b"/base/dir", 1.25)
    for k in api.FlowField.NAMES:
        assert np.array_equal(d["fields"][k], getattr(f, k)), k
    assert d["params"] == {**params_dict(p), "bc_types": d["params"]["bc_types"],
                           "bc_values": d["params"]["bc_values"]}
    st, g2, f2, p2, t2, name, prefix, base = api.checkpoint_read(path)
    assert st == A.CFD_SUCCESS
    assert (t2, name, prefix, base) == (1.25, "rk2", "myrun", "/base/dir")
    for k in api.FlowField.NAMES:
        assert np.array_equal(getattr(f2, k), getattr(f, k)), k
    gd, gd2 = grid_dict(g), grid_dict(g2)
    for k in gd:
        assert np.array_equal(np.asarray(gd[k]), np.asarray(gd2[k])), k
    assert_params_equal(p, p2)
    # the bytes a second write produces are identical (deterministic encoder)
    path2 = str(tmp_path / "b.cfdchk")
    assert api.checkpoint_write(path2, g2, f2, p2, t2, name, prefix, base) == A.CFD_SUCCESS
    assert open(path2, "rb").read() == data


def test_roundtrip_3d_stretched_and_oracle_written_file(tmp_path):
    """test_checkpoint.c:228-256 (z, dz, inv_dz2) both ways: our writer vs the
    oracle's parser, and a file the oracle encodes read back by our reader."""
    g = api.Grid(6, 5, 4, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0)
    stretch(g)
    f = api.FlowField(6, 5, 4)
    known_field(f, 9.0)
    p = nondefault_params()
    path = str(tmp_path / "s.cfdchk")
    assert api.checkpoint_write(path, g, f, p, 0.5, "rk4", None, None) == A.CFD_SUCCESS
    d = fmt.decode(open(path, "rb").read())
    gd = grid_dict(g)
    for k in gd:
        assert np.array_equal(np.asarray(d["grid"][k]), np.asarray(gd[k])), k
    assert d["crc_ok"] and d["prefix"] == b"" and d["base"] == b""
    blob = fmt.encode(gd, {k: getattr(f, k) for k in api.FlowField.NAMES}, params_dict(p), 0.5,
                      b"rk4")
    assert blob == open(path, "rb").read()
    opath = str(tmp_path / "o.cfdchk")
    open(opath, "wb").write(fmt.encode(gd, {k: getattr(f, k) * 2 for k in api.FlowField.NAMES},
                                       params_dict(p), 7.0, b"projection_hip", b"pre", b"dir"))
    st, g2, f2, p2, t2, name, prefix, base = api.checkpoint_read(opath, caps=(128, 0, 0))
    assert st == A.CFD_SUCCESS and t2 == 7.0 and name == "projection_hip"
    assert prefix is None and base is None
    for k in api.FlowField.NAMES:
        assert np.array_equal(getattr(f2, k), getattr(f, k) * 2), k


def _sample(tmp_path):
    g = api.Grid(10, 7, 3, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0)
    f = api.FlowField(10, 7, 3)
    known_field(f, 1.5)
    path = str(tmp_path / "c.cfdchk")
    assert api.checkpoint_write(path, g, f, nondefault_params(), 2.0, "projection_hip") == 0
    return path, open(path, "rb").read()


def test_reject_bad_version_and_endian(tmp_path):
    path, data = _sample(tmp_path)
    for off in (8, 12):  # format version, endian marker (checkpoint.c:250-251)
        bad = bytearray(data)
        bad[off] ^= 0x7F
        open(path, "wb").write(bytes(bad))
        assert api.checkpoint_read(path)[0] == A.CFD_ERROR_UNSUPPORTED


def test_reject_bad_magic(tmp_path):
    path, data = _sample(tmp_path)
    open(path, "wb").write(b"X" + data[1:])
    assert api.checkpoint_read(path)[0] == A.CFD_ERROR_INVALID


def test_reject_truncated_and_missing(tmp_path):
    path, data = _sample(tmp_path)
    for cut in (len(data) // 2, len(data) - 1, 20):
        open(path, "wb").write(data[:cut])
        assert api.checkpoint_read(path)[0] == A.CFD_ERROR_IO, cut
    assert api.checkpoint_read(str(tmp_path / "none.cfdchk"))[0] == A.CFD_ERROR_IO


def test_reject_crc_corruption_every_field(tmp_path):
    path, data = _sample(tmp_path)
    for name, off in fmt.field_offsets(data).items():
        bad = bytearray(data)
        bad[off + 13] ^= 0x01  # one bit of one value, structure intact
        open(path, "wb").write(bytes(bad))
        assert api.checkpoint_read(path)[0] == A.CFD_ERROR_IO, name
    bad = bytearray(data)
    bad[-1] ^= 0x80  # the stored CRC itself
    open(path, "wb").write(bytes(bad))
    assert api.checkpoint_read(path)[0] == A.CFD_ERROR_IO


def test_string_capacity_and_null_arguments(tmp_path):
    path, _ = _sample(tmp_path)
    assert api.checkpoint_read(path, caps=(4, 256, 512))[0] == A.CFD_ERROR_INVALID  # name > cap
    # "projection_hip" is 14 bytes: a 14-byte buffer has no room for the NUL
    assert api.checkpoint_read(path, caps=(14, 256, 512))[0] == A.CFD_ERROR_INVALID
    assert api.checkpoint_read(path, caps=(15, 256, 512))[0] == A.CFD_SUCCESS
    g = api.Grid(4, 4, 1)
    f = api.FlowField(5, 4, 1)
    p = api.params_default()
    out = str(tmp_path / "x.cfdchk")
    assert api.checkpoint_write(out, g, f, p, 0.0, "x") == A.CFD_ERROR_INVALID  # dims
    assert api.checkpoint_write(out, g, api.FlowField(4, 4, 1), p, 0.0, None) == \
        A.CFD_ERROR_INVALID


def test_crc_join_arithmetic_matches_zlib():
    """The GF(2) register join the device path relies on (chk_format.h
    chk_crc_join): crc(A || B) from crc(A) and the zero-register CRC of B."""
    rng = np.random.default_rng(5)
    a = rng.bytes(1000)
    b = rng.bytes(4096 + 24)
    P = 0xEDB88320

    def gf_mul(x, y):
        r = 0
        for _ in range(32):
            if x & 0x80000000:
                r ^= y
            x = (x << 1) & 0xFFFFFFFF
            y = (y >> 1) ^ P if y & 1 else y >> 1
        return r

    def xpow_bytes(n):
        r, sq = 0x80000000, 0x00800000
        while n:
            if n & 1:
                r = gf_mul(r, sq)
            sq = gf_mul(sq, sq)
            n >>= 1
        return r

    state_a = zlib.crc32(a) ^ 0xFFFFFFFF             # register after A
    raw0_b = zlib.crc32(b, 0xFFFFFFFF) ^ 0xFFFFFFFF  # register of B from zero
    joined = gf_mul(xpow_bytes(len(b)), state_a) ^ raw0_b
    assert joined ^ 0xFFFFFFFF == zlib.crc32(a + b)
