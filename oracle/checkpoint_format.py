"""TEST INFRASTRUCTURE ONLY (never shipped, never on the product path).

An independent restatement of the reference's `.cfdchk` restart format in
Python (struct + zlib), used by tests/ to check the files the product writes
and to author files the product must read or reject. It follows
lib/src/io/checkpoint.c:
  header   write_header        :249-258  magic, version 1, endian marker,
                                          library version 0.3.0 (cfd_version.h:11-13),
                                          flags (bit 0 = CRC), reserved
  grid     write_grid          :260-279
  field    write_field         :281-293  u, v, w, p, rho, T
  params   write_params        :295-327
  tail     cfd_checkpoint_write :357-364 time, 3 length-prefixed strings,
                                          CRC-32 of everything before it
The CRC is IEEE CRC-32 (reflected 0xEDB88320, init/xorout 0xFFFFFFFF,
checkpoint.c:40-50), which is exactly zlib.crc32.
"""
from __future__ import annotations

import struct
import zlib

import numpy as np

MAGIC = b"CFDCHK\0\0"
VERSION = 1
ENDIAN = 0x01020304
LIB_VERSION = (0, 3, 0)
FLAG_CRC = 1
FIELDS = ("u", "v", "w", "p", "rho", "T")
PARAM_F64_A = ("dt", "cfl", "gamma", "mu", "k")
PARAM_F64_B = ("tolerance", "source_amplitude_u", "source_amplitude_v", "source_decay_rate",
               "pressure_coupling", "alpha", "beta", "T_ref", "g0", "g1", "g2")
BC_TYPES = ("left", "right", "bottom", "top", "front", "back")
BC_VALUES = ("left", "right", "top", "bottom", "front", "back")


def _s(b: bytes | None) -> bytes:
    return b or b""


def encode(grid: dict, fields: dict, params: dict, time: float, solver: bytes,
           prefix: bytes | None = None, base: bytes | None = None, *, version=VERSION,
           endian=ENDIAN, flags=FLAG_CRC, crc_override=None) -> bytes:
    """grid: nx, ny, nz, bounds (6), x, y, dx, dy, z, dz, inv_dz2; fields: name ->
    array (nz, ny, nx); params: the names above + bc_types (6 ints) + bc_values."""
    nx, ny, nz = grid["nx"], grid["ny"], grid["nz"]
    out = [MAGIC, struct.pack("<IIHHHHQ", version, endian, *LIB_VERSION, flags, 0)]
    out.append(struct.pack("<QQQ6d", nx, ny, nz, *grid["bounds"]))
    for k in ("x", "y", "dx", "dy"):
        out.append(np.asarray(grid[k], dtype="<f8").tobytes())
    if nz > 1:
        out.append(np.asarray(grid["z"], dtype="<f8").tobytes())
        out.append(np.asarray(grid["dz"], dtype="<f8").tobytes())
        out.append(struct.pack("<d", grid["inv_dz2"]))
    out.append(struct.pack("<QQQ", nx, ny, nz))
    for k in FIELDS:
        a = np.ascontiguousarray(fields[k], dtype="<f8")
        assert a.size == nx * ny * nz
        out.append(a.tobytes())
    out.append(struct.pack("<5d", *(params[k] for k in PARAM_F64_A)))
    out.append(struct.pack("<i", params["max_iter"]))
    out.append(struct.pack("<11d", *(params[k] for k in PARAM_F64_B)))
    out.append(struct.pack("<6i", *params["bc_types"]))
    out.append(struct.pack("<6d", *params["bc_values"]))
    out.append(struct.pack("<d", time))
    for s in (solver, prefix, base):
        out.append(struct.pack("<I", len(_s(s))) + _s(s))
    body = b"".join(out)
    crc = zlib.crc32(body) if crc_override is None else crc_override
    return body + (struct.pack("<I", crc) if flags & FLAG_CRC else b"")


class Reader:
    def __init__(self, data: bytes):
        self.d = data
        self.o = 0

    def take(self, fmt: str):
        v = struct.unpack_from(fmt, self.d, self.o)
        self.o += struct.calcsize(fmt)
        return v

    def arr(self, n: int) -> np.ndarray:
        a = np.frombuffer(self.d, dtype="<f8", count=n, offset=self.o).copy()
        self.o += 8 * n
        return a

    def string(self) -> bytes:
        (n,) = self.take("<I")
        s = self.d[self.o:self.o + n]
        self.o += n
        return s


def decode(data: bytes) -> dict:
    """Parse a whole file; raises ValueError on a bad magic/CRC/size."""
    r = Reader(data)
    if r.take("8s")[0] != MAGIC:
        raise ValueError("magic")
    version, endian, ma, mi, pa, flags, _ = r.take("<IIHHHHQ")
    nx, ny, nz, *bounds = r.take("<QQQ6d")
    g = {"nx": nx, "ny": ny, "nz": nz, "bounds": bounds, "x": r.arr(nx), "y": r.arr(ny),
         "dx": r.arr(nx - 1), "dy": r.arr(ny - 1)}
    if nz > 1:
        g["z"] = r.arr(nz)
        g["dz"] = r.arr(nz - 1)
        (g["inv_dz2"],) = r.take("<d")
    if r.take("<QQQ") != (nx, ny, nz):
        raise ValueError("field dims")
    n = nx * ny * nz
    fields = {k: r.arr(n).reshape(nz, ny, nx) for k in FIELDS}
    p = dict(zip(PARAM_F64_A, r.take("<5d")))
    (p["max_iter"],) = r.take("<i")
    p.update(zip(PARAM_F64_B, r.take("<11d")))
    p["bc_types"] = r.take("<6i")
    p["bc_values"] = r.take("<6d")
    (time,) = r.take("<d")
    strings = [r.string() for _ in range(3)]
    body_end = r.o
    crc_ok = None
    if flags & FLAG_CRC:
        (stored,) = r.take("<I")
        crc_ok = stored == zlib.crc32(data[:body_end])
    if r.o != len(data):
        raise ValueError("trailing bytes")
    return {"version": version, "endian": endian, "lib_version": (ma, mi, pa), "flags": flags,
            "grid": g, "fields": fields, "params": p, "time": time, "solver": strings[0],
            "prefix": strings[1], "base": strings[2], "crc_ok": crc_ok}


def field_offsets(data: bytes) -> dict:
    """Byte offset of each field array in the file (for corruption tests)."""
    r = Reader(data)
    r.take("8s")
    r.take("<IIHHHHQ")
    nx, ny, nz, *_ = r.take("<QQQ6d")
    r.o += 8 * (2 * nx + 2 * ny - 2)
    if nz > 1:
        r.o += 8 * (2 * nz - 1) + 8
    r.o += 24
    n = nx * ny * nz
    return {k: r.o + 8 * n * q for q, k in enumerate(FIELDS)}
