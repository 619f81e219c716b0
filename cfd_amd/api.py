"""Python mirror of the reference's plugin interface for the projection path.

Names, argument meaning and error behaviour follow the reference C API
(lib/include/cfd/solvers/navier_stokes_solver.h, lib/include/cfd/core/grid.h,
lib/include/cfd/boundary/boundary_conditions.h): a Grid, a FlowField of
caller-owned host arrays, solver parameters, and solvers created by name from
a registry and driven with init/step/solve. Everything here is a thin wrapper
over libcfd_host.so / libcfd_hip.so; the numerics run in HIP.
"""
from __future__ import annotations

import ctypes as C
from typing import Optional

import numpy as np

from . import _abi as A
from . import _native


class CfdError(RuntimeError):
    def __init__(self, status: int, where: str):
        msg = _native.last_error()
        super().__init__(f"{where}: status {status} ({status_name(status)}) {msg}")
        self.status = status


def status_name(status: int) -> str:
    s = _native.host().cfd_get_error_string(status)
    return s.decode() if s else str(status)


def _check(status: int, where: str) -> None:
    if status != A.CFD_SUCCESS:
        raise CfdError(status, where)


def _view(ptr, n: int, shape) -> np.ndarray:
    buf = (C.c_double * n).from_address(C.addressof(ptr.contents))
    return np.frombuffer(buf, dtype=np.float64).reshape(shape)


class Grid:
    """grid_create + grid_initialize_uniform (grid.c:9-127)."""

    def __init__(self, nx, ny, nz=1, xmin=0.0, xmax=1.0, ymin=0.0, ymax=1.0, zmin=0.0,
                 zmax=0.0):
        h = _native.host()
        if nz > 1 and zmax <= zmin:
            zmax = zmin + 1.0
        self._ptr = h.grid_create(nx, ny, nz, xmin, xmax, ymin, ymax, zmin, zmax)
        if not self._ptr:
            raise CfdError(h.cfd_get_last_status(), "grid_create")
        h.grid_initialize_uniform(self._ptr)

    @classmethod
    def adopt(cls, ptr) -> "Grid":
        """Take ownership of a grid* the C library allocated (grid_destroy frees it)."""
        g = cls.__new__(cls)
        g._ptr = ptr
        return g

    @property
    def ptr(self):
        return self._ptr

    @property
    def c(self) -> A.Grid:
        return self._ptr.contents

    nx = property(lambda s: s.c.nx)
    ny = property(lambda s: s.c.ny)
    nz = property(lambda s: s.c.nz)

    @property
    def x(self):
        return np.ctypeslib.as_array(self.c.x, shape=(self.nx,))

    @property
    def y(self):
        return np.ctypeslib.as_array(self.c.y, shape=(self.ny,))

    @property
    def z(self):
        return np.ctypeslib.as_array(self.c.z, shape=(self.nz,)) if self.nz > 1 else np.zeros(1)

    @property
    def dx(self):
        return self.c.dx[0]

    @property
    def dy(self):
        return self.c.dy[0]

    @property
    def dz(self):
        return self.c.dz[0] if self.nz > 1 else 0.0

    @property
    def stride_z(self):
        return self.c.stride_z

    def __del__(self):
        try:
            if getattr(self, "_ptr", None):
                _native.host().grid_destroy(self._ptr)
                self._ptr = None
        except Exception:
            pass


class FlowField:
    """flow_field_create: SoA host arrays, exposed as (nz, ny, nx) numpy views."""

    NAMES = ("u", "v", "w", "p", "rho", "T")

    def __init__(self, nx, ny, nz=1):
        h = _native.host()
        self._ptr = h.flow_field_create(nx, ny, nz)
        if not self._ptr:
            raise CfdError(h.cfd_get_last_status(), "flow_field_create")
        self._bind_views()

    def _bind_views(self):
        c = self._ptr.contents
        n = c.nx * c.ny * c.nz
        for name in self.NAMES:
            setattr(self, name, _view(getattr(c, name), n, (c.nz, c.ny, c.nx)))

    @classmethod
    def adopt(cls, ptr) -> "FlowField":
        """Take ownership of a flow_field* the C library allocated."""
        f = cls.__new__(cls)
        f._ptr = ptr
        f._bind_views()
        return f

    @property
    def ptr(self):
        return self._ptr

    @property
    def shape(self):
        return self.u.shape

    def copy_from(self, other: "FlowField") -> None:
        for name in self.NAMES:
            getattr(self, name)[...] = getattr(other, name)

    def arrays(self):
        return {n: getattr(self, n).copy() for n in self.NAMES}

    def __del__(self):
        try:
            if getattr(self, "_ptr", None):
                _native.host().flow_field_destroy(self._ptr)
                self._ptr = None
        except Exception:
            pass


def params_default() -> A.SolverParams:
    """ns_solver_params_default (solver_explicit_euler.c:58-78)."""
    return _native.host().ns_solver_params_default()


def validation_params(dt: float, nu: float) -> A.SolverParams:
    """The parameter block the reference validation drivers build
    (lid_driven_cavity_common.h:258-270, taylor_green_3d_reference.h:274-286)."""
    p = A.SolverParams()
    p.dt = dt
    p.cfl = 0.5
    p.gamma = 1.4
    p.mu = nu
    p.k = 0.0
    p.max_iter = 1
    p.tolerance = 1e-6
    p.source_amplitude_u = 0.0
    p.source_amplitude_v = 0.0
    p.source_decay_rate = 0.0
    p.pressure_coupling = 0.1
    return p


def bc_apply_scalar_3d(arr: np.ndarray, bc_type: int) -> None:
    nz, ny, nx = arr.shape
    ptr = arr.ctypes.data_as(A.c_double_p)
    _check(_native.host().bc_apply_scalar_3d(ptr, nx, ny, nz, nx * ny if nz > 1 else 0, bc_type),
           "bc_apply_scalar_3d")


def dirichlet(left=0.0, right=0.0, top=0.0, bottom=0.0, front=0.0, back=0.0):
    return A.DirichletValues(left, right, top, bottom, front, back)


def bc_apply_dirichlet_velocity_3d(field: FlowField, uv, vv, wv) -> None:
    nz, ny, nx = field.shape
    c = field.ptr.contents
    _check(_native.host().bc_apply_dirichlet_velocity_3d(
        c.u, c.v, c.w, nx, ny, nz, nx * ny if nz > 1 else 0, C.byref(uv), C.byref(vv),
        C.byref(wv)), "bc_apply_dirichlet_velocity_3d")


def cavity_bc(field: FlowField, lid: float = 1.0) -> None:
    """Lid-driven cavity BCs as the reference drivers apply them before every
    step: Dirichlet velocity (u = lid on the y = ymax face) + Neumann p
    (lid_driven_cavity_common.h:140-160 / SURVEY.md §8d config 3)."""
    bc_apply_dirichlet_velocity_3d(field, dirichlet(top=lid), dirichlet(), dirichlet())
    bc_apply_scalar_3d(field.p, A.BC_TYPE_NEUMANN)


def checkpoint_write(path: str, grid: "Grid", field: "FlowField", params: A.SolverParams,
                     time: float, solver_name: str, run_prefix: Optional[str] = None,
                     base_dir: Optional[str] = None) -> int:
    """cfd_checkpoint_write (checkpoint.h:49-75) through libcfd_host.so."""
    enc = (lambda x: x.encode() if x is not None else None)
    return _native.host().cfd_checkpoint_write(
        path.encode(), grid.ptr if grid is not None else None,
        field.ptr if field is not None else None,
        C.byref(params) if params is not None else None, time, enc(solver_name),
        enc(run_prefix), enc(base_dir))


def checkpoint_read(path: str, caps=(128, 256, 512)):
    """cfd_checkpoint_read (checkpoint.h:77-115): returns (status, Grid, FlowField,
    params, time, solver_name, run_prefix, base_dir); cap 0 passes NULL."""
    h = _native.host()
    gp = C.POINTER(A.Grid)()
    fp = C.POINTER(A.FlowField)()
    prm = A.SolverParams()
    t = C.c_double(0.0)
    bufs = [C.create_string_buffer(c) if c else None for c in caps]
    st = h.cfd_checkpoint_read(path.encode(), C.byref(gp), C.byref(fp), C.byref(prm),
                               C.byref(t), bufs[0], caps[0], bufs[1], caps[1], bufs[2], caps[2])
    if st != A.CFD_SUCCESS:
        return st, None, None, prm, 0.0, None, None, None
    return (st, Grid.adopt(gp), FlowField.adopt(fp), prm, t.value,
            *[b.value.decode() if b is not None else None for b in bufs])


class Registry:
    """cfd_registry_create + cfd_registry_register_defaults."""

    def __init__(self):
        _native.hip()  # make the HIP plugin visible to register_defaults
        h = _native.host()
        self._ptr = h.cfd_registry_create()
        h.cfd_registry_register_defaults(self._ptr)

    def names(self):
        h = _native.host()
        n = h.cfd_registry_list(self._ptr, None, 0)
        arr = (C.c_char_p * max(n, 1))()
        h.cfd_registry_list(self._ptr, arr, n)
        return [arr[i].decode() for i in range(n)]

    def has(self, name: str) -> bool:
        return bool(_native.host().cfd_registry_has(self._ptr, name.encode()))

    def create(self, name: str) -> "Solver":
        h = _native.host()
        h.cfd_clear_error()
        ptr = h.cfd_solver_create(self._ptr, name.encode())
        if not ptr:
            raise CfdError(h.cfd_get_last_status(), f"cfd_solver_create({name})")
        return Solver(ptr, self)

    def __del__(self):
        try:
            if getattr(self, "_ptr", None):
                _native.host().cfd_registry_destroy(self._ptr)
                self._ptr = None
        except Exception:
            pass


class Solver:
    """An ns_solver_t driven through solver_init / solver_step / solver_solve."""

    def __init__(self, ptr, registry: Registry):
        self._ptr = ptr
        self._registry = registry

    @property
    def name(self) -> str:
        return self._ptr.contents.name.decode()

    def init(self, grid: Grid, params: A.SolverParams) -> int:
        return _native.host().solver_init(self._ptr, grid.ptr, C.byref(params))

    def step(self, field: FlowField, grid: Grid, params: A.SolverParams,
             stats: Optional[A.SolverStats] = None) -> int:
        st = stats if stats is not None else A.SolverStats()
        return _native.host().solver_step(self._ptr, field.ptr, grid.ptr, C.byref(params),
                                          C.byref(st))

    def solve(self, field: FlowField, grid: Grid, params: A.SolverParams,
              stats: Optional[A.SolverStats] = None) -> int:
        st = stats if stats is not None else A.SolverStats()
        return _native.host().solver_solve(self._ptr, field.ptr, grid.ptr, C.byref(params),
                                           C.byref(st))

    def close(self):
        if getattr(self, "_ptr", None):
            _native.host().solver_destroy(self._ptr)
            self._ptr = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def hip_available() -> bool:
    return bool(_native.hip().hip_projection_available())


def hip_config(**kw) -> A.HipProjConfig:
    cfg = _native.hip().hip_proj_config_default()
    for k, v in kw.items():
        if not hasattr(cfg, k):
            raise KeyError(k)
        setattr(cfg, k, v)
    return cfg


def slab_layout(nz: int, rank: int, size: int):
    """(k_offset, nz_local) of `rank`'s Z-slab (hip_proj_slab_layout; host only)."""
    ko, nl = C.c_size_t(), C.c_size_t()
    _check(_native.hip().hip_proj_slab_layout(nz, rank, size, C.byref(ko), C.byref(nl)),
           "hip_proj_slab_layout")
    return ko.value, nl.value


def comm_unique_id() -> bytes:
    """RCCL unique id bytes (rank 0 creates, the caller broadcasts)."""
    buf = C.create_string_buffer(128)
    _check(_native.hip().hip_proj_comm_unique_id(buf), "hip_proj_comm_unique_id")
    return buf.raw


class SlabComm:
    """One rank's Z-slab communicator (RCCL or in-process group endpoint)."""

    def __init__(self, handle, keepalive=None):
        if not handle:
            raise CfdError(_native.host().cfd_get_last_status(), "slab comm create")
        self._h = handle
        self._keep = keepalive

    @classmethod
    def rccl(cls, uid: bytes, rank: int, size: int, device: int = 0) -> "SlabComm":
        assert len(uid) == 128
        return cls(_native.hip().hip_proj_comm_create_rccl(uid, rank, size, device))

    @property
    def handle(self):
        return self._h

    @property
    def rank(self) -> int:
        return _native.hip().hip_proj_comm_rank(self._h)

    @property
    def size(self) -> int:
        return _native.hip().hip_proj_comm_size(self._h)

    @property
    def device_allreduce(self) -> bool:
        return bool(_native.hip().hip_proj_comm_device_allreduce(self._h))

    def allreduce_bench(self, iters: int, mode: int) -> float:
        """Collective: microseconds per two-value CG dot all-reduce
        (hip_proj_comm_mailbox_bench; mode 0 mailbox round trip inside one
        kernel, 1 one launch + mailbox per all-reduce, 2 ncclAllReduce +
        a check kernel)."""
        us = C.c_double(0.0)
        st = _native.hip().hip_proj_comm_mailbox_bench(self._h, iters, mode, C.byref(us))
        if st != A.CFD_SUCCESS:
            raise CfdError(st, "allreduce bench: " + _native.last_error())
        return us.value

    def close(self):
        if getattr(self, "_h", None):
            _native.hip().hip_proj_comm_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class LocalGroup:
    """In-process slab group: `size` ranks driven by host threads of this
    process (hip_proj_group_*); see run_ranks()."""

    def __init__(self, size: int):
        self._g = _native.hip().hip_proj_group_create(size)
        if not self._g:
            raise CfdError(_native.host().cfd_get_last_status(), "hip_proj_group_create")
        self.size = size
        self.comms = []

    def comm(self, rank: int, device: int = 0) -> SlabComm:
        c = SlabComm(_native.hip().hip_proj_comm_create_local(self._g, rank, device), self)
        self.comms.append(c)
        return c

    def close(self):
        for c in self.comms:
            c.close()
        self.comms = []
        if getattr(self, "_g", None):
            _native.hip().hip_proj_group_destroy(self._g)
            self._g = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def run_ranks(fn, n: int):
    """Run fn(rank) on n host threads (ctypes drops the GIL inside the C calls)
    and return the results in rank order; re-raises the first exception."""
    import threading

    out = [None] * n
    err = [None] * n

    def body(r):
        try:
            out[r] = fn(r)
        except BaseException as e:  # noqa: BLE001
            err[r] = e

    ts = [threading.Thread(target=body, args=(r,)) for r in range(n)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    for e in err:
        if e is not None:
            raise e
    return out


class HipProjection:
    """Device-resident projection context (hip_proj_* C-ABI). With `comm`, the
    context holds rank comm.rank's Z-slab of the global nx*ny*nz grid and its
    fields have shape (nz_local, ny, nx)."""

    def __init__(self, nx, ny, nz=1, comm: Optional[SlabComm] = None, **config):
        lib = _native.hip()
        self._cfg = hip_config(**config)
        self._comm = comm
        if comm is None:
            self._ctx = lib.hip_proj_create(nx, ny, nz, C.byref(self._cfg))
        else:
            self._ctx = lib.hip_proj_create_slab(nx, ny, nz, comm.handle, C.byref(self._cfg))
        if not self._ctx:
            raise CfdError(_native.host().cfd_get_last_status(), "hip_proj_create")
        ko, nl = C.c_size_t(), C.c_size_t()
        rk, sz = C.c_int(), C.c_int()
        lib.hip_proj_slab_info(self._ctx, C.byref(ko), C.byref(nl), C.byref(rk), C.byref(sz))
        self.k_offset, self.nz_local, self.rank, self.size = ko.value, nl.value, rk.value, sz.value
        self.nz_global = nz
        self.shape = (nl.value, ny, nx)

    def owned(self):
        """(local, global) plane slices this rank is authoritative for: its
        interior planes plus the global z faces it holds."""
        lo = 0 if self.rank == 0 else 1
        hi = self.nz_local if self.rank == self.size - 1 else self.nz_local - 1
        return slice(lo, hi), slice(self.k_offset + lo, self.k_offset + hi)

    @property
    def ctx(self):
        return self._ctx

    def _lib(self):
        return _native.hip()

    def upload(self, field: FlowField):
        _check(self._lib().hip_proj_upload(self._ctx, field.ptr), "hip_proj_upload")

    def download(self, field: FlowField):
        _check(self._lib().hip_proj_download(self._ctx, field.ptr), "hip_proj_download")

    def sync_host(self, field: FlowField):
        """hip_proj_sync_host: the whole of u, v, w, p (T) to the host field
        (the resident mode's full download)."""
        _check(self._lib().hip_proj_sync_host(self._ctx, field.ptr), "hip_proj_sync_host")

    def step(self, field: FlowField, grid: Grid, params: A.SolverParams,
             stats: Optional[A.SolverStats] = None) -> int:
        st = stats if stats is not None else A.SolverStats()
        return self._lib().hip_proj_step(self._ctx, field.ptr, grid.ptr, C.byref(params),
                                         C.byref(st))

    def mark_host_dirty(self):
        """hip_proj_mark_host_dirty: the next host-buffer step uploads in full."""
        _check(self._lib().hip_proj_mark_host_dirty(self._ctx), "hip_proj_mark_host_dirty")

    def step_device(self, grid: Grid, params: A.SolverParams,
                    stats: Optional[A.SolverStats] = None) -> int:
        st = stats if stats is not None else A.SolverStats()
        return self._lib().hip_proj_step_device(self._ctx, grid.ptr, C.byref(params),
                                                C.byref(st))

    def set_field(self, fid: int, arr: np.ndarray):
        a = np.ascontiguousarray(arr, dtype=np.float64)
        assert a.shape == self.shape, (a.shape, self.shape)
        _check(self._lib().hip_proj_set_field(self._ctx, fid, a.ctypes.data_as(A.c_double_p)),
               "hip_proj_set_field")

    def field_crc32(self, fid: int) -> int:
        """hip_proj_field_crc32: zlib CRC-32 of the packed field, computed on the GPU."""
        v = C.c_uint32(0)
        _check(self._lib().hip_proj_field_crc32(self._ctx, fid, C.byref(v)), "hip_proj_field_crc32")
        return v.value

    def checkpoint_write(self, path: str, grid: "Grid", params: A.SolverParams, time: float,
                         solver_name: str, run_prefix: Optional[str] = None,
                         base_dir: Optional[str] = None) -> int:
        enc = (lambda x: x.encode() if x is not None else None)
        return self._lib().hip_proj_checkpoint_write(
            self._ctx, path.encode(), grid.ptr, C.byref(params), time, enc(solver_name),
            enc(run_prefix), enc(base_dir))

    def checkpoint_read(self, path: str, caps=(128, 256, 512)):
        """(status, Grid, params, time, solver_name, run_prefix, base_dir)."""
        gp = C.POINTER(A.Grid)()
        prm = A.SolverParams()
        t = C.c_double(0.0)
        bufs = [C.create_string_buffer(c) if c else None for c in caps]
        st = self._lib().hip_proj_checkpoint_read(self._ctx, path.encode(), C.byref(gp),
                                                  C.byref(prm), C.byref(t), bufs[0], caps[0],
                                                  bufs[1], caps[1], bufs[2], caps[2])
        if st != A.CFD_SUCCESS:
            return st, None, prm, 0.0, None, None, None
        return (st, Grid.adopt(gp), prm, t.value,
                *[b.value.decode() if b is not None else None for b in bufs])

    def get_field(self, fid: int) -> np.ndarray:
        out = np.empty(self.shape, dtype=np.float64)
        _check(self._lib().hip_proj_get_field(self._ctx, fid, out.ctypes.data_as(A.c_double_p)),
               "hip_proj_get_field")
        return out

    def fill(self, fid: int, value: float):
        _check(self._lib().hip_proj_fill_field(self._ctx, fid, value), "hip_proj_fill_field")

    def set_density(self, rho: float):
        _check(self._lib().hip_proj_set_density(self._ctx, rho), "hip_proj_set_density")

    def apply_scalar_bc(self, fid: int, bc_type: int):
        _check(self._lib().hip_proj_apply_scalar_bc(self._ctx, fid, bc_type),
               "hip_proj_apply_scalar_bc")

    def apply_dirichlet(self, fid: int, values: A.DirichletValues):
        _check(self._lib().hip_proj_apply_dirichlet(self._ctx, fid, C.byref(values)),
               "hip_proj_apply_dirichlet")

    def poisson_stats(self) -> A.PoissonStats:
        s = A.PoissonStats()
        _check(self._lib().hip_proj_get_poisson_stats(self._ctx, C.byref(s)),
               "hip_proj_get_poisson_stats")
        return s

    def enable_timing(self, on: bool = True):
        self._lib().hip_proj_enable_timing(self._ctx, 1 if on else 0)

    def reset_timing(self):
        self._lib().hip_proj_reset_timing(self._ctx)

    def placement(self):
        """(per-draw probe ms per CG iteration, index kept) of the context's
        placement draws (hip_proj_get_placement); ([], -1) without draws."""
        buf = (C.c_double * 64)()
        pick = C.c_int(-1)
        n = self._lib().hip_proj_get_placement(self._ctx, buf, 64, C.byref(pick))
        return [round(buf[i], 4) for i in range(min(n, 64))], pick.value

    def clock_sample(self):
        """(MHz, workgroups): the effective shader clock of the sampled k_ccf
        workgroups since reset_timing (hip_proj_get_clock_sample)."""
        mhz, n = C.c_double(0.0), C.c_longlong(0)
        self._lib().hip_proj_get_clock_sample(self._ctx, C.byref(mhz), C.byref(n))
        return mhz.value, n.value

    def timing(self):
        ms = (C.c_double * A.HIP_KT_COUNT)()
        n = (C.c_longlong * A.HIP_KT_COUNT)()
        self._lib().hip_proj_get_timing_n(self._ctx, ms, n, A.HIP_KT_COUNT)
        return {name: (ms[i], n[i]) for i, name in enumerate(A.KERNEL_TIMERS)}

    def synchronize(self):
        _check(self._lib().hip_proj_synchronize(self._ctx), "hip_proj_synchronize")

    def device_bytes(self) -> int:
        return self._lib().hip_proj_device_bytes(self._ctx)

    def poisson_solve(self, method: int, x: np.ndarray, rhs: np.ndarray, dx, dy, dz,
                      params: Optional[A.PoissonParams] = None,
                      bc_mode: int = A.HIP_POISSON_BC_NEUMANN,
                      bc_values: Optional[np.ndarray] = None):
        """hip_proj_poisson_solve (bc_mode NEUMANN) or hip_proj_poisson_solve_ex
        (NONE / FIXED with bc_values): solves in place on x; returns (status, stats)."""
        assert x.dtype == np.float64 and x.flags["C_CONTIGUOUS"] and x.shape == self.shape
        r = np.ascontiguousarray(rhs, dtype=np.float64)
        st = A.PoissonStats()
        prm = C.byref(params) if params is not None else None
        if bc_mode == A.HIP_POISSON_BC_NEUMANN and bc_values is None:
            s = self._lib().hip_proj_poisson_solve(
                self._ctx, method, x.ctypes.data_as(A.c_double_p),
                r.ctypes.data_as(A.c_double_p), dx, dy, dz, prm, C.byref(st))
            return s, st
        bv = None if bc_values is None else np.ascontiguousarray(bc_values, dtype=np.float64)
        s = self._lib().hip_proj_poisson_solve_ex(
            self._ctx, method, x.ctypes.data_as(A.c_double_p), r.ctypes.data_as(A.c_double_p),
            dx, dy, dz, prm, C.byref(st), bc_mode,
            bv.ctypes.data_as(A.c_double_p) if bv is not None else None)
        return s, st

    def cg_fixed_iters(self, rhs: np.ndarray, dx, dy, dz, iters: int) -> float:
        a = np.ascontiguousarray(rhs, dtype=np.float64)
        return self._lib().hip_proj_cg_fixed_iters(self._ctx, a.ctypes.data_as(A.c_double_p),
                                                   dx, dy, dz, iters)

    def cg_fixed_iters_step_rhs(self, dx, dy, dz, iters: int, rho_over_dt: float) -> float:
        """hip_proj_cg_fixed_iters_ex with the last step's RHS (rho/dt) div u*."""
        return self._lib().hip_proj_cg_fixed_iters_ex(self._ctx, None, dx, dy, dz, iters,
                                                      rho_over_dt)

    def close(self):
        if getattr(self, "_ctx", None):
            _native.hip().hip_proj_destroy(self._ctx)
            self._ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
