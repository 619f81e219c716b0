"""CPU model of the multi-rank Z-slab path over torch.distributed (gloo),
world sizes 2 and 3, one process per rank.

Each rank takes its slab from the product library's own partition
(hip_proj_slab_layout), exchanges halo planes with the posting order the RCCL
backend uses (sends to-lower then to-upper, receives from-upper then
from-lower; with 2 ranks and periodic z both neighbours are the same peer),
applies the boundary conditions with the edge-rank face rule of k_bc_shell,
and runs the Red-Black SOR / Jacobi iteration with the global colour parity
(i + j + k + k_offset) and an all-reduced L-infinity residual -- the
schedule relax_solve() runs on the GPU. Gathered, the result must be bitwise
the single-domain oracle's. This covers the decomposition logic on a machine
without a GPU; tests/test_gpu_slabs.py and test_gpu_rccl.py run the device
path itself.
"""
import math
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from cfd_amd import _abi as A
from cfd_amd import api
from oracle import oracle
from tests import cases


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _halo(x, rank, size, periodic=False):
    lo = rank - 1 if rank > 0 else (size - 1 if periodic else -1)
    hi = rank + 1 if rank < size - 1 else (0 if periodic else -1)
    reqs, recv = [], {}
    if lo >= 0:
        reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(x[1])), lo))
    if hi >= 0:
        reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(x[-2])), hi))
    if hi >= 0:
        recv["hi"] = torch.empty(x.shape[1:], dtype=torch.float64)
        reqs.append(dist.irecv(recv["hi"], hi))
    if lo >= 0:
        recv["lo"] = torch.empty(x.shape[1:], dtype=torch.float64)
        reqs.append(dist.irecv(recv["lo"], lo))
    for r in reqs:
        r.wait()
    if "hi" in recv:
        x[-1] = recv["hi"].numpy()
    if "lo" in recv:
        x[0] = recv["lo"].numpy()


def _neumann(x, lo_face, hi_face):
    # x faces, y faces, then z faces on the ranks that hold them
    x[:, :, 0] = x[:, :, 1]
    x[:, :, -1] = x[:, :, -2]
    x[:, 0, :] = x[:, 1, :]
    x[:, -1, :] = x[:, -2, :]
    if lo_face:
        x[0] = x[1]
    if hi_face:
        x[-1] = x[-2]


def _linf(x, rhs, c):
    xc = x[1:-1, 1:-1, 1:-1]
    lap = ((x[1:-1, 1:-1, 2:] - 2.0 * xc + x[1:-1, 1:-1, :-2]) / c["dx2"]
           + (x[1:-1, 2:, 1:-1] - 2.0 * xc + x[1:-1, :-2, 1:-1]) / c["dy2"]
           + (x[2:, 1:-1, 1:-1] + x[:-2, 1:-1, 1:-1] - 2.0 * xc) * c["inv_dz2"])
    m = float(np.max(np.abs(lap - rhs[1:-1, 1:-1, 1:-1]))) if xc.size else 0.0
    t = torch.tensor([m], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0])


def _update(x, rhs, c):
    xc = x[1:-1, 1:-1, 1:-1]
    return -(rhs[1:-1, 1:-1, 1:-1] - (x[1:-1, 1:-1, 2:] + x[1:-1, 1:-1, :-2]) / c["dx2"]
             - (x[1:-1, 2:, 1:-1] + x[1:-1, :-2, 1:-1]) / c["dy2"]
             - (x[2:, 1:-1, 1:-1] + x[:-2, 1:-1, 1:-1]) * c["inv_dz2"]) * c["inv_factor"], xc


def _worker(rank, size, port, method, n, outdir):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=size)
    try:
        g, rhs_g = cases.cos_rhs(n)
        ko, nl = api.slab_layout(n, rank, size)
        rhs = rhs_g[ko:ko + nl].copy()
        x = np.zeros_like(rhs)
        dx = dy = dz = 1.0 / (n - 1)
        c = {"dx2": dx * dx, "dy2": dy * dy, "inv_dz2": 1.0 / (dz * dz)}
        c["inv_factor"] = 1.0 / (2.0 * (1.0 / c["dx2"] + 1.0 / c["dy2"] + c["inv_dz2"]))
        inv = 1.0 / (dx * dx)
        num = 3 * math.cos(math.pi / (n - 1)) * inv
        rj = num / (3 * inv)
        omega = 2.0 / (1.0 + math.sqrt(1.0 - rj * rj))
        K, J, I = np.meshgrid(np.arange(1, nl - 1) + ko, np.arange(1, n - 1), np.arange(1, n - 1),
                              indexing="ij")
        odd = ((I + J + K) & 1) == 1
        lo_face, hi_face = rank == 0, rank == size - 1
        maxit = 5000 if method == "rb" else 3000
        _halo(x, rank, size)
        res0 = _linf(x, rhs, c)
        tol = max(1e-6 * res0, 1e-10)
        it, conv = 0, False
        for it in range(maxit):
            if method == "rb":
                for colour in (odd, ~odd):  # the reference's "red" pass updates odd cells
                    pn, xc = _update(x, rhs, c)
                    xc[colour] = (xc + omega * (pn - xc))[colour]
                    _halo(x, rank, size)
            else:
                pn, _ = _update(x, rhs, c)
                x = x.copy()
                x[1:-1, 1:-1, 1:-1] = pn
                _halo(x, rank, size)
            _neumann(x, lo_face, hi_face)
            res = _linf(x, rhs, c)
            if res < tol or res < 1e-10:
                conv = True
                break
        lo = 0 if lo_face else 1
        hi = nl if hi_face else nl - 1
        np.save(os.path.join(outdir, f"x{rank}.npy"), x[lo:hi])
        np.save(os.path.join(outdir, f"meta{rank}.npy"),
                np.array([ko + lo, ko + hi, it + 1, int(conv)]))
        # periodic z exchange (the same-peer case when size == 2)
        y = np.full((nl, 3, 4), float(rank))
        y[1] += 10.0
        y[-2] += 20.0
        _halo(y, rank, size, periodic=True)
        lo_r, hi_r = (rank - 1) % size, (rank + 1) % size
        assert np.all(y[0] == lo_r + 20.0) and np.all(y[-1] == hi_r + 10.0)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("size,method", [(2, "rb"), (3, "rb"), (2, "jacobi")])
def test_gloo_slab_relaxation_bitwise(tmp_path, size, method):
    n = 17
    mp.spawn(_worker, args=(size, _free_port(), method, n, str(tmp_path)), nprocs=size,
             join=True)
    g, rhs = cases.cos_rhs(n)
    xo = np.zeros_like(rhs)
    prm = oracle.poisson_params(max_iterations=5000 if method == "rb" else 3000)
    if method == "rb":
        so, sto = oracle.redblack_solve(xo, rhs, g.dx, g.dy, g.dz, prm)
    else:
        so, sto = oracle.jacobi_solve(xo, rhs, g.dx, g.dy, g.dz, prm)
    x = np.full_like(rhs, np.nan)
    for r in range(size):
        a, b, iters, conv = np.load(tmp_path / f"meta{r}.npy")
        x[a:b] = np.load(tmp_path / f"x{r}.npy")
        assert iters == sto.iterations
        assert bool(conv) == (so == A.CFD_SUCCESS)
    np.testing.assert_array_equal(x, xo)
