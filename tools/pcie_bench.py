#!/usr/bin/env python3
"""PCIe-inclusive cost of the host-buffer boundary (hip_proj_step: upload
u, v, w, p from the caller's flow_field, one step, download u, v, w, p --
the path the projection_hip plugin's `step` takes) against the
HBM-resident step (hip_proj_step_device) at N^3 (default 512^3, BASELINE
configs[2]), and the field copy rate from pageable and from pinned host
memory. Then the same STEPS-step cavity run (lid BC re-applied on the host
before each step) through the full-transfer step and through the resident
mode (dirty_faces = 1): the two runs do identical work (same CG iterations,
bitwise-equal results), so the wall-time difference is the transfer saved.
One JSON line.

usage: N=512 python tools/pcie_bench.py
"""
import json
import os
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from cfd_amd import _abi as A  # noqa: E402
from cfd_amd import _native, api  # noqa: E402
from tests import cases  # noqa: E402


def timed(fn, reps=2):
    best = None
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        dt = time.perf_counter() - t0
        best = dt if best is None else min(best, dt)
    return best


def main():
    n = int(os.environ.get("N", "512"))
    g, f, p = cases.cavity(n, n, n, Re=1000.0, dt=1e-4)
    api.cavity_bc(f, 1.0)
    ctx = api.HipProjection(n, n, n)
    gb = n * n * n * 8 / 1e9
    out = {"run": "pcie_boundary", "grid": [n, n, n], "field_GB": round(gb, 4)}

    page = np.random.default_rng(0).standard_normal((n, n, n))
    out["h2d_pageable_GBps"] = gb / timed(lambda: ctx.set_field(A.HIP_FIELD_U, page))
    back = np.empty_like(page)
    lib = _native.hip()

    def get_into(a):
        assert lib.hip_proj_get_field(ctx.ctx, A.HIP_FIELD_U, a.ctypes.data_as(A.c_double_p)) == 0
    out["d2h_pageable_GBps"] = gb / timed(lambda: get_into(back))
    pin = torch.empty((n, n, n), dtype=torch.float64, pin_memory=True).numpy()
    pin[...] = page
    out["h2d_pinned_GBps"] = gb / timed(lambda: ctx.set_field(A.HIP_FIELD_U, pin))
    out["d2h_pinned_GBps"] = gb / timed(lambda: get_into(pin))
    assert np.array_equal(back, page) and np.array_equal(pin, page)
    del page, back, pin

    ctx.upload(f)
    assert ctx.step_device(g, p) == A.CFD_SUCCESS  # warm-up
    ctx.download(f)
    t0 = time.perf_counter()
    assert ctx.step_device(g, p) == A.CFD_SUCCESS
    ctx.synchronize()
    t_dev = time.perf_counter() - t0
    it_dev = ctx.poisson_stats().iterations
    t0 = time.perf_counter()
    assert ctx.step(f, g, p) == A.CFD_SUCCESS, _native.last_error()
    t_host = time.perf_counter() - t0
    it_host = ctx.poisson_stats().iterations
    ctx.close()
    cells = (n - 2) ** 3
    steps = int(os.environ.get("STEPS", "3"))
    runs = {}
    for mode in (0, 1):
        g, f, p = cases.cavity(n, n, n, Re=1000.0, dt=1e-4)
        c = api.HipProjection(n, n, n, dirty_faces=mode)
        walls, its = [], []
        for _ in range(steps):
            api.cavity_bc(f, 1.0)
            t0 = time.perf_counter()
            assert c.step(f, g, p) == A.CFD_SUCCESS, _native.last_error()
            walls.append(time.perf_counter() - t0)
            its.append(c.poisson_stats().iterations)
        t0 = time.perf_counter()
        c.sync_host(f)
        t_sync = time.perf_counter() - t0
        c.close()
        runs[mode] = (walls, its, t_sync, f)
    (wf, itf, _, ff), (wr, itr, t_sync, fr) = runs[0], runs[1]
    assert itf == itr, (itf, itr)
    same = all(np.array_equal(getattr(ff, k), getattr(fr, k)) for k in ("u", "v", "w", "p"))
    ss = slice(1, None)  # steady state: the resident run's first step uploads in full
    mean = lambda a: sum(a[ss]) / len(a[ss])
    out["cavity_run"] = {
        "steps": steps, "cg_iters": itf, "bitwise_equal_after_sync": same,
        "full_transfer_ms": [round(x * 1e3, 2) for x in wf],
        "resident_ms": [round(x * 1e3, 2) for x in wr],
        "sync_host_ms": round(t_sync * 1e3, 2),
        "full_transfer_MLUPS": [round(cells / x / 1e6, 2) for x in wf],
        "resident_MLUPS": [round(cells / x / 1e6, 2) for x in wr],
        "full_transfer_MLUPS_steady": round(cells / mean(wf) / 1e6, 2),
        "resident_MLUPS_steady": round(cells / mean(wr) / 1e6, 2),
        "saved_ms_per_step": round((mean(wf) - mean(wr)) * 1e3, 2)}
    out.update({
        "step_device_ms": round(t_dev * 1e3, 2), "step_device_cg_iters": it_dev,
        "step_device_MLUPS": round(cells / t_dev / 1e6, 2),
        "step_host_buffers_ms": round(t_host * 1e3, 2), "step_host_cg_iters": it_host,
        "step_host_buffers_MLUPS": round(cells / t_host / 1e6, 2),
        "transfer_GB_per_host_step": round(8 * gb, 3)})
    for k in list(out):
        if k.endswith("GBps"):
            out[k] = round(out[k], 2)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
