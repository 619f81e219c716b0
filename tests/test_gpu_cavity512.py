"""BASELINE configs[2] at its own size: the bench's 512^3 lid-driven cavity
trajectory (Re = 1000, dt = 1e-4, from rest, lid u = 1 on y = 1, the
reference's CG settings) against the oracle's run of the same steps,
committed as fixtures by tests/golden/make_golden.py cavity512 (the OpenMP
oracle, solver_projection.c:46-297 with cg_scalar_solve's loop,
linear_solver_cg.c:290-461; about 2.5 h on 8 cores).

The device path is driven exactly as bench.py drives it: fields filled on
the device, the caller BCs applied once (the step keeps the boundary faces),
projection_hip steps on the resident fields. Per step: CG iterations within
1 (the dot products are summed in another order), the initial CG residual
within 1e-6 relative and the final one within 1e-4 (it is 1e-6 of the
initial one, after ~1000 recursive updates), the interior L2 norm and max |.| of u, v,
w, p within 1e-9 relative; after steps 1, 6 and 25 the sampled planes
k = 1, 255, 510 (a stride-4 lattice, rows j = 1, 255, 509, 510, columns
i = 1, 255, 510) within 1e-9 of the field's largest interior value. The reference's
own backend-consistency bar is 1e-3 (tests/validation/test_cavity_backends.c:43)."""
import ctypes as C
import json
from pathlib import Path

import numpy as np
import pytest

from cfd_amd import _abi as A
from cfd_amd import api

pytestmark = pytest.mark.gpu

GOLD = Path(__file__).resolve().parent / "golden"
N = 512
REL = 1e-9


def _fixture():
    f = GOLD / f"cavity{N}_re1000_steps.json"
    if not f.exists():
        pytest.skip("512^3 fixture not generated (tests/golden/make_golden.py cavity512)")
    return json.loads(f.read_text())


def _interior_norms(a):
    import torch
    t = torch.from_numpy(a)[1:-1, 1:-1, 1:-1]
    return float(torch.linalg.vector_norm(t)), float(t.abs().max())


FIDS = {"u": A.HIP_FIELD_U, "v": A.HIP_FIELD_V, "w": A.HIP_FIELD_W, "p": A.HIP_FIELD_P}


def _init(ctx):
    """bench.py's make_ctx: fields filled on the device, caller BCs once."""
    for fid in FIDS.values():
        ctx.fill(fid, 0.0)
    ctx.set_density(1.0)
    ctx.apply_dirichlet(A.HIP_FIELD_U, api.dirichlet(top=1.0))
    ctx.apply_dirichlet(A.HIP_FIELD_V, api.dirichlet())
    ctx.apply_dirichlet(A.HIP_FIELD_W, api.dirichlet())
    ctx.apply_scalar_bc(A.HIP_FIELD_P, A.BC_TYPE_NEUMANN)


def check_step(row, iters, res0, res, vmax, pmax, field, worst):
    """One step against the fixture row: CG iterations +-1, residuals,
    max |u| / |p|, interior norms and (where committed) the sampled planes;
    field(k) returns the whole n^3 array of field k."""
    assert abs(iters - row["cg_iters"]) <= 1, (row["step"], iters, row["cg_iters"])
    assert res0 == pytest.approx(row["initial_residual"], rel=1e-6)
    # the final residual is the recursively updated r after ~1000
    # iterations, 1e-6 of the initial one: its rounding differs at
    # ~1e-6 relative (1e-12 of the initial residual)
    assert res == pytest.approx(row["final_residual"], rel=1e-4)
    assert vmax == pytest.approx(row["max_velocity"], rel=REL)
    assert pmax == pytest.approx(row["max_pressure"], rel=REL)
    snap = GOLD / f"cavity{N}_re1000_step{row['step']}_planes.npz"
    for k in FIDS:
        a = field(k)
        l2, mx = _interior_norms(a)
        ol2, omx = row["norms"][k]
        worst["norm_rel"] = max(worst["norm_rel"], abs(l2 - ol2) / ol2, abs(mx - omx) / omx)
        assert l2 == pytest.approx(ol2, rel=REL, abs=1e-300), (row["step"], k)
        assert mx == pytest.approx(omx, rel=REL, abs=1e-300), (row["step"], k)
        if snap.exists():
            z = np.load(snap)
            for kz in (1, 255, 510):
                pre = f"{k}_k{kz}_"
                plane = a[kz]
                # the field's scale (its interior max |.|): w on the
                # mid-plane k = 255 is ~0 by the z symmetry
                scale = max(float(z[pre + "stats"][2]), omx, 1e-300)
                li = z[pre + "lattice_idx"]
                got = {"lattice": plane[np.ix_(li, li)],
                       "rows": plane[z[pre + "rows_j"], :],
                       "cols": plane[:, z[pre + "cols_i"]].T}
                for part, val in got.items():
                    d = float(np.max(np.abs(val - z[pre + part]))) / scale
                    worst["plane_rel"] = max(worst["plane_rel"], d)
                    assert d <= REL, (row["step"], k, kz, part, d)
                s_sum, s_l2, s_max = z[pre + "stats"]
                # whole-plane L2 and max, also on the field's scale
                # (the L2 of n^2 cells: scale * n)
                assert float(np.sqrt(np.sum(plane * plane))) == pytest.approx(
                    s_l2, rel=REL, abs=REL * scale * plane.shape[0])
                assert float(np.max(np.abs(plane))) == pytest.approx(
                    s_max, rel=REL, abs=REL * scale)


@pytest.mark.timeout(900)
def test_cavity512_trajectory_vs_oracle(hip_lib):
    rec = _fixture()
    steps = rec["steps"]
    g = api.Grid(N, N, N, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0)
    params = api.validation_params(rec["dt"], 1.0 / rec["re"])
    ctx = api.HipProjection(N, N, N)
    try:
        _init(ctx)
        its = []
        worst = {"norm_rel": 0.0, "plane_rel": 0.0}
        for row in steps:
            st = A.SolverStats()
            s = ctx.step_device(g, params, st)
            assert s == A.CFD_SUCCESS, (row["step"], s, api._native.last_error())
            ps = ctx.poisson_stats()
            its.append((ps.iterations, row["cg_iters"]))
            check_step(row, ps.iterations, ps.initial_residual, ps.final_residual,
                       st.max_velocity, st.max_pressure, lambda k: ctx.get_field(FIDS[k]), worst)
    finally:
        ctx.close()
    print("cavity512 CG iterations (device, oracle):", its)
    print("cavity512 largest deviations from the oracle:", worst)


@pytest.mark.timeout(900)
def test_cavity512_single_reduction_cg_vs_oracle(hip_lib):
    """The north star's single-reduction CG (cg_variant 1: one reduction per
    iteration, on one device the fused march k_ccf) on the whole 25-step
    trajectory bench.py times (steps 6-25 after 5 warm-up steps, the 1063 ->
    1212 iteration jump at step 15 included), against the textbook-CG oracle
    at the single-device bars, with the sampled planes after steps 1, 6 and 25
    (it is the same Krylov method with other rounding: the iteration counts
    come out identical, profiles/r04_cc_cavity512_vs_oracle.jsonl)."""
    rec = _fixture()
    g = api.Grid(N, N, N, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0)
    params = api.validation_params(rec["dt"], 1.0 / rec["re"])
    ctx = api.HipProjection(N, N, N, cg_variant=1)
    try:
        _init(ctx)
        its = []
        worst = {"norm_rel": 0.0, "plane_rel": 0.0}
        for row in rec["steps"]:
            st = A.SolverStats()
            s = ctx.step_device(g, params, st)
            assert s == A.CFD_SUCCESS, (row["step"], s, api._native.last_error())
            ps = ctx.poisson_stats()
            its.append((ps.iterations, row["cg_iters"]))
            check_step(row, ps.iterations, ps.initial_residual, ps.final_residual,
                       st.max_velocity, st.max_pressure, lambda k: ctx.get_field(FIDS[k]), worst)
    finally:
        ctx.close()
    assert len(its) == 25
    print("cavity512 single-reduction CG iterations (device, oracle):", its)
    print("cavity512 single-reduction CG, largest deviations from the oracle:", worst)


@pytest.mark.timeout(600)
def test_cavity512_cg1_plugin_vs_oracle(hip_lib):
    """The single-reduction CG through the reference interface: the registry
    name projection_hip_cg1 (cfd_hip_register_solvers, reached by
    cfd_registry_register_defaults / init_simulation_with_solver,
    solver_registry.c:213-279) driven by solver_init + solver_step on host
    buffers, steps 1-2 of the trajectory against the fixture."""
    rec = _fixture()
    g = api.Grid(N, N, N, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0)
    params = api.validation_params(rec["dt"], 1.0 / rec["re"])
    f = api.FlowField(N, N, N)
    for k in ("u", "v", "w", "p", "T"):
        getattr(f, k)[...] = 0.0
    f.rho[...] = 1.0
    api.cavity_bc(f, 1.0)  # the caller BCs once, as the fixture's run
    reg = api.Registry()
    solver = reg.create("projection_hip_cg1")
    try:
        assert solver.name == "projection_hip_cg1"
        assert solver.init(g, params) == A.CFD_SUCCESS, api._native.last_error()
        ctx = solver._ptr.contents.context
        assert ctx  # the plugin's context exists after init
        # the plugin keeps the hip_proj context as the first member of its own
        hctx = C.cast(ctx, C.POINTER(C.c_void_p))[0]
        lib = api._native.hip()
        lib.hip_proj_enable_timing(hctx, 1)
        worst = {"norm_rel": 0.0, "plane_rel": 0.0}
        for row in rec["steps"][:2]:
            st = A.SolverStats()
            s = solver.step(f, g, params, st)
            assert s == A.CFD_SUCCESS, (row["step"], s, api._native.last_error())
            assert st.iterations == 1
            ps = A.PoissonStats()
            assert lib.hip_proj_get_poisson_stats(hctx, C.byref(ps)) == 0
            check_step(row, ps.iterations, ps.initial_residual, ps.final_residual,
                       st.max_velocity, st.max_pressure, lambda k: getattr(f, k), worst)
        # the fused single-reduction march ran, one launch per CG iteration
        ms = (C.c_double * 64)()
        n = (C.c_longlong * 64)()
        assert lib.hip_proj_get_timing_n(hctx, ms, n, 64) == A.HIP_KT_COUNT
        total_its = sum(r["cg_iters"] for r in rec["steps"][:2])
        kt = {k: n[i] for i, k in enumerate(A.KERNEL_TIMERS)}
        # plain (+ first) launches and x-fold launches time apart (ABI 3)
        assert abs(kt["cc_fused"] + kt["cc_fold"] - total_its) <= 2, (kt, total_its)
        assert kt["cc_fold"] > 0
        assert kt["cg_sweep_a"] == 0 and kt["cg_sweep_b"] == 0, kt
    finally:
        solver.close()
    print("cavity512 through projection_hip_cg1, largest deviations from the oracle:", worst)


@pytest.mark.timeout(900)
@pytest.mark.parametrize("cgv,nsteps", [(0, 6), (1, 3)], ids=["textbook", "single_reduction"])
def test_cavity512_slabs8_vs_oracle(hip_lib, monkeypatch, cgv, nsteps):
    """configs[3]'s decomposition at its real slab depth (VERDICT r03 item
    3): the same trajectory on 8 in-process Z-slab ranks (64 planes each,
    6 x 64 + 2 x 63 interior planes) against the fixture with the
    single-device bars; every rank's CG statistics must agree (one all-ranks
    reduction per dot product). Textbook CG steps 1-6; the single-reduction
    CG (cg_variant 1, what bench.py runs at N > 1: the fused slab form, one
    all-reduce per iteration) steps 1-3."""
    monkeypatch.setenv("CFD_HIP_GROUP_TIMEOUT_S", "120")
    rec = _fixture()
    steps = rec["steps"][:nsteps]
    g = api.Grid(N, N, N, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0)
    params = api.validation_params(rec["dt"], 1.0 / rec["re"])
    nr = 8
    grp = api.LocalGroup(nr)
    ctxs = [api.HipProjection(N, N, N, comm=grp.comm(r, 0), cg_variant=cgv) for r in range(nr)]
    assert [c.nz_local - 2 for c in ctxs] == [64] * 6 + [63] * 2
    try:
        api.run_ranks(lambda r: _init(ctxs[r]), nr)  # BCs are per-rank collective calls

        def body(r):
            st = A.SolverStats()
            s = ctxs[r].step_device(g, params, st)
            ps = ctxs[r].poisson_stats()
            return s, ps.iterations, ps.initial_residual, ps.final_residual, st.max_velocity, \
                st.max_pressure

        its = []
        worst = {"norm_rel": 0.0, "plane_rel": 0.0}
        for row in steps:
            out = api.run_ranks(body, nr)
            for r, o in enumerate(out):
                assert o[0] == A.CFD_SUCCESS, (row["step"], r, o[0], api._native.last_error())
                assert o[1:4] == out[0][1:4], (row["step"], r)  # the same CG decisions
            s, it, r0, r1, vmax, pmax = out[0]
            vmax = max(o[4] for o in out)
            pmax = max(o[5] for o in out)
            its.append((it, row["cg_iters"]))

            def field(k):
                a = np.empty((N, N, N))
                for c in ctxs:
                    loc, glob = c.owned()
                    a[glob] = c.get_field(FIDS[k])[loc]
                return a

            check_step(row, it, r0, r1, vmax, pmax, field, worst)
    finally:
        for c in ctxs:
            c.close()
        grp.close()
    print(f"cavity512 on 8 slabs (cg_variant {cgv}), CG iterations (device, oracle):", its)
    print(f"cavity512 on 8 slabs (cg_variant {cgv}), largest deviations from the oracle:", worst)


@pytest.mark.timeout(1200)
@pytest.mark.parametrize("world,cgv,nsteps", [(2, 0, 2), (2, 1, 25), (4, 1, 6)],
                         ids=["rccl2_textbook", "rccl2_single_reduction_25",
                              "rccl4_single_reduction_6"])
def test_cavity512_rccl_vs_oracle(hip_lib, tmp_path, world, cgv, nsteps):
    """The bench's N > 1 path: the trajectory on RCCL Z-slab ranks (one
    process per rank, sharing the device through RCCL's socket transport)
    with the device-mailbox all-reduce of the CG dot products
    (tests/rccl_cavity512_worker.py), against the fixture at the
    single-device bars: per-rank CG statistics, interior norms from the
    ranks' partial sums and the sampled planes each rank owns after steps 1,
    6 and 25. The single-reduction CG (the fused slab form, one mailbox
    all-reduce per iteration) over all 25 steps on 2 ranks -- steps 6-25 are
    bench.py's timed steps, the 1063 -> 1212 iteration jump at step 15
    included -- and steps 1-6 on 4 ranks (128-plane slabs); textbook CG steps
    1-2 on 2. Every step of every rank must have run its dots over the
    mailbox: no ncclAllReduce span in its timers, and for the
    single-reduction CG one interior march launch per iteration."""
    import os
    import subprocess
    import sys

    rec = _fixture()
    root = Path(__file__).resolve().parents[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["CFD_HIP_DEVICE_ALLREDUCE"] = "1"
    out = tmp_path / "rccl512.json"
    env["CFD_CAV512_OUT"] = str(out)
    env["CFD_CAV512_CG_VARIANT"] = str(cgv)
    env["CFD_CAV512_STEPS"] = str(nsteps)
    psteps = [s for s in (1, 6, 25) if s <= nsteps]
    env["CFD_CAV512_PLANE_STEPS"] = ",".join(map(str, psteps))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--rdzv-backend=c10d", "--rdzv-endpoint=127.0.0.1:0",
           "--local-addr=127.0.0.1", str(root / "tests" / "rccl_cavity512_worker.py")]
    # the workers' per-step progress lines pass through (visible with -s)
    proc = subprocess.Popen(cmd, cwd=root, env=env, stdout=subprocess.PIPE,
                            stderr=subprocess.STDOUT, text=True)
    log = []
    for line in proc.stdout:
        log.append(line)
        print(line, end="", flush=True)
    rc = proc.wait(timeout=60)
    assert rc == 0, "".join(log)[-3000:]
    got = json.loads(out.read_text())
    assert got["world"] == world and got["device_allreduce"] is True
    assert len(got["steps"]) == nsteps
    worst = {"norm_rel": 0.0, "plane_rel": 0.0}
    for row, g in zip(rec["steps"][:nsteps], got["steps"]):
        assert g["device_allreduce"] is True, row["step"]
        for rk, red in enumerate(g["reduction"]):
            assert red["allreduce_spans"] == 0, (row["step"], rk, red)  # mailbox, every step
            if cgv == 1:
                assert abs(red["march_launches"] - g["iters"]) <= 1, (row["step"], rk, red)
            else:
                assert abs(red["sweep_a_launches"] - g["iters"]) <= 1, (row["step"], rk, red)
        assert abs(g["iters"] - row["cg_iters"]) <= 1, (row["step"], g["iters"])
        assert g["res0"] == pytest.approx(row["initial_residual"], rel=1e-6)
        assert g["res"] == pytest.approx(row["final_residual"], rel=1e-4)
        assert g["vmax"] == pytest.approx(row["max_velocity"], rel=REL)
        assert g["pmax"] == pytest.approx(row["max_pressure"], rel=REL)
        for k in FIDS:
            ol2, omx = row["norms"][k]
            worst["norm_rel"] = max(worst["norm_rel"], abs(g["norms"][k][0] - ol2) / ol2)
            assert g["norms"][k][0] == pytest.approx(ol2, rel=REL, abs=1e-300), (row["step"], k)
            assert g["norms"][k][1] == pytest.approx(omx, rel=REL, abs=1e-300), (row["step"], k)
    # the sampled planes, from the rank that owns each
    planes = np.load(tmp_path / "rccl512_planes.npz")
    for st in psteps:
        z = np.load(GOLD / f"cavity{N}_re1000_step{st}_planes.npz")
        for k in FIDS:
            omx = rec["steps"][st - 1]["norms"][k][1]
            for kz in (1, 255, 510):
                pre = f"{k}_k{kz}_"
                plane = planes[f"{k}_{kz}_s{st}"]
                scale = max(float(z[pre + "stats"][2]), omx, 1e-300)
                li = z[pre + "lattice_idx"]
                got_p = {"lattice": plane[np.ix_(li, li)],
                         "rows": plane[z[pre + "rows_j"], :],
                         "cols": plane[:, z[pre + "cols_i"]].T}
                for part, val in got_p.items():
                    d = float(np.max(np.abs(val - z[pre + part]))) / scale
                    worst["plane_rel"] = max(worst["plane_rel"], d)
                    assert d <= REL, (st, k, kz, part, d)
    print(f"cavity512 on {world} RCCL ranks (cg_variant {cgv}, {nsteps} steps), iterations:",
          [g["iters"] for g in got["steps"]], "largest deviations:", worst)
