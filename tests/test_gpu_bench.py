"""bench.py's contract on the GPU: the JSON line the driver parses, at a small
size, for one rank and for the N-rank Z-slab path (rehearsed on one GPU with
CFD_BENCH_SHARED_GPU: every rank on device 0, RCCL over its socket
transport). The 8-GPU run itself is the driver's."""
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent
KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
        "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"}


def _last_json(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out[-3000:]
    return json.loads(lines[0])


def _env():
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return env


def test_bench_one_gpu_contract(hip_lib):
    r = subprocess.run([sys.executable, "bench.py", "--size", "66", "--steps", "2", "--warmup",
                        "1", "--cpu-cg-iters", "2"], cwd=ROOT, env=_env(), capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    d = _last_json(r.stdout)
    assert KEYS <= set(d)
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["value"] > 0
    assert d["unit"] == "MLUPS" and d["higher_is_better"] is True
    assert d["roofline"]["bound"] == "hbm" and d["roofline"]["peak"] == 8000.0
    assert 0 < d["roofline"]["frac"] < 1
    cpu = d["cpu_baseline"]
    assert cpu["kind"] == "port" and cpu["cores"] >= 1 and cpu["value"] > 0
    assert cpu["placement"] in ("bound", "unbound") and set(cpu["placements"]) == {"bound",
                                                                                 "unbound"}
    assert d["cg_sweeps"]["cg_sweep_bx"]["kernel"].startswith("k_cgA<")  # the fold sweep


def test_bench_512_single_reduction_default(hip_lib):
    """At 512^3 on one GPU the default CG is the single-reduction z-march
    (bench.cg_variant_auto); its line carries k_ccf's roofline and the textbook
    iteration beside it."""
    r = subprocess.run([sys.executable, "bench.py", "--size", "512", "--steps", "1", "--warmup",
                        "0", "--no-cpu-baseline"], cwd=ROOT, env=_env(), capture_output=True,
                       text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    d = _last_json(r.stdout)
    assert KEYS <= set(d)
    assert d["cg_variant"] == 1 and d["value"] > 0
    assert d["roofline"]["kernel"] == "k_ccf<false, false, false>"
    assert d["roofline"]["bytes_per_cell"] == 40.0 and 0 < d["roofline"]["frac"] < 1
    assert d["cg_iters_per_step"][0] > 0 and d["cg_iter_ms"] > 0
    cmp = d["cg_variant_compare"]
    assert cmp["cg_variant"] == 0 and cmp["cg_iters"] > 0
    # the compare times the main run's first timed step (step 1 here): the
    # same CG iteration count within the variants' rounding
    assert cmp["step"] == 1 and abs(cmp["cg_iters"] - cmp["main_same_step"]["cg_iters"]) <= 2
    # plain and fold launches apart, their counts summing to the iterations
    sp = d["ccf_launches"]
    assert sp["cc_fused"]["launches"] + sp["cc_fold"]["launches"] == sum(d["cg_iters_per_step"])
    assert sp["cc_fold"]["avg_ms"] > sp["cc_fused"]["avg_ms"] > 0
    # the march's effective shader clock over the timed region
    clk = d["clock"]
    assert clk["sampled_workgroups"] > 0 and 500.0 < clk["k_ccf_shader_MHz"] < 3000.0
    # the reference caller's step on host buffers beside the resident one
    pl = d["plugin_step"]
    assert pl["full"]["cg_iters"] == pl["resident"]["cg_iters"] == pl["dirty_faces"]["cg_iters"]
    assert pl["ms_full"] > pl["ms_resident"] > 0 and pl["ms_dirty_faces"] > 0
    assert 0 < pl["pcie_share"]["full"] < 1


@pytest.mark.parametrize("case,world,size,cgv,probe", [("cavity", 2, 66, -1, "auto"),
                                                        ("tg", 2, 66, -1, "auto"),
                                                        ("cavity", 2, 66, -1, "on"),
                                                        ("cavity", 4, 66, 1, "auto"),
                                                        ("cavity", 8, 130, 1, "auto")])
def test_bench_multi_rank_rehearsal(hip_lib, case, world, size, cgv, probe):
    """N ranks over RCCL on the one device; 8 ranks is the driver's largest
    launch (here 128 interior planes = 16 per rank). cgv -1: the bench's own
    choice (textbook CG below 512^3), 1: the single-reduction slab form;
    probe "on": both forms step first and the faster per CG iteration runs
    (the default at 512^3 on N > 1)."""
    env = _env()
    env["CFD_BENCH_SHARED_GPU"] = "1"
    # c10d rendezvous on port 0: the agent binds a free port itself (a port
    # probed free here can be taken before torchrun binds it: EADDRINUSE)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--rdzv-backend=c10d", "--rdzv-endpoint=127.0.0.1:0", "--local-addr=127.0.0.1",
           "bench.py", "--gpus", str(world),
           "--size", str(size), "--steps", "2", "--warmup", "1", "--case", case,
           "--cg-variant", str(cgv), "--cg-probe", probe]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    d = _last_json(r.stdout)
    assert KEYS <= set(d)
    assert d["n_gpus"] == world and d["value"] > 0 and d["scaling"] == "strong"
    assert d["cpu_baseline"] is None  # CPU baseline at N=1 only
    assert f"z-slab x{world}" in d["config"]["parallelism"]
    # per-rank device times (sweeps, halo, all-reduce) for reading the 1 -> N curve
    ranks = d["ranks"]
    assert [q["rank"] for q in ranks] == list(range(world))
    for q in ranks:
        assert q["sweep_ms_per_iter"] > 0 and q["halo_ms_per_iter"] > 0
        if q["dot_allreduce"] == "ncclAllReduce":
            assert q["allreduce_ms_per_iter"] > 0
    # the other CG variant measured beside the timed region
    # the other CG variant than the timed one (cavity slabs: single-reduction
    # timed, textbook beside it; Taylor-Green: the other way round)
    choice = d["cg_variant_choice"]
    if probe == "on":
        pr = choice["probe"]
        assert pr["budget_pick"] == 0 and d["cg_variant"] == pr["picked"]
        # both forms stepped the same steps of the trajectory
        assert pr["cg0"]["cg_iters"] > 0 and pr["cg1"]["cg_iters"] > 0
        faster = min((0, 1), key=lambda v: pr[f"cg{v}"]["ms_per_cg_iter"])
        assert pr["picked"] == faster
    else:
        assert "probe" not in choice
        assert d["cg_variant"] == (cgv if cgv >= 0 else 0)
    cmp = d["cg_variant_compare"]
    assert cmp["cg_variant"] == 1 - d["cg_variant"] and cmp["cg_iters"] > 0
    assert cmp["ms_per_cg_iter_wall"] > 0


def _oracle_convection(nx, ny, nz, steps, tol):
    """The oracle's run of bench.convection_setup: RB-SOR projection steps
    with the energy equation (solver_projection.c:46-297 with the RB-SOR
    solve, energy_solver.c:21-334)."""
    import numpy as np

    sys.path.insert(0, str(ROOT))
    import bench
    from cfd_amd import _abi as A
    from cfd_amd import api
    from oracle import oracle

    g, p, T0 = bench.convection_setup(nx, ny, nz)
    f = api.FlowField(nx, ny, nz)
    f.u[...] = f.v[...] = f.w[...] = f.p[...] = 0.0
    f.rho[...] = 1.0
    f.T[...] = np.broadcast_to(T0[None, None, :], f.T.shape)
    oracle.set_projection_poisson_params(oracle.poisson_params(tolerance=tol,
                                                               max_iterations=20000))
    its = []
    try:
        for _ in range(steps):
            s, _, it = oracle.projection_step(f, g, p, A.ORACLE_POISSON_REDBLACK)
            assert s == A.CFD_SUCCESS
            its.append(it)
    finally:
        oracle.set_projection_poisson_params(None)
    return f, its


@pytest.mark.parametrize("world", [1, 2])
def test_bench_convection_launcher_bitwise(hip_lib, tmp_path, world):
    """configs[4]'s launcher (bench.py --case convection): 1 rank, and 2 ranks
    over RCCL (shared device), at 24 x 24 x 18 with the RB-SOR tolerance
    at 1e-3 (this small Neumann problem stalls above 1e-6); every rank's
    owned planes of u, v, w, p, T and the RB-SOR iteration counts bitwise
    the oracle's."""
    import numpy as np

    nx, nz, steps = 24, 18, 2
    dump = tmp_path / "conv"
    args = ["bench.py", "--gpus", str(world), "--case", "convection", "--size", str(nx),
            "--nz", str(nz), "--steps", str(steps), "--warmup", "0", "--relax-tol", "1e-3",
            "--dump", str(dump)]
    env = _env()
    if world > 1:
        env["CFD_BENCH_SHARED_GPU"] = "1"
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={world}", "--rdzv-backend=c10d",
               "--rdzv-endpoint=127.0.0.1:0", "--local-addr=127.0.0.1"] + args
    else:
        cmd = [sys.executable] + args
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    d = _last_json(r.stdout)
    assert KEYS <= set(d) and d["n_gpus"] == world and d["value"] > 0
    assert len(d["ranks"]) == world
    for q in d["ranks"]:
        assert q["relax_sweep_ms_per_iter"] > 0
        if world > 1:
            assert q["relax_halo_ms_per_iter"] > 0
    if world == 1:
        # one GPU in 3-D: two RB-SOR iterations per sweep (k_rb2)
        assert 0 < d["roofline"]["frac"] < 1 and d["roofline"]["kernel"].startswith("k_rb2")
    fo, its = _oracle_convection(nx, nx, nz, steps, 1e-3)
    assert all(i > 10 for i in its)
    assert d["rbsor_iters_per_step"] == its
    got = {k: np.full((nz, nx, nx), np.nan) for k in ("u", "v", "w", "p", "T")}
    for rk in range(world):
        z = np.load(f"{dump}.rank{rk}.npz")
        assert list(z["iters"]) == its
        for k in got:
            got[k][int(z["k0"]):int(z["k1"])] = z[k]
    for k, a in got.items():
        np.testing.assert_array_equal(a, getattr(fo, k), err_msg=k)
