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


@pytest.mark.parametrize("case,world,size", [("cavity", 2, 66), ("tg", 2, 66), ("cavity", 4, 66),
                                             ("cavity", 8, 130)])
def test_bench_multi_rank_rehearsal(hip_lib, case, world, size):
    """N ranks over RCCL on the one device; 8 ranks is the driver's largest
    launch (here 128 interior planes = 16 per rank)."""
    env = _env()
    env["CFD_BENCH_SHARED_GPU"] = "1"
    # c10d rendezvous on port 0: the agent binds a free port itself (a port
    # probed free here can be taken before torchrun binds it: EADDRINUSE)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--rdzv-backend=c10d", "--rdzv-endpoint=127.0.0.1:0", "--local-addr=127.0.0.1",
           "bench.py", "--gpus", str(world),
           "--size", str(size), "--steps", "2", "--warmup", "1", "--case", case]
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
    cmp = d["cg_variant_compare"]
    assert cmp["cg_variant"] == 1 and cmp["cg_iters"] > 0 and cmp["ms_per_cg_iter_wall"] > 0
