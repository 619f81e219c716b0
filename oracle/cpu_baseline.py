"""TEST INFRASTRUCTURE ONLY -- the CPU baseline leg of bench.py.

Runs in its own process (bench.py starts it after the GPU timed region, with
OMP_PROC_BIND=close OMP_PLACES=cores and OMP_NUM_THREADS set), so the OpenMP
runtime of the oracle is configured by those variables at load and no HIP
runtime is present in this process. It times the oracle (the C restatement
of the reference's OpenMP projection path, solver_projection_omp.c:26-279 /
linear_solver_cg_omp.c:260-394) on a bounded sample of the bench's workload:
one 512^3 lid-driven cavity step from rest, predictor + divergence +
corrector in full, the first `cg_iters` CG iterations timed and scaled to the
GPU's iterations per step. Prints one JSON object.

The sample is repeated `--repeat` times (fresh fields each time); the value
is the median, with the min and max beside it (the GPU pool's hosts are
shared, and one sample swung 41 % between boxes in round 2).

usage: python -m oracle.cpu_baseline --size N --dt DT --re RE --k-gpu K
                                     --cg-iters C [--scalar-cg-iters S] [--repeat R]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def host_cpu_model():
    try:
        for line in Path("/proc/cpuinfo").read_text().splitlines():
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, required=True)
    ap.add_argument("--dt", type=float, required=True)
    ap.add_argument("--re", type=float, required=True)
    ap.add_argument("--k-gpu", type=float, required=True)
    ap.add_argument("--cg-iters", type=int, default=100)
    ap.add_argument("--scalar-cg-iters", type=int, default=0)
    ap.add_argument("--repeat", type=int, default=3)
    a = ap.parse_args()
    affinity = len(os.sched_getaffinity(0))  # before OpenMP binds this thread

    from cfd_amd import api
    from oracle import oracle

    n = a.size
    threads = int(os.environ.get("OMP_NUM_THREADS", "1"))
    g = api.Grid(n, n, n, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0)
    p = api.validation_params(a.dt, 1.0 / a.re)
    n_int = (n - 2) ** 3

    def sample(nthreads, cg_iters):
        oracle.set_threads(nthreads)
        f = api.FlowField(n, n, n)
        f.rho[...] = 1.0
        api.cavity_bc(f, 1.0)
        oracle.lib().oracle_set_poisson_cap(cg_iters)
        t0 = time.perf_counter()
        s, _, it = oracle.projection_step(f, g, p)
        wall = time.perf_counter() - t0
        oracle.lib().oracle_set_poisson_cap(0)
        ph = oracle.last_phase_ms()
        t_cg_iter = ph[2] / max(it, 1) / 1e3
        t_step = (ph[0] + ph[1] + ph[3]) / 1e3 + a.k_gpu * t_cg_iter
        return s, it, wall, t_cg_iter, t_step

    runs = [sample(threads, a.cg_iters) for _ in range(max(1, a.repeat))]
    vals = sorted(n_int / r[4] / 1e6 for r in runs)
    med = vals[len(vals) // 2]
    s, it, wall, t_cg_iter, t_step = min(runs, key=lambda r: abs(n_int / r[4] / 1e6 - med))
    # CG iteration bytes as the survey credits them (80 B/cell)
    out = {"value": round(med, 4), "unit": "MLUPS", "cores": threads,
           "kind": "port",
           "runs": [round(v, 4) for v in vals], "min": round(vals[0], 4),
           "max": round(vals[-1], 4),
           "sample": (f"{n}^3 cavity step 1 on the host, {len(runs)} times (median reported): "
                      f"predictor+divergence+corrector timed in full, {it} CG iterations "
                      f"timed ({t_cg_iter*1e3:.1f} ms/iter) and scaled to the GPU's "
                      f"{a.k_gpu:.0f} iterations/step; OpenMP x{threads} "
                      f"(OMP_PROC_BIND={os.environ.get('OMP_PROC_BIND')}, "
                      f"OMP_PLACES={os.environ.get('OMP_PLACES')}); sample wall {wall:.1f} s"),
           "cg_iter_ms": round(t_cg_iter * 1e3, 2),
           # timed CG iterations -> the GPU's iterations per step (the factor
           # the sampled CG time is multiplied by)
           "scale_factor": round(a.k_gpu / max(it, 1), 3),
           "cg_iters_timed": it,
           "cg_iter_GBps_80": round(80.0 * n_int / t_cg_iter / 1e9, 2),
           "status": s,
           "host_cpu_model": host_cpu_model(), "host_cpus": os.cpu_count(),
           "affinity_cpus": affinity,
           "omp_proc_bind": os.environ.get("OMP_PROC_BIND"),
           "omp_places": os.environ.get("OMP_PLACES")}
    if a.scalar_cg_iters > 0:
        # the scalar reference configuration: one thread
        s1, it1, wall1, t1_cg, t1_step = sample(1, a.scalar_cg_iters)
        out["scalar_1core"] = {"value": round(n_int / t1_step / 1e6, 4), "unit": "MLUPS",
                               "cores": 1, "cg_iter_ms": round(t1_cg * 1e3, 1),
                               "sample": f"same step, {it1} CG iterations timed, wall {wall1:.1f} s",
                               "status": s1}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
