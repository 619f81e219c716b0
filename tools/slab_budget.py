#!/usr/bin/env python3
"""Per-iteration budget of one Z-slab rank's CG iteration at N = 2, 4, 8 on
512^3, every piece timed on ONE GPU as its own line,
then the projected per-iteration time of both CG forms and the projected
1 -> N speedup. Writes one JSON object (stdout, and --out).

Pieces (device time per iteration, kernel events of the context's timers;
fixed iterations, tolerance 0, a random right-hand side):
  march_P      single-device k_ccf on the rank's slab shape 512 x 512 x (P+2):
               the interior launch's march with stage c (an upper bound: it
               covers P planes, the slab's interior launch P - 2)
  textbook_P   single-device sweeps A + B (+ the fold) on the same shape
  edge2_ccf    k_ccf on 512 x 512 x 4 (2 planes): proxy of the edge planes'
               k_ccf<NOC> launch (342 one-plane tiles there, 171 two-plane here)
  edge2_cc2    k_cc2 on those 2 planes (CFD_HIP_CCF=0 form): the edge SpMV
  edge2_sweepB sweep B on those 2 planes: textbook's edge launch
  plane_copy   one 2 MiB plane device-to-device on this GPU (HBM; the xGMI
               transfer is estimated from the link rate below)
  allreduce    the 2-value dot all-reduce on 2 / 4 / 8 RCCL ranks sharing this
               GPU (hip_proj_comm_mailbox_bench): mode 0 mailbox round trip,
               mode 1 one launch + mailbox, mode 2 ncclAllReduce + a kernel;
               launch_gap = mode 1 - mode 0. Ranks sharing one device are a
               lower bound for the round trip over xGMI
Projection (rank 0's slab, halo overlapped with the interior launch):
  cg1 = march_P + edge2_ccf + edge2_cc2 + rt + 3 gap + max(0, halo - march_P)
  cg0 = textbook_P + edge2_sweepB + 2 rt + 3 gap + max(0, halo - sweepB_P)
  halo = 2 MiB / XGMI_GBPS + RCCL_US (two neighbours on separate links, in
  parallel)

usage: python tools/slab_budget.py [--iters 100] [--out profiles/r06_slab_budget.json]
       (the allreduce part starts torch.distributed.run itself)
"""
import argparse
import json
import os
import subprocess
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

N = 512
XGMI_GBPS = 64.0   # assumed per-direction rate of one xGMI link for a 2 MiB plane
RCCL_US = 10.0     # assumed fixed cost of a grouped send/recv on the halo stream


def slab_planes(world):
    """Interior planes of rank 0 (the largest slab) of 512^3 on `world` ranks."""
    nint = N - 2
    return nint // world + (1 if nint % world else 0)


def per_iter(nx, ny, nz, variant, iters, env=None):
    import numpy as np

    from cfd_amd import _abi as A
    from cfd_amd import _native, api

    saved = {}
    for k, v in (env or {}).items():
        saved[k] = os.environ.get(k)
        os.environ[k] = v
    try:
        ctx = api.HipProjection(nx, ny, nz, cg_variant=variant)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    rng = np.random.default_rng(1)
    rhs = np.zeros((nz, ny, nx))
    rhs[1:-1, 1:-1, 1:-1] = rng.standard_normal((nz - 2, ny - 2, nx - 2))
    h = 1.0 / (nx - 1)
    prm = _native.host().poisson_solver_params_default()
    prm.max_iterations = iters
    prm.tolerance = 0.0
    prm.absolute_tolerance = 0.0
    x = np.zeros_like(rhs)
    ctx.poisson_solve(A.HIP_POISSON_CG, x, rhs, h, h, h, prm)  # warm-up
    best = None
    for _ in range(3):  # median of three timed solves
        x[...] = 0.0
        ctx.reset_timing()
        ctx.enable_timing(True)
        s, st = ctx.poisson_solve(A.HIP_POISSON_CG, x, rhs, h, h, h, prm)
        ctx.enable_timing(False)
        kt = ctx.timing()
        per = {k: v[0] / st.iterations for k, v in kt.items() if v[1] and k != "cg_setup"}
        loop = sum(per.values())
        best = sorted((best or []) + [(loop, per)], key=lambda t: t[0])
    ctx.close()
    loop, per = best[len(best) // 2]
    return round(loop, 5), {k: round(v, 5) for k, v in per.items()}


def plane_copy_us():
    import torch
    n = N * N
    a = torch.empty(n, dtype=torch.float64, device="cuda")
    b = torch.empty_like(a)
    for _ in range(10):
        b.copy_(a)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(200):
        b.copy_(a)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / 200


def allreduce_worker():
    """One rank of the all-reduce microbenchmark (under torch.distributed.run)."""
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    os.environ["NCCL_HOSTID"] = f"cfd-budget-rank{rank}"
    import torch  # noqa: F401
    import torch.distributed as dist

    from cfd_amd import api

    dist.init_process_group("gloo")
    uid = [api.comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    comm = api.SlabComm.rccl(uid[0], rank, world, 0)
    out = {"world": world, "device_allreduce": comm.device_allreduce}
    # 8 processes sharing one GPU's queues time-slice: fewer exchanges there
    iters = int(os.environ.get("CFD_BUDGET_AR_ITERS", "2000" if world <= 4 else "100"))
    for mode in (0, 1, 2):
        if mode < 2 and not comm.device_allreduce:
            continue
        comm.allreduce_bench(50, mode)  # warm-up
        out[f"mode{mode}_us"] = round(comm.allreduce_bench(iters, mode), 3)
    allv = [None] * world
    dist.all_gather_object(allv, out)
    comm.close()
    if rank == 0:
        # the slowest rank's figure per mode
        res = {"world": world, "device_allreduce": all(v["device_allreduce"] for v in allv)}
        for m in (0, 1, 2):
            vals = [v[f"mode{m}_us"] for v in allv if f"mode{m}_us" in v]
            if vals:
                res[f"mode{m}_us"] = max(vals)
        print("ALLREDUCE " + json.dumps(res), flush=True)
    dist.destroy_process_group()


def allreduce_run(world):
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["CFD_HIP_DEVICE_ALLREDUCE"] = "1"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--rdzv-backend=c10d", "--rdzv-endpoint=127.0.0.1:0",
           "--local-addr=127.0.0.1", str(Path(__file__).resolve()), "--allreduce-worker"]
    import signal
    # its own process group: on a timeout the launcher AND its ranks go
    p = subprocess.Popen(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                         text=True, start_new_session=True)
    try:
        so, se = p.communicate(timeout=150)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.communicate()
        return {"world": world, "error": "timeout 150 s (ranks sharing one GPU's queues)"}
    if p.returncode != 0:
        return {"world": world, "error": (so + se)[-800:]}
    for line in so.splitlines():
        if line.startswith("ALLREDUCE "):
            return json.loads(line[len("ALLREDUCE "):])
    return {"world": world, "error": "no result line"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--out", default="")
    ap.add_argument("--worlds", default="2,4,8")
    ap.add_argument("--allreduce-worker", action="store_true")
    ap.add_argument("--k-mean", type=float, default=1147.1,
                    help="mean CG iterations per timed step (steps 6-25 of the cavity512 fixture)")
    ap.add_argument("--other-ms", type=float, default=13.0,
                    help="one-GPU non-CG ms per step (predictor, setup, corrector, ...)")
    ap.add_argument("--pieces", default="",
                    help="reuse the pieces of an earlier run (its JSON) and measure only "
                         "the all-reduce worlds they lack")
    args = ap.parse_args()
    if args.allreduce_worker:
        allreduce_worker()
        return
    import torch  # noqa: F401  (one HIP runtime in the process)

    worlds = [int(w) for w in args.worlds.split(",") if w]
    t0 = time.time()
    if args.pieces:
        pieces = json.loads(Path(args.pieces).read_text())["pieces"]
        ar = pieces.setdefault("allreduce", {})
        for world in worlds:
            if "mode0_us" not in ar.get(str(world), {}) and world <= 4:
                ar[str(world)] = allreduce_run(world)
                print(json.dumps({"piece": "allreduce", **ar[str(world)]}), flush=True)
        return finish(args, worlds, pieces, t0)
    pieces = {}
    one = {"cg1": per_iter(N, N, N, 1, args.iters), "cg0": per_iter(N, N, N, 0, args.iters)}
    pieces["one_gpu_512"] = {k: {"ms": v[0], "timers": v[1]} for k, v in one.items()}
    print(json.dumps({"piece": "one_gpu_512", **pieces["one_gpu_512"]}), flush=True)
    for world in worlds:
        P = slab_planes(world)
        # the slab interior launch's z-run length (projection_hip.hip init_ctx:
        # 11 on slabs of <= 100 planes, else 16), forced on the one-device shape
        kc = {"CFD_HIP_CCF_KC": "11" if P <= 100 else "16", "CFD_HIP_CCF_KC_FIXED": "1"}
        c1 = per_iter(N, N, P + 2, 1, args.iters, kc)
        c0 = per_iter(N, N, P + 2, 0, args.iters)
        pieces[f"slab_{world}"] = {"planes": P, "march_P": {"ms": c1[0], "timers": c1[1]},
                                   "textbook_P": {"ms": c0[0], "timers": c0[1]}}
        print(json.dumps({"piece": f"slab_{world}", **pieces[f"slab_{world}"]}), flush=True)
    e1 = per_iter(N, N, 4, 1, args.iters)
    e2 = per_iter(N, N, 4, 1, args.iters, {"CFD_HIP_CCF": "0"})
    e0 = per_iter(N, N, 4, 0, args.iters)
    pieces["edge2"] = {"ccf": {"ms": e1[0], "timers": e1[1]},
                       "cc2": {"ms": e2[1].get("cc_spmv"), "timers": e2[1]},
                       "sweepB": {"ms": e0[1].get("cg_sweep_b"), "timers": e0[1]}}
    print(json.dumps({"piece": "edge2", **pieces["edge2"]}), flush=True)
    pieces["plane_copy_us"] = round(plane_copy_us(), 2)
    print(json.dumps({"piece": "plane_copy_us", "us": pieces["plane_copy_us"]}), flush=True)
    ar = {}
    for world in worlds:
        if world > 4:  # 8 processes time-slice one GPU (11 ms per exchange in r06c)
            continue
        ar[str(world)] = allreduce_run(world)
        print(json.dumps({"piece": "allreduce", **ar[str(world)]}), flush=True)
    pieces["allreduce"] = ar
    finish(args, worlds, pieces, t0)


def finish(args, worlds, pieces, t0):
    ar = pieces["allreduce"]
    # one 2 MiB plane per neighbour, the two on separate links in parallel
    halo_ms = (1.0 * N * N * 8 / (XGMI_GBPS * 1e9) * 1e3) + RCCL_US * 1e-3
    # mailbox figures from ranks sharing one GPU are valid while every rank's
    # one-wave kernel stays resident; at 8 processes the GPU time-slices their
    # queues (ms per exchange): those worlds take the line through the valid
    # ones (a lower bound's extrapolation, marked as such)
    valid = sorted((int(w), a) for w, a in ar.items()
                   if "mode0_us" in a and "mode1_us" in a and a["mode0_us"] < 100.0)

    def rt_gap(world):
        for w, a in valid:
            if w == world:
                return a["mode0_us"], a["mode1_us"] - a["mode0_us"], "measured (ranks sharing one GPU)"
        if len(valid) < 2:
            return None
        (w0, a0), (w1, a1) = valid[-2], valid[-1]
        slope = (a1["mode0_us"] - a0["mode0_us"]) / (w1 - w0)
        rt = a1["mode0_us"] + slope * (world - w1)
        gap = max(a0["mode1_us"] - a0["mode0_us"], a1["mode1_us"] - a1["mode0_us"])
        return rt, gap, f"extrapolated from the {w0}- and {w1}-rank measurements"

    proj = {}
    t1 = pieces["one_gpu_512"]["cg1"]["ms"]
    k_mean, other1 = args.k_mean, args.other_ms
    for world in worlds:
        sl = pieces.get(f"slab_{world}")
        got = rt_gap(world)
        if sl is None or got is None:
            continue
        rt_us, gap_us, src = got
        rt, gap = rt_us * 1e-3, max(0.0, gap_us) * 1e-3
        march = sl["march_P"]["ms"]
        tb = sl["textbook_P"]["ms"]
        sweep_b = sl["textbook_P"]["timers"].get("cg_sweep_b", tb / 2)
        cg1 = (march + pieces["edge2"]["ccf"]["ms"] + (pieces["edge2"]["cc2"]["ms"] or 0.0) + rt
               + 3 * gap + max(0.0, halo_ms - march))
        cg0 = (tb + (pieces["edge2"]["sweepB"]["ms"] or 0.0) + 2 * rt + 3 * gap
               + max(0.0, halo_ms - sweep_b))
        step1 = k_mean * t1 + other1
        proj[str(world)] = {"cg0": round(cg0, 4), "cg1": round(cg1, 4),
                            "speedup_vs_1gpu_k_ccf": {"cg0": round(t1 / cg0, 2),
                                                      "cg1": round(t1 / cg1, 2)},
                            # whole step: the timed trajectory's mean CG
                            # iterations and the non-CG kernels split N ways
                            "step_speedup": {v: round(step1 / (k_mean * t + other1 / world), 2)
                                             for v, t in (("cg0", cg0), ("cg1", cg1))},
                            "terms_ms": {"march_P": march, "textbook_P": tb,
                                         "edge2_ccf": pieces["edge2"]["ccf"]["ms"],
                                         "edge2_cc2": pieces["edge2"]["cc2"]["ms"],
                                         "edge2_sweepB": pieces["edge2"]["sweepB"]["ms"],
                                         "allreduce_rt": round(rt, 5), "launch_gap": round(gap, 5),
                                         "allreduce_source": src,
                                         "halo_est": round(halo_ms, 5)}}
    dev = ""
    try:
        import torch
        dev = torch.cuda.get_device_name(0)
    except Exception:  # noqa: BLE001
        pass
    out = {"tool": "tools/slab_budget.py", "grid": [N, N, N], "iters": args.iters,
           "measured_on": f"one GPU ({dev}), allreduce ranks sharing it",
           "assumptions": {"xgmi_GBps_per_direction": XGMI_GBPS, "rccl_send_recv_us": RCCL_US,
                           "k_mean": k_mean, "other_ms_per_step_1gpu": other1},
           "pieces": pieces, "projected_ms_per_iter": proj, "wall_s": round(time.time() - t0, 1)}
    line = json.dumps(out)
    print(line, flush=True)
    if args.out:
        Path(args.out).write_text(json.dumps(out, indent=1) + "\n")


if __name__ == "__main__":
    main()
