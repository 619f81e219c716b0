#!/usr/bin/env python3
"""Benchmark of the MI355X-native Chorin projection step (BASELINE.json metric:
"MLUPS + achieved HBM GB/s, 512^3 projection step, 1/2/4/8xMI355X").

Workload (BASELINE.json configs[2]): 512^3 lid-driven
cavity, Re = 1000 (nu = 1e-3), dt = 1e-4, projection_hip with the CPU
reference's CG settings (rel 1e-6, abs 1e-10). Fields are synthetic (the
cavity starts at rest), generated and kept resident in HBM; a "step" is one
full projection step (predictor, CG pressure solve to convergence,
corrector). value = interior cells updated per second over all ranks, in
MLUPS.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
For N > 1 launch with torch.distributed.run (one rank per GPU): the grid is
split into N Z-slabs (hip_proj_create_slab), halo planes and CG dot products
move over RCCL (a communicator our library creates from a unique id that
rank 0 broadcasts over a gloo group), and the total work is fixed, so the
scaling is strong.

--case tg: configs[3], Taylor-Green at --size^3 on N Z-slabs.
--case convection: configs[4], natural convection (Boussinesq energy
equation coupled) on a --size x --size x --nz grid (default 1024 x 1024 x
512), Red-Black SOR pressure solve, N Z-slabs over RCCL (the configuration
BASELINE.json names on 8 GPUs); the setup restates
tests/validation/test_natural_convection.c:140-293 (convection_setup). Its
line reports MLUPS, RB-SOR iterations per step, per-rank relaxation timers
(sweep / halo / all-reduce per iteration) and, at N = 1, a roofline on
k_rb1 (24 B/cell per iteration). --dump PREFIX writes every rank's owned
planes of u, v, w, p, T to PREFIX.rank<r>.npz (parity tests).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBPS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# Algorithmic HBM bytes per interior cell:
BYTES_SWEEP_A = 24.0    # read r, p_old; write p_new
BYTES_SWEEP_B = 24.0    # read p, r; write r
BYTES_SWEEP_AX = 64.0   # every 4th iteration, sweep A + read x, p_{it-4..it-2}; write x
                        # (the 4 pending alpha p folded; p_{it-1} is sweep A's p_old)
BYTES_CC_UPDATE = 66.0  # cg_variant 1, k_cc1: read r, w, p_old, s; write p, s, r (56) + x fold / 4
BYTES_CC_SPMV = 16.0    # cg_variant 1, k_cc2: read r (stencil); write w
BYTES_CC_SPMV_NOW = 8.0 # cg_variant 1 on Z-slabs, k_cc2 without the w store: read r (stencil)
BYTES_CC_FUSED = 40.0   # cg_variant 1, k_ccf: read r, p_old; write p, r (32)
                        # + the x fold's 32 B every 4th iteration (read x, p_{it-3},
                        # p_{it-2}; write x; p_{it-1} is the march's own p_old)
BYTES_CG_SMALL_ITER = 64.0    # small grids, k_cg_small per iteration (x updated every iteration)
BYTES_CG_ITER_SURVEY = 80.0   # SURVEY.md §8d textbook CG iteration (x, r, p, Ap)
BYTES_STEP_FIXED_SURVEY = 176.0  # SURVEY.md §8d per-step non-CG bytes


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--size", type=int, default=0,
                    help="grid points per axis (default 512; convection: 1024 x 1024 x 512)")
    ap.add_argument("--case", choices=("cavity", "tg", "convection"), default="cavity",
                    help="cavity: configs[2] (default, every N); tg: configs[3] Taylor-Green; "
                         "convection: configs[4] natural convection with RB-SOR")
    ap.add_argument("--nz", type=int, default=0,
                    help="convection: z points (default size / 2)")
    ap.add_argument("--relax-max-iter", type=int, default=20000,
                    help="convection: RB-SOR iteration cap per step (the 1024^2 x 512 solve "
                         "needs ~13 000; the reference's default 5000 would fail the step)")
    ap.add_argument("--relax-tol", type=float, default=1e-6,
                    help="convection: RB-SOR relative tolerance (the reference default 1e-6)")
    ap.add_argument("--allow-max-iter", action="store_true",
                    help="convection: a step whose RB-SOR solve hits the cap does not stop "
                         "the run (PMC profiling passes with a small cap only)")
    ap.add_argument("--dump", default="",
                    help="convection: write each rank's owned planes to DUMP.rank<r>.npz")
    ap.add_argument("--re", type=float, default=1000.0)
    ap.add_argument("--dt", type=float, default=1e-4)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-cg-iters", type=int, default=40,
                    help="CG iterations timed in each CPU baseline sample")
    ap.add_argument("--cpu-repeat", type=int, default=3,
                    help="CPU baseline samples per placement (the median is reported)")
    ap.add_argument("--cpu-scalar-cg-iters", type=int, default=5,
                    help="CG iterations in the 1-thread CPU sample (0: skip it)")
    ap.add_argument("--cpu-timeout", type=int, default=420,
                    help="seconds allowed for the CPU baseline child process")
    ap.add_argument("--kchunk", type=int, default=0)
    ap.add_argument("--sweep-rows", type=int, default=16)
    ap.add_argument("--sweep-variant", type=int,
                    default=int(os.environ.get("CFD_BENCH_SWEEP_VARIANT", "15")),
                    help="CG sweep variant: bit0 NT stores, bit1 NT loads, bit2 plane prefetch, "
                         "bit3 one edge load (built: 0-4, 7, 15, and 23 / 31 with 16 rows; "
                         "default 15, or CFD_BENCH_SWEEP_VARIANT)")
    ap.add_argument("--cg-variant", type=int, default=-1, choices=(-1, 0, 1),
                    help="0: textbook CG (the reference's loop); 1: single-reduction "
                         "(Chronopoulos-Gear) CG, one fused z-march per iteration; -1 "
                         "(default): 1 on one GPU at n >= 512, where it is measured faster "
                         "(DESIGN.md section 5); on N > 1 at 512^3 the committed budget's "
                         "pick, then the live probe (--cg-probe); else 0")
    ap.add_argument("--cg-probe", choices=("auto", "on", "off"), default="auto",
                    help="N > 1: step both CG forms from fresh contexts before the run and "
                         "keep the faster per CG iteration (auto: when --cg-variant is -1 "
                         "on the 512^3 cavity)")
    ap.add_argument("--cg-probe-steps", type=int, default=2,
                    help="timed steps per form in the probe (after one untimed step)")
    ap.add_argument("--fixed-cg-iters", type=int, default=200,
                    help="fixed-iteration CG microbench per variant after the timed region "
                         "(SURVEY.md §8d config 3; 0: skip)")
    ap.add_argument("--no-plugin-step", action="store_true",
                    help="skip the host-buffer plugin-step measurement after the timed region")
    ap.add_argument("--plugin-steps", type=int, default=3,
                    help="host-buffer plugin steps per mode (the first is not averaged)")
    ap.add_argument("--no-compare-cg-variant", action="store_true",
                    help="skip the side measurement of the other CG variant after the "
                         "timed region")
    return ap.parse_args()


def progress(msg):
    """A progress line on stderr (long runs: one every minute or so)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def dist_env():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return rank, world, local


def main():
    args = parse()
    rank, world, local = dist_env()
    if os.environ.get("CFD_BENCH_SHARED_GPU") == "1":
        # rehearsal of the N-rank path on a 1-GPU box: every rank on device 0,
        # each rank its own NCCL_HOSTID so RCCL accepts the shared device
        # (its socket transport then stands in for xGMI; timings meaningless)
        os.environ["NCCL_HOSTID"] = f"cfd-bench-rank{rank}"
        local = 0
    import torch  # noqa: F401  (imported first: one HIP runtime in the process)
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo")
    from cfd_amd import _abi as A
    from cfd_amd import _native, api

    lib = _native.hip()
    if lib.hip_projection_available() != 1:
        raise SystemExit("bench: no HIP device")
    torch.cuda.set_device(local)

    if args.size <= 0:
        args.size = 1024 if args.case == "convection" else 512
    n = args.size
    if args.case == "convection":
        comm = None
        if world > 1:
            uid = [api.comm_unique_id() if rank == 0 else None]
            dist.broadcast_object_list(uid, src=0)
            comm = api.SlabComm.rccl(uid[0], rank, world, local)
        run_convection(args, rank, world, local, comm, lib, torch, dist)
        if comm is not None:
            comm.close()
        if world > 1:
            dist.destroy_process_group()
        return
    tg = args.case == "tg"
    if tg:
        # configs[3]: Taylor-Green on [0, 2pi]^3, nu = 0.01, dt = 1e-3, periodic
        # BCs before every step (taylor_green_3d_reference.h:177-300)
        nu, dt, L = 0.01, 1e-3, 2.0 * math.pi
    else:
        nu, dt, L = 1.0 / args.re, args.dt, 1.0
    g = api.Grid(n, n, n, 0.0, L, 0.0, L, 0.0, L)
    params = api.validation_params(dt, nu)
    comm = None
    if world > 1:
        uid = [api.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        comm = api.SlabComm.rccl(uid[0], rank, world, local)
    def make_ctx(cg_variant):
        c = api.HipProjection(n, n, n, comm=comm, device=local, kchunk=args.kchunk,
                              sweep_rows=args.sweep_rows, sweep_variant=args.sweep_variant,
                              cg_variant=cg_variant)
        for fid in (A.HIP_FIELD_U, A.HIP_FIELD_V, A.HIP_FIELD_W, A.HIP_FIELD_P):
            c.fill(fid, 0.0)
        c.set_density(1.0)
        if tg:
            import numpy as np
            x = np.asarray(g.x)
            z = np.asarray(g.z)[c.k_offset:c.k_offset + c.nz_local]
            cz = np.cos(z)[:, None, None]
            c.set_field(A.HIP_FIELD_U, np.cos(x)[None, None, :] * np.sin(x)[None, :, None] * cz)
            c.set_field(A.HIP_FIELD_V, -np.sin(x)[None, None, :] * np.cos(x)[None, :, None] * cz)
        else:
            # caller BCs (lid_driven_cavity_common.h:142-148, 3-D form): u = 1 on
            # the lid; the step preserves boundary faces, so applying them once
            # is the same as before every step
            c.apply_dirichlet(A.HIP_FIELD_U, api.dirichlet(top=1.0))
            c.apply_dirichlet(A.HIP_FIELD_V, api.dirichlet())
            c.apply_dirichlet(A.HIP_FIELD_W, api.dirichlet())
            c.apply_scalar_bc(A.HIP_FIELD_P, A.BC_TYPE_NEUMANN)
        c.synchronize()
        return c

    ctx = None

    def step():
        if tg:  # periodic BCs on u, v, w, p before every step (collective on slabs)
            for fid in (A.HIP_FIELD_U, A.HIP_FIELD_V, A.HIP_FIELD_W, A.HIP_FIELD_P):
                ctx.apply_scalar_bc(fid, A.BC_TYPE_PERIODIC)
        s = ctx.step_device(g, params)
        if s != A.CFD_SUCCESS:
            raise RuntimeError(f"step failed {s}: {_native.last_error()}")
        return ctx.poisson_stats().iterations

    def timed_steps(nsteps):
        """(max-over-ranks seconds, CG iterations) of the next nsteps steps."""
        ctx.synchronize()
        if world > 1:
            dist.barrier()
        ta = time.perf_counter()
        its = sum(step() for _ in range(nsteps))
        ctx.synchronize()
        e = time.perf_counter() - ta
        if world > 1:
            tt = torch.tensor([e], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            e = float(tt[0])
        return e, its

    auto = args.cg_variant < 0
    if auto:
        args.cg_variant = cg_variant_auto(n, world, args.case)
    probe = None
    if cg_probe_wanted(args, n, world, auto):
        # N > 1: both CG forms step the trajectory's first steps on THIS node
        # (fresh contexts, the first step untimed), the faster per CG
        # iteration is the run's; every rank takes the same max-over-ranks
        # times, so every rank picks the same form
        progress("cg_variant probe")
        probe = {"steps": f"{1 + args.cg_probe_steps} per form from a fresh context, "
                          f"the first untimed (max over ranks)"}
        for v in (args.cg_variant, 1 - args.cg_variant):
            ctx = make_ctx(v)
            step()
            e, its = timed_steps(args.cg_probe_steps)
            ctx.close()
            ctx = None
            probe[f"cg{v}"] = {"cg_iters": its, "ms": round(e * 1e3, 3),
                               "ms_per_cg_iter": round(e * 1e3 / max(1, its), 5)}
        faster = 1 if probe["cg1"]["ms_per_cg_iter"] < probe["cg0"]["ms_per_cg_iter"] else 0
        probe["budget_pick"] = args.cg_variant
        probe["picked"] = faster
        args.cg_variant = faster
    solver_name = "projection_hip_cg1" if args.cg_variant == 1 else "projection_hip"
    ctx = make_ctx(args.cg_variant)
    # placement draws of the CG fields at creation (hip_proj_get_placement):
    # each draw's probe time per CG iteration and the one kept
    place_ms, place_pick = ctx.placement()

    for w in range(args.warmup):
        step()
        progress(f"warm-up step {w + 1}/{args.warmup}")
    ctx.synchronize()
    ctx.reset_timing()
    ctx.enable_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    iters, step_ms = [], []
    for k in range(args.steps):
        ts = time.perf_counter()
        iters.append(step())  # returns after the step's CG solve has drained
        step_ms.append((time.perf_counter() - ts) * 1e3)
        if k % 5 == 4:
            progress(f"timed step {k + 1}/{args.steps}")
    ctx.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    ctx.enable_timing(False)
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt[0])
    # effective shader clock of the march's own workgroups over the timed
    # region (sampled launches, hip_proj_get_clock_sample), so the line
    # says which clock its box ran at
    clk_mhz, clk_wg = ctx.clock_sample()

    n_int = (n - 2) ** 3
    n_loc = (n - 2) ** 2 * (ctx.nz_local - 2)  # interior cells of this rank's slab
    ms_step = elapsed / args.steps * 1e3
    # strong scaling: the ranks share one n^3 grid, so the job updates n_int
    # cells per step whatever the rank count
    mlups = n_int * args.steps / elapsed / 1e6
    k_mean = sum(iters) / len(iters)
    # SURVEY.md §8d credit: (176 + 80 k) B/cell per step for textbook CG. Ours
    # moves 58 B per CG iteration, so the credit divided by the wall time is
    # NOT a bandwidth (it can exceed the HBM peak); the line reports it as an
    # equivalent rate of the survey's byte model only, next to measured_GBps
    credited = (BYTES_STEP_FIXED_SURVEY + BYTES_CG_ITER_SURVEY * k_mean) * n_int
    credited_equiv = credited * args.steps / elapsed / 1e9

    kt = ctx.timing()
    # the march's plain (+ first) and x-fold launches time apart (ABI 3);
    # the roofline is on their sum, one launch per CG iteration
    kt_all = dict(kt)
    kt_all["cc_march"] = (kt["cc_fused"][0] + kt["cc_fold"][0], kt["cc_fused"][1] + kt["cc_fold"][1])
    sweeps = {}   # timer -> (kernel symbol, B/cell, avg ms, launches, achieved GB/s, total ms)
    sweep_set = sweep_kernels(args.sweep_rows, world > 1, args.sweep_variant, args.cg_variant,
                              ctx.nz_local - 2)
    for key, kname, bpc in sweep_set:
        ms, cnt = kt_all[key]
        avg = ms / cnt if cnt else None
        ach = bpc * n_loc / (avg * 1e-3) / 1e9 if cnt else None
        sweeps[key] = (kname, bpc, avg, cnt, ach, ms)
    small_ms, small_n = kt.get("cg_small", (0.0, 0))
    if small_n:
        # small grids: each solve is ONE persistent launch (k_cg_small) that
        # moves 64 B/cell per iteration (A: r, p_old -> p; B: p, r, x -> r, x)
        its_per_launch = sum(iters) / small_n
        bpc_small = BYTES_CG_SMALL_ITER * its_per_launch
        avg = small_ms / small_n
        sweeps["cg_small"] = ("k_cg_small", bpc_small, avg, small_n,
                              bpc_small * n_loc / (avg * 1e-3) / 1e9, small_ms)
    if small_n:  # one iteration = the solve's time / its iterations
        cg_iter_ms = small_ms / max(1, sum(iters))
    elif args.cg_variant == 1 and "cc_march" in sweeps:  # the march (+ the slab SpMV)
        cg_iter_ms = (sweeps["cc_march"][2] or 0.0) + (
            (sweeps["cc_spmv"][2] or 0.0) if "cc_spmv" in sweeps else 0.0)
    elif args.cg_variant == 1:  # one iteration = update + SpMV
        cg_iter_ms = (sweeps["cc_update"][2] or 0.0) + (sweeps["cc_spmv"][2] or 0.0)
    else:  # one CG iteration = the mean of the two sweep A forms + sweep B
        na = sweeps["cg_sweep_a"][3] + sweeps["cg_sweep_bx"][3]
        avg_a = (sweeps["cg_sweep_a"][5] + sweeps["cg_sweep_bx"][5]) / na if na else 0.0
        cg_iter_ms = avg_a + (sweeps["cg_sweep_b"][2] or 0.0)
    # roofline on the dominant sweep (largest total time)
    dom = max(sweeps, key=lambda k: sweeps[k][5] or 0.0)
    kname, bpc_dom, avg_dom, _, ach_dom, _ = sweeps[dom]
    # measured HBM bytes: the committed PMC profile of THESE kernel sources
    # (2*FETCH_SIZE + WRITE_SIZE per launch) x this run's launch counts
    prof = pmc_profile(n_loc)
    traffic = traffic_src = measured_gbps = None
    measured_from = []
    if prof is not None:
        bpl = (prof_record(prof, kname) or {}).get("hbm_bytes_per_launch")
        traffic = round(bpl) if bpl else None
        traffic_src = (prof["file"] + ": " + ("k_ccf<*, *, false> (launch-weighted)"
                                              if kname == "k_ccf<false, false, false>"
                                              else kname)) if bpl else None
        names = {k: v[0] for k, v in sweeps.items() if k != "cc_march"}
        tot = 0.0
        for key, (ms, cnt) in kt.items():
            if not cnt:
                continue
            kn = names.get(key) or TIMER_KERNEL.get(key)
            rec = prof_record(prof, kn, key) if kn else None
            if rec and "hbm_bytes_per_launch" in rec:
                tot += rec["hbm_bytes_per_launch"] * cnt
                measured_from.append(kn)
        measured_gbps = round(tot * world / elapsed / 1e9, 1) if measured_from else None

    # measured HBM roof of this GPU (same library, 16-B lanes), after the
    # timed region
    import ctypes as C
    cg, tr = C.c_double(0.0), C.c_double(0.0)
    if lib.cfd_hip_stream_bench(local, 1 << 27, 5, C.byref(cg), C.byref(tr)) != A.CFD_SUCCESS:
        cg.value = tr.value = 0.0

    ranks = None
    tot_iters = max(1, sum(iters))
    if world > 1:  # per-rank device times, so the driver's 1 -> N curve can be read
        per_it = lambda key: round(kt[key][0] / tot_iters, 4) if kt[key][1] else None
        mine = {"rank": rank, "planes": ctx.nz_local - 2,
                "sweep_ms_per_iter": round(cg_iter_ms, 4),
                "halo_ms_per_iter": per_it("halo"),
                # with the device mailbox the all-reduce runs inside the sweeps
                "allreduce_ms_per_iter": per_it("allreduce"),
                "dot_allreduce": "mailbox (in sweep)" if comm.device_allreduce else "ncclAllReduce",
                "timers_ms": {k: round(v[0], 3) for k, v in kt.items() if v[1]}}
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)

    # SURVEY.md §8d config 3's fixed-iteration CG microbench (one GPU): 200
    # iterations, no early exit, x0 = 0, on the last step's own RHS and on
    # the cos(pi x) cos(pi y) cos(pi z) RHS (interior mean removed), for the
    # CG variant of this context; the CG-iteration roofline without the
    # convergence tail or the step's other kernels
    progress("timed region done")
    fixed200 = {}
    cos_rhs = None
    if world == 1 and not tg and args.fixed_cg_iters > 0:
        import numpy as np
        xs = np.asarray(g.x)
        cx = np.cos(np.pi * xs)
        cos_rhs = (cx[:, None, None] * cx[None, :, None]) * cx[None, None, :]
        cos_rhs -= cos_rhs[1:-1, 1:-1, 1:-1].mean()
        fixed200[f"cg_variant_{args.cg_variant}"] = fixed_cg(ctx, g, params, n_int,
                                                             args.cg_variant, cos_rhs,
                                                             args.fixed_cg_iters)

    # side measurement of the other CG variant (same grid, ranks and stepping
    # from the same initial state), after the timed region: per CG iteration,
    # since its iteration counts differ from the main run's by rounding
    # The other variant times the SAME step as the main run's first timed
    # one: a fresh context steps the warm-up steps untimed, then step
    # warmup + 1 is timed (its CG iterations are that step's count), next to
    # the main run's own wall time of that step
    other = None
    if not args.no_compare_cg_variant:
        progress("cg_variant_compare")
        ctx.close()
        ctx = make_ctx(1 - args.cg_variant)
        for _ in range(args.warmup):
            step()
        ctx.synchronize()
        ctx.reset_timing()
        ctx.enable_timing(True)
        if world > 1:
            dist.barrier()
        ta = time.perf_counter()
        it2 = step()
        ctx.synchronize()
        tb = time.perf_counter()
        ctx.enable_timing(False)
        e2 = tb - ta
        if world > 1:
            tt = torch.tensor([e2], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            e2 = float(tt[0])
        k2 = ctx.timing()
        per2 = lambda key: round(k2[key][0] / max(1, it2), 4) if k2[key][1] else None
        other = {"cg_variant": 1 - args.cg_variant, "step": args.warmup + 1,
                 "timed": f"step {args.warmup + 1} of a fresh context after "
                          f"{args.warmup} untimed steps (the main run's first timed step)",
                 "cg_iters": it2, "ms_step": round(e2 * 1e3, 3),
                 "ms_per_cg_iter_wall": round(e2 * 1e3 / max(1, it2), 4),
                 "kernel_ms_per_iter": {k: per2(k) for k in k2 if k2[k][1]},
                 "main_same_step": {"cg_iters": iters[0], "ms_step": round(step_ms[0], 3),
                                    "ms_per_cg_iter_wall": round(step_ms[0] / max(1, iters[0]),
                                                                 4)},
                 "main_ms_per_cg_iter_wall_all_steps": round(elapsed * 1e3 / tot_iters, 4)}
        if cos_rhs is not None:
            fixed200[f"cg_variant_{1 - args.cg_variant}"] = fixed_cg(
                ctx, g, params, n_int, 1 - args.cg_variant, cos_rhs, args.fixed_cg_iters)
    del cos_rhs

    # the reference caller's throughput: projection_hip_cg1 through
    # solver_step on host buffers (solver_registry.c:438-458, as
    # run_simulation_step drives it, simulation_api.c:185-202), full
    # transfers and the resident dirty-faces mode, beside the HBM-resident
    # step on the same steps; never `value`
    plug = None
    if world == 1 and not tg and not args.no_plugin_step:
        progress("plugin_step")
        ctx.close()
        ctx = None
        plug = plugin_step(n, g, params, make_ctx, args.plugin_steps)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and not tg:
        progress("cpu_baseline")
        cpu = cpu_baseline(n, args, k_mean)

    if rank == 0:
        out = {
            "metric": "MLUPS + achieved HBM GB/s, 512^3 projection step, 1/2/4/8xMI355X",
            "value": round(mlups, 3),
            "unit": "MLUPS",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": ("synthetic (Taylor-Green IC generated on the host, uploaded once)" if tg
                     else "synthetic (cavity at rest + lid BC, generated in HBM)"),
            "config": {"workload": (f"{n}^3 Taylor-Green nu=0.01, dt=1e-3" if tg else
                                    f"{n}^3 lid-driven cavity Re={args.re:g}, dt={args.dt:g}")
                                   + f", {solver_name} (CG rel 1e-6"
                                   + (", single-reduction Chronopoulos-Gear CG)"
                                      if args.cg_variant == 1 else ", textbook CG)"),
                       # the registry name whose pressure solve this run times
                       # (projection_hip_plugin.c cfd_hip_register_solvers)
                       "solver": solver_name,
                       "grid": [n, n, n], "interior_cells": n_int,
                       "parallelism": (f"z-slab x{world} (RCCL halo, "
                                       + ("peer-memory" if comm.device_allreduce else "RCCL")
                                       + " dot all-reduce)") if world > 1 else "single GPU"},
            "measured_GBps": measured_gbps,
            "measured_GBps_kernels": measured_from or None,
            # the survey's textbook-CG byte model (80 B/cell per iteration) over
            # the wall time: a throughput in those units, not HBM traffic
            "survey80_equiv_rate": {"value": round(credited_equiv, 1),
                                    "unit": "GB-equivalent/s (SURVEY §8d 176+80k B/cell model)"},
            "cg_iters_per_step": iters,
            "cg_iter_ms": round(cg_iter_ms, 4),
            "roofline": {"bound": "hbm", "kernel": kname,
                         "achieved": round(ach_dom, 1) if ach_dom else None,
                         "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(ach_dom / HBM_PEAK_GBPS, 4) if ach_dom else None,
                         "traffic": traffic, "traffic_source": traffic_src,
                         "algorithmic_bytes": bpc_dom * n_loc,
                         "bytes_per_cell": bpc_dom,
                         "avg_launch_ms": round(avg_dom, 4) if avg_dom else None,
                         "stream_copy_GBps": round(cg.value, 1) or None,
                         "stream_triad_GBps": round(tr.value, 1) or None,
                         "frac_of_stream_copy": (round(ach_dom / cg.value, 4)
                                                 if ach_dom and cg.value else None)},
            "kernels": {k: {"total_ms": round(v[0], 3), "launches": v[1],
                            "avg_ms": round(v[0] / v[1], 4) if v[1] else None}
                        for k, v in kt.items() if v[1]},
            "cg_sweeps": {k: {"kernel": v[0], "bytes_per_cell": v[1],
                              "avg_ms": round(v[2], 4) if v[2] else None,
                              "achieved_GBps": round(v[4], 1) if v[4] else None}
                          for k, v in sweeps.items()},
            "ranks": ranks,
            "ccf_launches": ccf_split(kt, n_loc, world) if args.cg_variant == 1 else None,
            "clock": {"k_ccf_shader_MHz": round(clk_mhz, 1) if clk_wg else None,
                      "sampled_workgroups": clk_wg,
                      "how": ("wave 0 of every workgroup of 2 in 8 k_ccf launches stamps "
                              "s_memtime / s_memrealtime at its start and end; MHz = 100 x "
                              "sum d memtime / sum d memrealtime (rank 0)")},
            "box": box_id(torch, local),
            "placement": {"probe_ms_per_iter": place_ms, "picked": place_pick,
                          "how": ("the CG fields allocated 6 times at context creation, 40 "
                                  "assignments of those buffers to the 7 roles each timed on "
                                  "a 16-iteration probe solve, the fastest kept "
                                  "(projection_hip.hip placement_draws)")},
            "step_ms": [round(v, 2) for v in step_ms],
            "cg_variant": args.cg_variant,
            "cg_variant_choice": cg_variant_choice(world, args, probe),
            "cg_variant_compare": other,
            "plugin_step": plug,
            "cg_fixed200": ({"iterations": args.fixed_cg_iters, "x0": "zero",
                             "early_exit": False, **fixed200} if fixed200 else None),
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    if ctx is not None:
        ctx.close()
    if comm is not None:
        comm.close()
    if world > 1:
        dist.destroy_process_group()


# natural convection (test_natural_convection.c:50-61 constants)
CONV_RA, CONV_PR, CONV_BETA, CONV_G = 1e3, 0.71, 0.003333, 9.81
CONV_T_HOT, CONV_T_COLD, CONV_T_REF = 310.0, 290.0, 300.0
BYTES_RB_ITER = 24.0  # k_rb1: read X, rhs; write Y
BYTES_RB2_SWEEP = 24.0  # k_rb2: read X, rhs; write Y2 -- two iterations (12 B/cell each)


def convection_setup(nx, ny, nz):
    """configs[4]: the de Vahl Davis cavity of test_natural_convection.c:140-293
    in 3-D on [0,1] x [0,1] x [0,0.5]: alpha, nu from Ra and Pr (:145-147), dt
    half the thermal limit dx^2 / (2 alpha 3) (:150-154), hot x = 0 and cold
    x = 1 Dirichlet walls, Neumann elsewhere, no-slip walls, fluid at rest
    with T linear in x. Returns (grid, params, T0) with T0(x) the initial T
    of every node of an x column."""
    from cfd_amd import _abi as A
    from cfd_amd import api
    import numpy as np

    dT = CONV_T_HOT - CONV_T_COLD
    nu_alpha = CONV_G * CONV_BETA * dT / CONV_RA
    alpha = math.sqrt(nu_alpha / CONV_PR)
    nu = CONV_PR * alpha
    g = api.Grid(nx, ny, nz, 0.0, 1.0, 0.0, 1.0, 0.0, 0.5)
    dx = 1.0 / (nx - 1)
    p = api.params_default()
    p.dt = 0.5 * dx * dx / (2.0 * alpha * 3.0)
    p.mu, p.alpha, p.beta, p.T_ref = nu, alpha, CONV_BETA, CONV_T_REF
    p.gravity[0], p.gravity[1], p.gravity[2] = 0.0, -CONV_G, 0.0
    p.source_amplitude_u = p.source_amplitude_v = 0.0
    tb = p.thermal_bc
    tb.left = tb.right = A.BC_TYPE_DIRICHLET
    tb.top = tb.bottom = tb.front = tb.back = A.BC_TYPE_NEUMANN
    tb.dirichlet_values.left, tb.dirichlet_values.right = CONV_T_HOT, CONV_T_COLD
    T0 = CONV_T_HOT - dT * np.asarray(g.x)
    return g, p, T0


def run_convection(args, rank, world, local, comm, lib, torch, dist):
    """configs[4] on N Z-slabs: projection_hip with the one-pass RB-SOR
    pressure solve and the energy equation, fields resident in HBM."""
    import numpy as np

    from cfd_amd import _abi as A
    from cfd_amd import _native, api

    nx = ny = args.size
    nz = args.nz or args.size // 2
    g, p, T0 = convection_setup(nx, ny, nz)
    ctx = api.HipProjection(nx, ny, nz, comm=comm, device=local,
                            poisson_method=A.HIP_POISSON_REDBLACK,
                            poisson_max_iter=args.relax_max_iter,
                            poisson_tolerance=args.relax_tol, relax_two_pass=0)
    for fid in (A.HIP_FIELD_U, A.HIP_FIELD_V, A.HIP_FIELD_W, A.HIP_FIELD_P):
        ctx.fill(fid, 0.0)
    ctx.set_field(A.HIP_FIELD_T, np.broadcast_to(T0[None, None, :], ctx.shape))
    ctx.set_density(1.0)
    for fid in (A.HIP_FIELD_U, A.HIP_FIELD_V, A.HIP_FIELD_W):
        ctx.apply_dirichlet(fid, api.dirichlet())
    ctx.synchronize()

    def step():
        s = ctx.step_device(g, p)
        if s != A.CFD_SUCCESS and not (args.allow_max_iter and s == A.CFD_ERROR_MAX_ITER):
            raise RuntimeError(f"convection step failed {s}: {_native.last_error()}")
        return ctx.poisson_stats().iterations

    for _ in range(args.warmup):
        step()
    ctx.synchronize()
    ctx.reset_timing()
    ctx.enable_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    iters = [step() for _ in range(args.steps)]
    ctx.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    ctx.enable_timing(False)
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt[0])
    kt = ctx.timing()
    n_int = (nx - 2) * (ny - 2) * (nz - 2)
    n_loc = (nx - 2) * (ny - 2) * (ctx.nz_local - 2)
    tot_it = max(1, sum(iters))
    per_it = lambda key: round(kt[key][0] / tot_it, 4) if kt[key][1] else None
    mine = {"rank": rank, "planes": ctx.nz_local - 2,
            "relax_sweep_ms_per_iter": round((kt["relax"][0] + kt["relax2"][0]) / tot_it, 4),
            "relax_halo_ms_per_iter": per_it("halo"),
            "relax_allreduce_ms_per_iter": per_it("allreduce"),
            "timers_ms": {k: round(v[0], 3) for k, v in kt.items() if v[1]}}
    ranks = [mine]
    if world > 1:
        ranks = [None] * world
        dist.all_gather_object(ranks, mine)
    if args.dump:
        loc, glob = ctx.owned()
        out = {k: ctx.get_field(fid)[loc] for k, fid in
               (("u", A.HIP_FIELD_U), ("v", A.HIP_FIELD_V), ("w", A.HIP_FIELD_W),
                ("p", A.HIP_FIELD_P), ("T", A.HIP_FIELD_T))}
        np.savez(f"{args.dump}.rank{rank}.npz", k0=glob.start, k1=glob.stop,
                 iters=np.array(iters), **out)
    roof = None
    rms, rn = kt["relax"]
    r2ms, r2n = kt["relax2"]
    if world == 1 and (rn or r2n):
        # measured HBM bytes per sweep: the committed PMC profile of these
        # kernel sources at this grid (2*FETCH_SIZE + WRITE_SIZE)
        prof = pmc_profile(n_loc)
        def traffic_of(prefixes):
            if prof is None:
                return None, None
            recs = [(k, v) for k, v in prof["kernels"].items()
                    if k.startswith(prefixes) and "hbm_bytes_per_launch" in v]
            if not recs:
                return None, None
            return (round(sum(v["hbm_bytes_per_launch"] for _, v in recs) / len(recs)),
                    prof["file"] + ": " + ", ".join(k for k, _ in recs))
        if r2n:
            # two RB-SOR iterations per sweep (k_rb2, rb2.hpp): 24 B/cell per
            # sweep = 12 B/cell per iteration. Working sweeps per step of n
            # iterations: sweep 0 is one k_rb1 sweep (it also gives the exact
            # initial residual), then k_rb2 on iterates 1, 3, ... <= n, i.e.
            # (n + 1) // 2; the launches queued after the decision return at
            # once and add ~4 us each to the kernel total
            sweeps = sum(max(1, (i + 1) // 2) for i in iters)
            avg = r2ms / max(1, sweeps)
            ach = BYTES_RB2_SWEEP * n_loc / (avg * 1e-3) / 1e9
            traffic, traffic_src = traffic_of(("k_rb2<",))
            roof = {"bound": "hbm", "kernel": "k_rb2 (two RB-SOR iterations per sweep)",
                    "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": traffic,
                    "traffic_source": traffic_src,
                    "algorithmic_bytes": BYTES_RB2_SWEEP * n_loc,
                    "bytes_per_cell": BYTES_RB2_SWEEP, "iterations_per_sweep": 2,
                    # what bounds it (r06, after the VALU trim): the bytes it
                    # moves, 31.7 fetched + 8.1 written B/cell per sweep at the
                    # box's copy rate, half the reads the tile's halo; the
                    # on-chip part alone runs 1.17 ms per iteration
                    # (profiles/r06ah_rb2_xmap_kc.jsonl, the diagnostic build)
                    "limiter": ("HBM bytes of the tile halo (no-memory build 1.17 vs 1.66 ms per "
                                "iteration, DESIGN.md §3 r06)"),
                    "avg_sweep_ms": round(avg, 4), "sweeps": sweeps, "launches": r2n,
                    "one_iteration_sweeps": rn}
        else:
            # one sweep per RB-SOR iteration on one device, plus the sweep whose
            # residual shows convergence (sweeps 0..n of an n-iteration solve;
            # the launches queued after it return at once and are not counted).
            # A sweep is ONE launch: k_rb1m runs the full-width TC-64 tiles and
            # the narrow strip of the columns past them in one grid
            # (kernels.hpp k_rb1m), or k_rb1 alone when 124 divides the columns.
            sweeps = sum(iters) + len(iters)
            avg = rms / sweeps
            ach = BYTES_RB_ITER * n_loc / (avg * 1e-3) / 1e9
            traffic, traffic_src = traffic_of(("k_rb1<", "k_rb1m<"))
            roof = {"bound": "hbm", "kernel": "k_rb1m (one RB-SOR sweep per launch: TC-64 tiles "
                                              "+ the narrow TC-16 strip in one grid)",
                    "achieved": round(ach, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(ach / HBM_PEAK_GBPS, 4), "traffic": traffic,
                    "traffic_source": traffic_src,
                    "algorithmic_bytes": BYTES_RB_ITER * n_loc, "bytes_per_cell": BYTES_RB_ITER,
                    "avg_sweep_ms": round(avg, 4), "sweeps": sweeps, "launches": rn}
    ctx.close()
    if rank == 0:
        print(json.dumps({
            "metric": "MLUPS + achieved HBM GB/s, natural convection step (configs[4])",
            "value": round(n_int * args.steps / elapsed / 1e6, 3),
            "unit": "MLUPS", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f64",
            "data": "synthetic (fluid at rest, T linear in x, generated in HBM)",
            "config": {"workload": f"{nx}x{ny}x{nz} natural convection Ra=1e3, Pr=0.71, "
                                   "projection_hip with the RB-SOR pressure solve (two "
                                   "iterations per sweep on one GPU)",
                       "grid": [nx, ny, nz], "interior_cells": n_int,
                       "relax_max_iter": args.relax_max_iter, "relax_tol": args.relax_tol,
                       "relax_max_iter_note": ("the reference's default cap is 5000 "
                                               "(linear_solver.c:37-47); the 1024^2 x 512 "
                                               "solve needs ~13 000 iterations, so the "
                                               "reference would fail this step at its "
                                               "default: the cap is raised for both"),
                       "parallelism": f"z-slab x{world} (RCCL halo)" if world > 1
                                      else "single GPU"},
            "rbsor_iters_per_step": iters,
            "rbsor_iter_ms": round(elapsed * 1e3 / tot_it, 4),
            "roofline": roof, "ranks": ranks, "cpu_baseline": None}))


# timer -> kernel symbol in the PMC profile (the CG sweeps are named per variant)
# (predictor / corrector: k_pred3 / k_corr3 by default, k_pred2 / k_corr2 with
# CFD_HIP_PC3=0; FL 0 is the product variant)
_PC_OLD = os.environ.get("CFD_HIP_PC3", "1") == "0"
TIMER_KERNEL = {"predictor": "k_pred2<false, 0>" if _PC_OLD else "k_pred3<false, 0>",
                "corrector": "k_corr2<0>" if _PC_OLD else "k_corr3<0>",
                "cg_setup": "k_cg_setup<true, false, true, false>",
                # one device: the march's plain (+ first) and fold launches
                "cc_fused": "k_ccf<false, false, false>",
                "cc_fold": "k_ccf<false, false, false>"}


def sweep_kernels(rows, dist_, variant, cg_variant, planes=None):
    """(timer, kernel symbol as rocprofv3 prints it, algorithmic B/cell) of the
    CG sweeps a run launches; the symbols key the committed PMC profile."""
    d = "true" if dist_ else "false"
    # sweep B marches z downwards on one device (CFD_HIP_CGB_REV=0: upwards)
    rev = "true" if (not dist_ and os.environ.get("CFD_HIP_CGB_REV", "1") != "0") else "false"
    if cg_variant == 1 and not dist_:
        # one z-march per iteration (ccf.hpp); the timer spans the plain and
        # the fold launches, so the byte count is their mean
        return (("cc_march", "k_ccf<false, false, false>", BYTES_CC_FUSED),)
    if cg_variant == 1:
        # Z-slabs, fused form (r05): the edge planes' march (k_ccf<.., true>,
        # untimed, 2 planes), the r halo, the interior march with w and the
        # dots (the timer), then w = A r in registers on the two edge planes
        # completing the one reduction (k_cc2 without the w store): its bytes
        # per slab cell are 8 B x 2 / planes
        return (("cc_march", "k_ccf<false, false, false>", BYTES_CC_FUSED),
                ("cc_spmv", f"k_cc2<{rows}, {d}, false, false>",
                 BYTES_CC_SPMV_NOW * 2.0 / planes if planes else BYTES_CC_SPMV_NOW))
    return (("cg_sweep_a", f"k_cgA<{rows}, false, {d}, {variant}, false>", BYTES_SWEEP_A),
            ("cg_sweep_b", f"k_cgB<{rows}, {d}, {variant}, {rev}>", BYTES_SWEEP_B),
            ("cg_sweep_bx", f"k_cgA<{rows}, false, {d}, {variant & ~4}, true>", BYTES_SWEEP_AX))


BYTES_CG_TEXTBOOK = 58.0  # textbook CG per iteration: sweeps A + B (48) + the x fold / 4 (10)
BYTES_CCF_PLAIN = 32.0    # k_ccf plain launch: read r_it, p_{it-1}; write p_it, r_{it+1}
BYTES_CCF_FOLD = 64.0     # k_ccf fold launch: + read x, p_{it-3}, p_{it-2}; write x


def ccf_split(kt, n_loc, world):
    """The march's plain (+ first) and x-fold launches apart: average launch
    time, count and algorithmic rate on their own bytes (32 / 64 B/cell). On
    Z-slabs the timers hold the interior launch only."""
    out = {}
    for key, bpc in (("cc_fused", BYTES_CCF_PLAIN), ("cc_fold", BYTES_CCF_FOLD)):
        ms, cnt = kt[key]
        if not cnt:
            out[key] = None
            continue
        avg = ms / cnt
        gbps = bpc * n_loc / (avg * 1e-3) / 1e9
        out[key] = {"launches": cnt, "avg_ms": round(avg, 4), "bytes_per_cell": bpc,
                    "achieved_GBps": round(gbps, 1),
                    "frac_of_8TBps": round(gbps / HBM_PEAK_GBPS, 4)}
    out["note"] = ("cc_fused: the first and plain launches (32 B/cell; the first reads no "
                   "p_{it-1}), cc_fold: every 4th, which also folds x" +
                   ("; Z-slabs: the interior launch" if world > 1 else ""))
    return out


def plugin_step(n, g, params, make_ctx, nsteps):
    """projection_hip_cg1 through the reference interface on host buffers:
    Registry().create + solver_init + solver_step on a flow_field, from rest
    (the cavity BCs once, as the fixture's run), `nsteps` steps with full
    transfers (u, v, w, p up and down every step) and with the resident
    dirty-faces mode (CFD_HIP_DIRTY_FACES: only the boundary shell moves),
    beside the HBM-resident step_device of the same steps. Steps 2.. are
    averaged (step 1 of the resident mode uploads in full). pcie_share =
    1 - resident / host-buffer time of the same steps."""
    import ctypes as C

    from cfd_amd import _abi as A
    from cfd_amd import _native, api

    lib = _native.hip()
    out = {"solver": "projection_hip_cg1", "steps": nsteps, "averaged_steps": f"2..{nsteps}"}
    f = api.FlowField(n, n, n)
    reg = api.Registry()

    def reset_field():
        for k in ("u", "v", "w", "p", "T"):
            getattr(f, k)[...] = 0.0
        f.rho[...] = 1.0
        api.cavity_bc(f, 1.0)

    saved = os.environ.get("CFD_HIP_DIRTY_FACES")
    try:
        for mode, env in (("full", None), ("dirty_faces", "1000")):
            if env is None:
                os.environ.pop("CFD_HIP_DIRTY_FACES", None)
            else:
                os.environ["CFD_HIP_DIRTY_FACES"] = env
            reset_field()
            solver = reg.create("projection_hip_cg1")
            try:
                if solver.init(g, params) != A.CFD_SUCCESS:
                    raise RuntimeError("plugin init: " + _native.last_error())
                hctx = C.cast(solver._ptr.contents.context, C.POINTER(C.c_void_p))[0]
                ms, its = [], []
                for _ in range(nsteps):
                    st = A.SolverStats()
                    t0 = time.perf_counter()
                    s = solver.step(f, g, params, st)
                    ms.append((time.perf_counter() - t0) * 1e3)
                    if s != A.CFD_SUCCESS:
                        raise RuntimeError(f"plugin step {s}: {_native.last_error()}")
                    ps = A.PoissonStats()
                    lib.hip_proj_get_poisson_stats(hctx, C.byref(ps))
                    its.append(ps.iterations)
            finally:
                solver.close()
            out[mode] = {"ms_per_step": [round(v, 2) for v in ms], "cg_iters": its}
    finally:
        if saved is None:
            os.environ.pop("CFD_HIP_DIRTY_FACES", None)
        else:
            os.environ["CFD_HIP_DIRTY_FACES"] = saved
    del f
    c = make_ctx(1)
    try:
        ms, its = [], []
        for _ in range(nsteps):
            t0 = time.perf_counter()
            if c.step_device(g, params) != A.CFD_SUCCESS:
                raise RuntimeError("resident step: " + _native.last_error())
            its.append(c.poisson_stats().iterations)
            c.synchronize()
            ms.append((time.perf_counter() - t0) * 1e3)
    finally:
        c.close()
    out["resident"] = {"ms_per_step": [round(v, 2) for v in ms], "cg_iters": its}
    mean = lambda v: sum(v[1:]) / max(1, len(v) - 1)
    res = mean(out["resident"]["ms_per_step"])
    cells = (n - 2) ** 3
    for mode in ("full", "dirty_faces", "resident"):
        m = mean(out[mode]["ms_per_step"])
        out[mode]["ms_mean"] = round(m, 2)
        out[mode]["MLUPS"] = round(cells / (m * 1e-3) / 1e6, 2)
    out["ms_full"] = out["full"]["ms_mean"]
    out["ms_dirty_faces"] = out["dirty_faces"]["ms_mean"]
    out["ms_resident"] = round(res, 2)
    out["pcie_share"] = {"full": round(1.0 - res / out["ms_full"], 4),
                         "dirty_faces": round(1.0 - res / out["ms_dirty_faces"], 4)}
    return out


def fixed_cg(ctx, g, params, n_int, cg_variant, cos_rhs, iters):
    """ms per iteration of `iters` CG iterations (no early exit, x0 = 0) on the
    context's last step's RHS and on cos_rhs, with the algorithmic rate in
    both byte models (40 B/cell: the single-reduction march; 58: textbook)."""
    rho_over_dt = 1.0 / params.dt  # rho = 1 (the cavity)
    out = {"bytes_per_cell_moved": BYTES_CC_FUSED if cg_variant == 1 else BYTES_CG_TEXTBOOK}
    for name, rhs in (("step_rhs", None), ("cos_rhs", cos_rhs)):
        if rhs is None:
            ms = ctx.cg_fixed_iters_step_rhs(g.dx, g.dy, g.dz, iters, rho_over_dt)
        else:
            ms = ctx.cg_fixed_iters(rhs, g.dx, g.dy, g.dz, iters)
        if ms <= 0:
            out[name] = None
            continue
        per = ms / iters
        out[name] = {"ms_per_iter": round(per, 4),
                     "GBps_40": round(BYTES_CC_FUSED * n_int / (per * 1e-3) / 1e9, 1),
                     # r04's count for the march (before the fold read p_{it-1}
                     # from its own registers), the key the r04 review named
                     "GBps_42": round(42.0 * n_int / (per * 1e-3) / 1e9, 1),
                     "GBps_58": round(BYTES_CG_TEXTBOOK * n_int / (per * 1e-3) / 1e9, 1),
                     "frac_of_8TBps_own_bytes": round(out["bytes_per_cell_moved"] * n_int
                                                      / (per * 1e-3) / 1e9 / HBM_PEAK_GBPS, 4)}
    return out


def box_id(torch, device):
    """Which box and card ran the line (host name, device name and UUID), so
    lines from different boxes can be told apart when their rates differ."""
    import socket
    out = {"host": socket.gethostname()}
    try:
        pr = torch.cuda.get_device_properties(device)
        out["device"] = pr.name
        uuid = getattr(pr, "uuid", None)
        out["uuid"] = str(uuid) if uuid is not None else None
    except Exception as e:  # noqa: BLE001
        out["error"] = str(e)[:200]
    return out


def slab_budget():
    """The committed N-rank per-iteration budget (written by
    tools/slab_budget.py from one-GPU timings of each piece of a slab
    iteration): the file profiles/slab_budget_current.json names, else the
    newest profiles/*_slab_budget.json by name; None without one."""
    cur = ROOT / "profiles" / "slab_budget_current.json"
    paths = []
    try:
        paths.append(ROOT / "profiles" / json.loads(cur.read_text())["file"])
    except (OSError, ValueError, KeyError, TypeError):
        pass
    paths += sorted((ROOT / "profiles").glob("*_slab_budget.json"), reverse=True)
    for path in paths:
        try:
            d = json.loads(path.read_text())
        except (OSError, ValueError):
            continue
        if isinstance(d.get("projected_ms_per_iter"), dict):
            d["file"] = path.name
            return d
    return None


def cg_variant_auto(n, world, case="cavity"):
    """The bench's CG variant for the cavity:
    - one GPU at n >= 512: the single-reduction march k_ccf (1.05-1.17 vs
      1.31-1.35 ms per iteration at 512^3 on the same box, DESIGN.md
      section 3);
    - Z-slabs (N > 1): the variant whose projected per-iteration time at this
      N is lower in the committed slab budget (tools/slab_budget.py: every
      piece of one rank's iteration -- edge launch, interior march, edge
      SpMV, plane exchange, the dot all-reduces -- timed on one GPU at that
      N's slab shape); with no budget for this N,
      textbook CG, the reference's loop.
    The Taylor-Green case keeps the textbook CG its parity tests pin."""
    if case != "cavity":
        return 0
    if world == 1:
        return 1 if n >= 512 else 0
    b = slab_budget()
    proj = (b or {}).get("projected_ms_per_iter", {}).get(str(world)) if n == 512 else None
    if not proj or "cg0" not in proj or "cg1" not in proj:
        return 0
    return 1 if proj["cg1"] < proj["cg0"] else 0


def cg_probe_wanted(args, n, world, auto):
    """The live probe of both CG forms (N > 1): by default where the variant
    is the bench's own choice on the cavity at the metric's 512^3 (the
    committed budget is a one-GPU projection; the node running the line
    settles it); --cg-probe on / off forces it either way."""
    if args.cg_probe == "off" or args.case != "cavity" or world == 1:
        return False
    return args.cg_probe == "on" or (auto and n == 512)


def cg_variant_choice(world, args, probe=None):
    """Why this run's CG variant was chosen (the bench line's record)."""
    if args.case != "cavity":
        return {"rule": "Taylor-Green: textbook CG"}
    if world == 1:
        return {"rule": "one GPU at n >= 512: single-reduction march (k_ccf)"}
    b = slab_budget()
    proj = (b or {}).get("projected_ms_per_iter", {}).get(str(world))
    out = {"rule": "N > 1: the lower projected per-iteration time of the committed slab "
                   "budget at this N (textbook CG without one)",
           "budget_file": b["file"] if b else None, "projected_ms_per_iter": proj,
           "measured_on": (b or {}).get("measured_on")}
    if probe is not None:
        out["rule"] = ("N > 1: the form with the lower wall time per CG iteration in the live "
                       "probe on this node (the committed budget's pick beside it)")
        out["probe"] = probe
    return out


def prof_record(prof, kname, key=None):
    """PMC record of a timer's kernel. The one-device single-reduction march
    spans k_ccf's first, plain and fold launches (k_ccf<*, *, false>): their
    bytes per launch averaged over the profiled launch counts; with the timer
    key, "cc_fused" averages the first and plain launches and "cc_fold" is
    the fold launch's record."""
    if kname == "k_ccf<false, false, false>":
        want = {"cc_fused": ("k_ccf<true, false, false>", "k_ccf<false, false, false>"),
                "cc_fold": ("k_ccf<false, true, false>",)}.get(key)
        recs = [v for k, v in prof["kernels"].items()
                if k.startswith("k_ccf<") and k.endswith(", false>")
                and (want is None or k in want)
                and "hbm_bytes_per_launch" in v and v.get("calls")]
        n = sum(v["calls"] for v in recs)
        if n:
            return {"hbm_bytes_per_launch":
                    sum(v["hbm_bytes_per_launch"] * v["calls"] for v in recs) / n}
    return prof["kernels"].get(kname)


def pmc_profile(cells):
    """The newest committed PMC profile (profiles/*_traffic*.json, written by
    tools/prof_summary.py) taken on this grid with the kernels this run loads
    -- the same HIP sources, or the same device code in the library
    (cfd_amd._sha.device_code_sha: host-only edits keep it) -- or None: a
    profile of other kernel code is never used."""
    from cfd_amd._native import HIP_LIB, kernel_source_sha
    from cfd_amd._sha import device_code_sha

    sha = kernel_source_sha()
    dev = device_code_sha(HIP_LIB)
    for path in sorted((ROOT / "profiles").glob("*traffic*.json"), reverse=True):
        try:
            d = json.loads(path.read_text())
        except (OSError, ValueError):
            continue
        same = d.get("source_sha") == sha or (dev is not None and d.get("device_sha") == dev)
        if same and d.get("cells_per_launch") == float(cells):
            d["file"] = path.name
            return d
    return None


def cpu_baseline(n, args, k_gpu):
    """The oracle (OpenMP port of the reference projection) timed on this host
    on a bounded sample of the same step, in child processes that hold no HIP
    runtime (oracle/cpu_baseline.py). Threads: every CPU of this process's
    affinity mask, but no more than an OMP_NUM_THREADS the box sets (the GPU
    pool gives each 1-GPU box a 16-CPU share of a 256-CPU host and sets it to
    16; the mask still shows all 256). Two placements, since the host is
    shared with other boxes: OMP_PROC_BIND=close OMP_PLACES=cores (threads on
    the first cores of the mask) and unbound (the OS picks idle CPUs); the
    faster median is the reported value, both are recorded with the min and
    max of their `cpu_repeat` samples."""
    import subprocess

    affinity = len(os.sched_getaffinity(0))
    env_threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    threads = min(affinity, env_threads) if env_threads > 0 else affinity
    runs = {}
    for name, bind in (("bound", {"OMP_PROC_BIND": "close", "OMP_PLACES": "cores"}),
                       ("unbound", {"OMP_PROC_BIND": "false"})):
        progress(f"cpu_baseline placement {name}")
        env = dict(os.environ, OMP_NUM_THREADS=str(threads), CFD_AMD_NO_TORCH="1", **bind)
        if name == "unbound":
            env.pop("OMP_PLACES", None)
        cmd = [sys.executable, "-m", "oracle.cpu_baseline", "--size", str(n), "--dt",
               str(args.dt), "--re", str(args.re), "--k-gpu", str(k_gpu), "--cg-iters",
               str(args.cpu_cg_iters), "--repeat", str(args.cpu_repeat),
               "--scalar-cg-iters", str(args.cpu_scalar_cg_iters if name == "bound" else 0)]
        try:
            r = subprocess.run(cmd, cwd=str(ROOT), env=env, capture_output=True, text=True,
                               timeout=args.cpu_timeout)
        except subprocess.TimeoutExpired:
            runs[name] = {"error": f"timeout {args.cpu_timeout} s"}
            continue
        if r.returncode != 0:
            runs[name] = {"error": f"exit {r.returncode}: {r.stderr.strip()[-400:]}"}
            continue
        runs[name] = json.loads(r.stdout.strip().splitlines()[-1])
    ok = {k: v for k, v in runs.items() if "value" in v}
    if not ok:
        return {"error": "cpu baseline failed", "runs": runs}
    best = max(ok, key=lambda k: ok[k]["value"])
    out = dict(ok[best])
    out["placement"] = best
    out["placements"] = {k: {"value": v.get("value"), "min": v.get("min"), "max": v.get("max"),
                             "runs": v.get("runs"), "cg_iter_ms": v.get("cg_iter_ms"),
                             "error": v.get("error")} for k, v in runs.items()}
    if "scalar_1core" not in out and "bound" in ok:
        out["scalar_1core"] = ok["bound"].get("scalar_1core")
    out["omp_num_threads_env"] = env_threads or None
    out["cores_note"] = (f"{threads} threads: the box's CPU share (OMP_NUM_THREADS={env_threads}) "
                         f"of an affinity mask of {affinity} CPUs on a shared host")
    return out


if __name__ == "__main__":
    main()
