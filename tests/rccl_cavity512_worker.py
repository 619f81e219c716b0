"""Worker for test_gpu_cavity512.py::test_cavity512_rccl_vs_oracle: steps
1..$CFD_CAV512_STEPS of the bench's 512^3 cavity trajectory on N RCCL Z-slab
ranks (one process per rank, launched by torch.distributed.run; on a one-GPU
box every rank gets its own NCCL_HOSTID so RCCL accepts the shared device).
Rank 0 writes the per-step CG statistics, the interior L2 / max |.| of u, v,
w, p (combined from the ranks' partial sums) and, per step, how the CG dots
were reduced (the timers: no ncclAllReduce span when the device mailbox
carries them; the march launches per iteration) to $CFD_CAV512_OUT, and the
planes k = 1, 255, 510 after the steps in $CFD_CAV512_PLANE_STEPS (gathered
from their owners) next to it."""
import json
import os
import sys

RANK = int(os.environ.get("RANK", "0"))
WORLD = int(os.environ.get("WORLD_SIZE", "1"))
os.environ["NCCL_HOSTID"] = f"cfd-cav512-rank{RANK}"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import torch.distributed as dist  # noqa: E402

from cfd_amd import _abi as A  # noqa: E402
from cfd_amd import api  # noqa: E402

N, STEPS = 512, int(os.environ.get("CFD_CAV512_STEPS", "2"))
FIDS = {"u": A.HIP_FIELD_U, "v": A.HIP_FIELD_V, "w": A.HIP_FIELD_W, "p": A.HIP_FIELD_P}


def main():
    dist.init_process_group("gloo")
    uid = [api.comm_unique_id() if RANK == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    comm = api.SlabComm.rccl(uid[0], RANK, WORLD, 0)
    g = api.Grid(N, N, N, 0.0, 1.0, 0.0, 1.0, 0.0, 1.0)
    params = api.validation_params(1e-4, 1e-3)
    ctx = api.HipProjection(N, N, N, comm=comm,
                            cg_variant=int(os.environ.get("CFD_CAV512_CG_VARIANT", "0")))
    for fid in FIDS.values():
        ctx.fill(fid, 0.0)
    ctx.set_density(1.0)
    ctx.apply_dirichlet(A.HIP_FIELD_U, api.dirichlet(top=1.0))
    ctx.apply_dirichlet(A.HIP_FIELD_V, api.dirichlet())
    ctx.apply_dirichlet(A.HIP_FIELD_W, api.dirichlet())
    ctx.apply_scalar_bc(A.HIP_FIELD_P, A.BC_TYPE_NEUMANN)
    loc, glob = ctx.owned()
    plane_steps = {int(v) for v in os.environ.get("CFD_CAV512_PLANE_STEPS", "1").split(",") if v}
    steps = []
    planes = {}
    ctx.enable_timing(True)
    for s in range(1, STEPS + 1):
        ctx.reset_timing()
        st = A.SolverStats()
        rc = ctx.step_device(g, params, st)
        if rc != A.CFD_SUCCESS:
            raise SystemExit(f"rank {RANK} step {s}: status {rc}")
        ps = ctx.poisson_stats()
        kt = ctx.timing()
        # how this step's dots were reduced: ncclAllReduce spans (+ finish
        # kernels) are timed as "allreduce"; the mailbox runs inside the
        # sweeps and leaves none
        red = {"allreduce_spans": kt["allreduce"][1],
               "march_launches": kt["cc_fused"][1] + kt["cc_fold"][1],
               "sweep_a_launches": kt["cg_sweep_a"][1] + kt["cg_sweep_bx"][1]}
        part = {}
        for k, fid in FIDS.items():
            a = ctx.get_field(fid)[loc]
            # the interior planes this rank owns (global 1 .. N-2)
            ks = [i for i in range(a.shape[0]) if 1 <= glob.start + i <= N - 2]
            t = torch.from_numpy(np.ascontiguousarray(a[ks][:, 1:-1, 1:-1]))
            part[k] = (float(torch.sum(t * t)), float(t.abs().max()))
            if s in plane_steps:
                for kz in (1, 255, 510):
                    if glob.start <= kz < glob.stop:
                        planes[f"{k}_{kz}_s{s}"] = a[kz - glob.start].copy()
        mine = (ps.iterations, ps.initial_residual, ps.final_residual, st.max_velocity,
                st.max_pressure, part, red)
        if RANK == 0:
            print(f"rank 0 step {s}: {ps.iterations} CG iterations, {red}", flush=True)
        allp = [None] * WORLD
        dist.all_gather_object(allp, mine)
        if RANK == 0:
            if any(p[:3] != allp[0][:3] for p in allp):
                raise SystemExit(f"ranks disagree on the CG statistics at step {s}: {allp}")
            norms = {k: [float(np.sqrt(sum(p[5][k][0] for p in allp))),
                         max(p[5][k][1] for p in allp)] for k in FIDS}
            steps.append({"iters": allp[0][0], "res0": allp[0][1], "res": allp[0][2],
                          "vmax": max(p[3] for p in allp), "pmax": max(p[4] for p in allp),
                          "norms": norms, "reduction": [p[6] for p in allp],
                          "device_allreduce": bool(comm.device_allreduce)})
    allplanes = [None] * WORLD
    dist.all_gather_object(allplanes, planes)
    dev_ar = bool(comm.device_allreduce)
    ctx.close()
    comm.close()
    if RANK == 0:
        out = os.environ["CFD_CAV512_OUT"]
        merged = {}
        for p in allplanes:
            merged.update(p)
        np.savez(out.replace(".json", "_planes.npz"), **merged)
        with open(out, "w") as fh:
            json.dump({"world": WORLD, "device_allreduce": dev_ar, "steps": steps}, fh)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
