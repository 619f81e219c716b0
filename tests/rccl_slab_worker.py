"""Worker for test_gpu_rccl.py: the Z-slab path over the RCCL backend, one
process per rank (launched by torch.distributed.run).

On a one-GPU box the ranks share the device, which RCCL refuses for ranks of
one host ("Duplicate GPU detected"); each rank therefore gets its own
NCCL_HOSTID, so RCCL treats them as two hosts and moves the halo planes and
all-reduces over its socket transport. The calls our library makes
(grouped ncclSend/ncclRecv, ncclAllReduce on the context stream) are the
same as over xGMI on an 8-GPU node.
"""
import os
import sys

RANK = int(os.environ.get("RANK", "0"))
WORLD = int(os.environ.get("WORLD_SIZE", "1"))
if os.environ.get("CFD_RCCL_SHARED_GPU", "1") == "1":
    os.environ["NCCL_HOSTID"] = f"cfd-slab-test-rank{RANK}"

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402,F401
import torch.distributed as dist  # noqa: E402

from cfd_amd import _abi as A  # noqa: E402
from cfd_amd import api  # noqa: E402

FIELDS = {"u": A.HIP_FIELD_U, "v": A.HIP_FIELD_V, "w": A.HIP_FIELD_W, "p": A.HIP_FIELD_P}


def run_case(comm, name, g, f, p, n_steps, bc_dev, **cfg):
    ctx = api.HipProjection(g.nx, g.ny, g.nz, comm=comm, **cfg)
    sl = slice(ctx.k_offset, ctx.k_offset + ctx.nz_local)
    for k, fid in FIELDS.items():
        ctx.set_field(fid, getattr(f, k)[sl])
    ctx.set_density(1.0)
    hist = []
    for _ in range(n_steps):
        bc_dev(ctx)
        st = A.SolverStats()
        s = ctx.step_device(g, p, st)
        if s != A.CFD_SUCCESS:
            raise RuntimeError(f"{name}: rank {RANK} step status {s}")
        hist.append((ctx.poisson_stats().iterations, st.max_velocity, st.max_pressure))
    loc, glob = ctx.owned()
    part = (glob.start, glob.stop, {k: ctx.get_field(fid)[loc] for k, fid in FIELDS.items()})
    ctx.close()
    parts = [None] * WORLD
    dist.all_gather_object(parts, (part, hist))
    return parts


def main():
    dist.init_process_group("gloo")
    from oracle import oracle
    from tests import cases

    uid = [api.comm_unique_id() if RANK == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    comm = api.SlabComm.rccl(uid[0], RANK, WORLD, 0)
    assert comm.rank == RANK and comm.size == WORLD
    want_mb = os.environ.get("CFD_HIP_DEVICE_ALLREDUCE", "1") != "0"
    if comm.device_allreduce != want_mb:
        raise SystemExit(f"device all-reduce active={comm.device_allreduce}, expected {want_mb}")

    def cavity_bc(c):
        c.apply_dirichlet(A.HIP_FIELD_U, api.dirichlet(top=1.0))
        c.apply_dirichlet(A.HIP_FIELD_V, api.dirichlet())
        c.apply_dirichlet(A.HIP_FIELD_W, api.dirichlet())
        c.apply_scalar_bc(A.HIP_FIELD_P, A.BC_TYPE_NEUMANN)

    def tg_bc(c):
        for fid in FIELDS.values():
            c.apply_scalar_bc(fid, A.BC_TYPE_PERIODIC)

    failures = []

    def check(name, parts, f, ohist, exact):
        hists = [h for _, h in parts]
        if any(h != hists[0] for h in hists):
            failures.append(f"{name}: ranks disagree on state {hists}")
        for (ih, vh, ph), (io, vo, po) in zip(hists[0], ohist):
            if exact and (ih, vh, ph) != (io, vo, po):
                failures.append(f"{name}: stats {(ih, vh, ph)} != {(io, vo, po)}")
            if not exact and (abs(ih - io) > 1 or abs(vh - vo) > 1e-9 * abs(vo)):
                failures.append(f"{name}: stats {(ih, vh)} vs {(io, vo)}")
        for k in FIELDS:
            got = np.full(getattr(f, k).shape, np.nan)
            for (a, b, d), _ in parts:
                got[a:b] = d[k]
            ref = getattr(f, k)
            if exact:
                if not np.array_equal(got, ref):
                    failures.append(f"{name}: field {k} not bitwise")
            else:
                err = float(np.max(np.abs(got - ref))) / max(1.0, float(np.max(np.abs(ref))))
                if not err <= 1e-10:
                    failures.append(f"{name}: field {k} rel err {err}")

    # Red-Black SOR cavity: bitwise the oracle
    g, f, p = cases.cavity(17, 17, 17, Re=100.0, dt=5e-4)
    parts = run_case(comm, "rbsor", g, f, p, 3, cavity_bc, poisson_method=A.HIP_POISSON_REDBLACK,
                     poisson_tolerance=1e-2)
    if RANK == 0:
        oracle.set_projection_poisson_params(oracle.poisson_params(tolerance=1e-2))
        ohist = []
        for _ in range(3):
            api.cavity_bc(f, 1.0)
            s, st, it = oracle.projection_step(f, g, p, A.ORACLE_POISSON_REDBLACK)
            ohist.append((it, st.max_velocity, st.max_pressure))
        oracle.set_projection_poisson_params(None)
        check("rbsor", parts, f, ohist, exact=True)

    # CG cavity and periodic Taylor-Green: to rounding
    for name, (g, f, p), bc_dev, bc_host in (
            ("cg-cavity", cases.cavity(33, 33, 33, Re=100.0, dt=5e-4), cavity_bc,
             lambda ff: api.cavity_bc(ff, 1.0)),
            ("cg-tg", cases.tg3(17), tg_bc, cases.tg3_bc)):
        parts = run_case(comm, name, g, f, p, 3, bc_dev)
        if RANK == 0:
            ohist = []
            for _ in range(3):
                bc_host(f)
                s, st, it = oracle.projection_step(f, g, p, A.ORACLE_POISSON_CG)
                ohist.append((it, st.max_velocity, st.max_pressure))
            check(name, parts, f, ohist, exact=False)

    # single-reduction CG (cg_variant 1): one all-reduce of two values per
    # iteration (mailbox or ncclAllReduce); against the textbook oracle to
    # the variant's gate (iterations +-2, fields 1e-6)
    g, f, p = cases.cavity(33, 33, 33, Re=100.0, dt=5e-4)
    parts = run_case(comm, "cc-cavity", g, f, p, 3, cavity_bc, cg_variant=1)
    if RANK == 0:
        ohist = []
        for _ in range(3):
            api.cavity_bc(f, 1.0)
            s, st, it = oracle.projection_step(f, g, p, A.ORACLE_POISSON_CG)
            ohist.append(it)
        hists = [h for _, h in parts]
        if any(h != hists[0] for h in hists):
            failures.append(f"cc-cavity: ranks disagree on state {hists}")
        if any(abs(h[0] - io) > 2 for h, io in zip(hists[0], ohist)):
            failures.append(f"cc-cavity: iterations {[h[0] for h in hists[0]]} vs {ohist}")
        for k in ("u", "v", "w"):
            got = np.full(getattr(f, k).shape, np.nan)
            for (a, b, d), _ in parts:
                got[a:b] = d[k]
            ref = getattr(f, k)
            err = float(np.max(np.abs(got - ref))) / max(1e-300, float(np.max(np.abs(ref))))
            if not err <= 1e-6:
                failures.append(f"cc-cavity: field {k} rel err {err}")

    comm.close()
    ok = [not failures]
    dist.broadcast_object_list(ok, src=0)
    dist.destroy_process_group()
    if RANK == 0:
        for m in failures:
            print("FAIL", m)
        if not failures:
            print("RCCL_SLAB_OK")
    sys.exit(0 if ok[0] else 1)


if __name__ == "__main__":
    main()
