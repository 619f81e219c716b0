"""The Z-slab path over RCCL with two processes (tests/rccl_slab_worker.py)."""
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent


@pytest.mark.parametrize("world,device_allreduce", [(2, "0"), (2, "1"), (4, "1")])
def test_rccl_slabs(hip_lib, world, device_allreduce):
    """device_allreduce=1 (the default): CG dots through the one-shot
    peer-memory mailbox (IPC-mapped between the processes, verified by a
    collective probe at communicator creation); 0: ncclAllReduce. With 4
    ranks the middle ranks exchange halos with two neighbours."""
    env = dict(os.environ)
    env["CFD_HIP_DEVICE_ALLREDUCE"] = device_allreduce
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env["PYTHONPATH"] = str(ROOT) + os.pathsep + env.get("PYTHONPATH", "")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--rdzv-backend=c10d", "--rdzv-endpoint=127.0.0.1:0", "--local-addr=127.0.0.1",
           str(ROOT / "tests" / "rccl_slab_worker.py")]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "RCCL_SLAB_OK" in r.stdout, out[-4000:]
