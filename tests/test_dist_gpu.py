"""The RCCL leg of the multi-GPU path (pinoloco/dist.py) on the MI355X.

bench.py gathers the per-problem controller outputs [u_0, x_state] over RCCL after the
timed region: pl_mpc_export copies them from the library's stream into a torch buffer,
then dist.all_gather runs on torch's stream.  A one-GPU box cannot run two ranks, so this
runs that exact sequence in a world-size-1 "nccl" (RCCL) group and checks the gathered
rows against the library's own state, plus the max-over-ranks reduction of the timing.
The N > 1 path runs as two ranks on the one GPU with gloo for the collectives
(test_sharded_solve_two_ranks_gloo): each rank solves its shard of the global batch, and
the gathered rows equal one process solving the whole batch, bit for bit."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import make_robot

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_rccl_export_and_gather_world1():
    import torch
    import torch.distributed as dist
    from pinoloco import dist as pdist
    from pinoloco.ocp import BatchedOCP
    from pinoloco.synthetic import build_batch
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(_free_port())
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    try:
        R = make_robot("go2")
        B, N = 5, 20
        lay, P, X, XS, T0 = build_batch(R, "whole_body_rnea", N, B, 0)
        bo = BatchedOCP(R, "whole_body_rnea", N, batch=B, device=0)
        bo.set_params(P)
        bo.set_x(X)
        bo.init_solver()
        bo.mpc_setup(XS, T0)
        bo.mpc_step(0)
        bo.mpc_step(1)
        mine = torch.empty((B, lay.nu[0] + lay.nx), dtype=torch.float64, device="cuda:0")
        bo.mpc_export(mine.data_ptr())
        bo.sync()
        allp = pdist.gather_rows(mine, dist)
        torch.cuda.synchronize()
        assert pdist.max_over_ranks(1.25, dist) == 1.25
        got = allp.cpu().numpy()
        assert got.shape == (B, lay.nu[0] + lay.nx)
        x = bo.get_x()
        u0 = x[:, lay.ndx:lay.ndx + lay.nu[0]]
        assert np.array_equal(got[:, :lay.nu[0]], u0)
        assert np.array_equal(got[:, lay.nu[0]:], bo.mpc_state())
        bo.close()
    finally:
        dist.destroy_process_group()


def test_sharded_solve_two_ranks_gloo(tmp_path):
    """SURVEY 8e weak scaling, end to end on one GPU: torch.distributed.run starts two rank
    processes (gloo for the collectives: one GPU cannot host two RCCL ranks); rank r solves
    problems synthetic.shard(7, 2, r) for two MPC steps through the C-ABI and the rows
    [u_0, x_state] are all-gathered.  The result equals a single process solving all 7
    problems with the same ADMM kernel: problems are independent and a problem's bits do
    not depend on its batch (k_admm forced on both sides)."""
    from pinoloco.ocp import BatchedOCP
    from pinoloco.synthetic import build_batch
    total, steps = 7, 2
    out = str(tmp_path / "rows.npy")
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(here, "_dist_solve_worker.py"), out, str(total), str(steps)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=150)
    assert r.returncode == 0, r.stderr[-3000:]
    got = np.load(out)
    R = make_robot("go2")
    lay, P, X, XS, T0 = build_batch(R, "whole_body_rnea", 20, total, 0)
    bo = BatchedOCP(R, "whole_body_rnea", 20, batch=total, device=0)
    bo.set_admm_kernel("sweep")
    bo.set_params(P)
    bo.set_x(X)
    bo.init_solver()
    bo.mpc_setup(XS, T0)
    for k in range(steps):
        bo.mpc_step(k)
    want = bo.mpc_download()
    bo.close()
    assert got.shape == want.shape == (total, lay.nu[0] + lay.nx)
    assert np.array_equal(got, want)
