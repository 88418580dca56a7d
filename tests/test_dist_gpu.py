"""The RCCL leg of the multi-GPU path (pinoloco/dist.py) on the MI355X.

bench.py gathers the per-problem controller outputs [u_0, x_state] over RCCL after the
timed region: pl_mpc_export copies them from the library's stream into a torch buffer,
then dist.all_gather runs on torch's stream.  A one-GPU box cannot run two ranks, so this
runs that exact sequence in a world-size-1 "nccl" (RCCL) group and checks the gathered
rows against the library's own state, plus the max-over-ranks reduction of the timing.
The N > 1 sharding itself is covered with gloo at world size 2 (tests/test_dist.py)."""
import os
import socket

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
