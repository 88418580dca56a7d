"""World-size-2 gloo run of the multi-GPU plumbing (pinoloco/dist.py, synthetic.shard).

Each rank builds its shard of the global batch from the global problem index,
runs host-side work through the C-ABI on it (pl_state_integrate of each
problem's state), and the rows are all-gathered; rank 0 checks that the
gathered job equals the single-process computation problem by problem and that
the timed-region reduction is a MAX.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import ROOT

GLOBAL_B = 7  # odd on purpose: shards of 4 and 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _work(R, XS, first=0):
    from pinoloco.ocp import Dynamics
    integ = Dynamics(R).state_integrate()
    rows = []
    for b, xs in enumerate(XS):
        dx = np.sin(np.arange(2 * R.nv) + (first + b) * 0.1) * 0.05
        rows.append(integ(xs, dx))
    return np.array(rows)


def _rank_main(rank, world, port, out_dir):
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "pino-locoman_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    from pinoloco import dist as pdist, robots
    from pinoloco.synthetic import build_batch, shard
    d = pdist.init("gloo")
    assert d is not None and d.get_world_size() == world
    R = robots.ROBOTS["go2"]()
    R.set_gait_sequence("trot", 0.8)
    first, count = shard(GLOBAL_B, world, rank)
    _, P, _, XS, _ = build_batch(R, "whole_body_rnea", 8, count, first)
    rows = torch.from_numpy(np.concatenate([P[:, :5], _work(R, XS, first)], 1))
    allr = pdist.gather_rows(rows, d)
    tmax = pdist.max_over_ranks(float(rank + 1), d)
    if rank == 0:
        np.save(os.path.join(out_dir, "gathered.npy"), allr.numpy())
        np.save(os.path.join(out_dir, "tmax.npy"), np.array([tmax]))
    d.barrier()
    d.destroy_process_group()


@pytest.mark.slow
def test_gloo_world2_shard_and_gather(tmp_path):
    from pinoloco import robots
    from pinoloco.synthetic import build_batch
    port = _free_port()
    mp.start_processes(_rank_main, args=(2, port, str(tmp_path)), nprocs=2, join=True, start_method="spawn")
    got = np.load(tmp_path / "gathered.npy")
    R = robots.ROBOTS["go2"]()
    R.set_gait_sequence("trot", 0.8)
    _, P, _, XS, _ = build_batch(R, "whole_body_rnea", 8, GLOBAL_B, 0)
    want = np.concatenate([P[:, :5], _work(R, XS)], 1)
    assert got.shape == want.shape
    assert np.array_equal(got, want)
    assert float(np.load(tmp_path / "tmax.npy")[0]) == 2.0
