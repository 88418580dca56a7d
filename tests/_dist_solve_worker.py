"""Rank program of tests/test_dist_gpu.py::test_sharded_solve_two_ranks_gloo (not a test).

Run under torch.distributed.run with two ranks on the one GPU of a test box: each rank
solves its contiguous shard of the global batch (synthetic.shard, seeds from the global
problem index) through the C-ABI, downloads [u_0, x_state] per problem and all-gathers the
rows over gloo; rank 0 writes the gathered rows to argv[1]."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pino-locoman_amd"))


def main():
    import torch
    from pinoloco import dist as pdist
    from pinoloco import robots
    from pinoloco.ocp import BatchedOCP
    from pinoloco.synthetic import build_batch, shard
    out, total, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    world, rank, _ = pdist.env_ranks()
    dist = pdist.init("gloo")
    R = robots.ROBOTS["go2"]()
    R.set_gait_sequence("trot", 0.8)
    first, count = shard(total, world, rank)
    lay, P, X, XS, T0 = build_batch(R, "whole_body_rnea", 20, count, first)
    bo = BatchedOCP(R, "whole_body_rnea", 20, batch=count, device=0)
    bo.set_admm_kernel("sweep")
    bo.set_params(P)
    bo.set_x(X)
    bo.init_solver()
    bo.mpc_setup(XS, T0)
    for k in range(steps):
        bo.mpc_step(k)
    rows = bo.mpc_download()
    bo.close()
    allp = pdist.gather_rows(torch.from_numpy(rows), dist)
    if rank == 0:
        np.save(out, allp.numpy())
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
