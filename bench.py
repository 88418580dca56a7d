#!/usr/bin/env python
"""MPC solves/sec of the batched OSQP-SQP inner loop (B2G whole_body_rnea, N=50).

One "step" = one MPC step of the whole per-GPU batch, entirely on the device:
gait schedule + x_init update, warm start, sqp_data (node evaluation and dual
Jacobians), OSQP update (Ruiz scaling + block KKT factor), ADMM (<= 100 iterations,
termination checks every 25), Armijo/filter line search and the state update
x <- integrate(x, DX[1]) (run_mpc.py:127-143).  Inputs are resident in HBM when
the timed region starts; nothing crosses PCIe inside it.

Multi-GPU: one process per GPU (torchrun), problems [rank*B, (rank+1)*B) with
seeds from the global problem index (weak scaling, no data-path collective); the
per-problem results are all-gathered over RCCL after the timed region.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "pino-locoman_amd"))

from pinoloco import robots  # noqa: E402
from pinoloco.ocp import BatchedOCP, Layout, default_weights  # noqa: E402

METRIC = "MPC solves/sec (B2G whole_body_rnea N=50) at batch; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)


def random_problem(R, lay, gidx):
    """Per-problem randomisation, seed = 1234 + global index."""
    rng = np.random.default_rng(1234 + gidx)
    q = R.q0.copy()
    q[:3] += rng.normal(0.0, 0.01, 3)
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    ang = rng.uniform(0.0, 0.05)
    q[3:7] = np.concatenate([axis * np.sin(ang / 2), [np.cos(ang / 2)]])
    q[7:] = np.clip(q[7:] + rng.normal(0.0, 0.05, R.nj), R.joint_pos_min, R.joint_pos_max)
    v = rng.normal(0.0, 0.1, R.nv)
    t0 = rng.uniform(0.0, 0.8)
    vx = rng.uniform(0.0, 0.3)
    return np.concatenate([q, v]), t0, vx


def build_batch(R, dynamics, N, B, first):
    lay = Layout(R, dynamics, N)
    Q, Rw, W = default_weights(R, dynamics, lay)
    P = np.zeros((B, lay.np))
    X = np.zeros((B, lay.n))
    XS = np.zeros((B, lay.nx))
    T0 = np.zeros(B)
    fg = 9.81 * R.mass
    fdes = np.array([0, 0, 0.8 * fg / 2] * 2 + [0, 0, 1.2 * fg / 2] * 2 + ([0, 0, 0] if R.ext_force_frame else []))
    udes = np.concatenate([np.zeros(lay.na), fdes, np.zeros(R.nj)])
    x0 = np.zeros(lay.n)
    for i in range(N):
        o = lay.x_off[i] + lay.ndx
        x0[o:o + lay.nu[i]] = udes[:lay.nu[i]]
    for b in range(B):
        xs, t0, vx = random_problem(R, lay, first + b)
        vals = dict(x_init=xs, dt_min=0.01, dt_max=0.08, n_contacts=2, swing_period=0.4, swing_height=0.07,
                    swing_vel_limits=[0.1, -0.2], Q_diag=Q, R_diag=Rw, base_vel_des=[vx, 0, 0, 0, 0, 0],
                    ext_force_des=[0, 0, 0], arm_vel_des=[0, 0, 0], tau_prev=np.zeros(R.nj), W_diag=W,
                    contact_schedule=np.ones((4, N)), swing_schedule=np.zeros((4, N)))
        P[b] = lay.pack(vals)
        X[b] = x0
        XS[b] = xs
        T0[b] = t0
    return lay, P, X, XS, T0


def admm_bytes_per_problem_iter(sz):
    """Algorithmic HBM bytes of one ADMM iteration of one problem (roofline):
    both sweeps read the factor once (2 * S), A is read once, and the vectors
    x, rhs, bt, q (7n) and z, y, l, u, rho (7m) are read / written once."""
    return 8.0 * (2 * sz["S_stride"] + sz["nnz"] + 7 * sz["n"] + 7 * sz["m"])


def cpu_baseline(R, dynamics, N, n_problems=2, n_steps=2):
    """Oracle (numpy restatement of the reference path) on a bounded sample, 1 core."""
    sys.path.insert(0, HERE)
    from oracle.ocp import OracleOCP  # noqa: E402  (checker / baseline only)
    lay, P, X, XS, T0 = build_batch(R, dynamics, N, n_problems, 0)
    from pinoloco.gait import horizon_dts
    o = OracleOCP(R, dynamics, N)
    dts = horizon_dts(0.01, 0.08, N)
    elapsed, solves = 0.0, 0
    for b in range(n_problems):
        xs = XS[b].copy()
        x = X[b].copy()
        oo = OracleOCP(R, dynamics, N)
        for k in range(n_steps):
            p = P[b].copy()
            c, s = R.gait_sequence.get_gait_schedule(T0[b] + k * 0.01, dts, N)
            vals = o.unpack(p)
            p = oo.pack_params(x_init=xs, dt_min=0.01, dt_max=0.08, contact=c, swing=s, n_contacts=2,
                               swing_period=0.4, swing_height=0.07, swing_vel_limits=[0.1, -0.2],
                               Q_diag=vals["Q_diag"], R_diag=vals["R_diag"], base_vel_des=vals["base_vel_des"],
                               ext_force_des=[0, 0, 0], arm_vel_des=[0, 0, 0], tau_prev=np.zeros(R.nj),
                               W_diag=vals.get("W_diag", np.zeros(R.nj)))
            if k == 0:
                oo.init_solver(x, p)  # OSQP setup: excluded like pl_ocp_init_solver
            else:
                x = oo.warm_start(x, p)
            t = time.perf_counter()
            x, _, _ = oo.sqp_step(x, p)
            DX, _ = oo.split(x)
            xs = oo.integrate_state(xs, DX[1])
            elapsed += time.perf_counter() - t
            solves += 1
    return {"value": solves / elapsed, "unit": "solves/s", "cores": 1, "kind": "port",
            "sample": f"{n_problems} problems x {n_steps} MPC steps, numpy oracle (oracle/), single thread"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1024, help="problems per GPU")
    ap.add_argument("--robot", default="b2g")
    ap.add_argument("--dynamics", default="whole_body_rnea")
    ap.add_argument("--nodes", type=int, default=50)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist_mod
        torch.cuda.set_device(local_rank)
        dist_mod.init_process_group("nccl")
        dist = dist_mod

    R = robots.ROBOTS[args.robot]()
    R.set_gait_sequence("trot", 0.8)
    B = args.batch
    lay, P, X, XS, T0 = build_batch(R, args.dynamics, args.nodes, B, rank * B)
    bo = BatchedOCP(R, args.dynamics, args.nodes, batch=B, device=local_rank, gait_type="trot", gait_period=0.8)
    bo.set_params(P)
    bo.set_x(X)
    bo.init_solver()
    bo.mpc_setup(XS, T0)

    def barrier_sync():
        bo.sync()
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    for k in range(args.warmup):
        bo.mpc_step(k)
    barrier_sync()
    bo.profile(1)
    barrier_sync()
    t0 = time.perf_counter()
    for k in range(args.warmup, args.warmup + args.steps):
        bo.mpc_step(k)
    barrier_sync()
    elapsed = time.perf_counter() - t0
    prof = bo.profile_read()
    bo.profile(0)
    if dist is not None:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=f"cuda:{local_rank}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        # final gather of per-problem controls + states over RCCL (outside the timed region)
        row = lay.nu[0] + lay.nx
        mine = torch.empty((B, row), dtype=torch.float64, device=f"cuda:{local_rank}")
        bo.mpc_export(mine.data_ptr())
        allp = [torch.empty_like(mine) for _ in range(world)]
        dist.all_gather(allp, mine)
        torch.cuda.synchronize()

    sz = bo.sizes()
    bytes_it = admm_bytes_per_problem_iter(sz)
    per_launch_bytes = bytes_it * prof["problem_iters"] / max(1, prof["launches"])
    avg_launch_s = prof["admm_ms"] / max(1, prof["launches"]) / 1e3
    achieved = per_launch_bytes / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    traffic = None
    tfile = os.path.join(HERE, "profiles", "admm_traffic.json")
    if os.path.exists(tfile):
        try:
            with open(tfile) as fh:
                tj = json.load(fh)
            if tj.get("batch") == B and tj.get("nodes") == args.nodes:
                traffic = tj.get("bytes_per_launch")
        except Exception:  # noqa: BLE001
            traffic = None

    if rank == 0:
        total = B * world * args.steps
        out = {
            "metric": METRIC,
            "value": total / elapsed,
            "unit": "solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (randomised initial state / gait phase / base velocity target, seed 1234 + problem)",
            "config": {"workload": f"{args.robot} {args.dynamics} N={args.nodes} MPC step", "batch_per_gpu": B,
                       "global_batch": B * world, "nodes": args.nodes, "robot": args.robot,
                       "dynamics": args.dynamics, "solver": "osqp-sqp (1 SQP iteration, max_iter 100)",
                       "parallelism": f"batch-sharded dp{world}"},
            "roofline": {"bound": "hbm", "kernel": "k_admm", "achieved": achieved, "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "bytes_per_problem_iter": bytes_it, "avg_launch_ms": avg_launch_s * 1e3,
                         "launches": prof["launches"]},
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(R, args.dynamics, args.nodes)
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
