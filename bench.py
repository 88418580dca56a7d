#!/usr/bin/env python
"""MPC solves/sec of the batched OSQP-SQP inner loop (B2G whole_body_rnea, N=50).

One "step" = one MPC step of the whole per-GPU batch, entirely on the device:
gait schedule + x_init update, warm start, sqp_data (node evaluation and dual
Jacobians), OSQP update (Ruiz scaling + block KKT factor), ADMM (<= 100 iterations,
termination checks every 25), Armijo/filter line search and the state update
x <- integrate(x, DX[1]) (run_mpc.py:127-143).  Inputs are resident in HBM when
the timed region starts; nothing crosses PCIe inside it.  A second, shorter timed pass
adds the per-step download of the controller output [u_0, x_state] (the "host_io" object:
the PCIe-inclusive rate, never `value`).

Multi-GPU: one process per GPU (torchrun), problems [rank*B, (rank+1)*B) with
seeds from the global problem index (weak scaling, no data-path collective); the
per-problem results are all-gathered over RCCL after the timed region.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B]

With --gpus N > 1 and no torchrun environment, bench.py launches the N ranks itself
(torch.distributed.run as a child process, before anything touches the GPU) and
relays rank 0's JSON line.  --dry-run exercises the same rank / shard / gather
plumbing over gloo on the CPU without solving (tests/test_bench.py).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "pino-locoman_amd"))

from pinoloco import robots  # noqa: E402
from pinoloco.ocp import BatchedOCP  # noqa: E402
from pinoloco import dist as pdist  # noqa: E402
from pinoloco.synthetic import build_batch, shard  # noqa: E402

METRIC = "MPC solves/sec (B2G whole_body_rnea N=50) at batch; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)


TRAFFIC_FILE = os.path.join(HERE, "profiles", "traffic", "admm_traffic.json")
TRAFFIC_SOURCES = ("pino-locoman_amd/csrc/k_admm.hip", "pino-locoman_amd/csrc/admm_common.h",
                   "pino-locoman_amd/csrc/state.h")


def admm_bytes_per_problem_iter(sz, node_table, padded=False, kernel="sweep", ndx=None):
    """Algorithmic HBM bytes of one ADMM iteration of one problem (roofline),
    per GPU mapping of the linear solve:

    * "sweep" (k_admm) and "sweep2" (k_admm2): the two sweeps read every factor block S_i
      once each, except S_0 and S_N which the fused turnaround steps read once per
      iteration;
    * "chain" (k_admm_rc): every S_i once, plus the reduced-chain blocks F_i, F_i^T, G_i
      (3 ndx^2 doubles) of the N nodes with a successor (k_admm_rc.hip header);

    and for all of them A read once, and the vectors x, rhs, bt, q (7n) and z, y, l, u, rho
    (7m) read / written once.  A factor block is the stored lower triangle nw (nw + 1) / 2
    of S_i; padded=True counts the 4x4 lane-tile slots the kernels actually stream
    (K x 64 lanes x 16)."""
    nw = node_table[:, 0].astype(float)
    blk = node_table[:, 9].astype(float) * 64 * 16 if padded else nw * (nw + 1) / 2
    vec = sz["nnz"] + 7 * sz["n"] + 7 * sz["m"]
    if kernel == "chain":
        return 8.0 * (blk.sum() + 3.0 * (len(nw) - 1) * float(ndx) ** 2 + vec)
    return 8.0 * (2 * blk.sum() - blk[0] - blk[-1] + vec)


HESS_FLOPS_FILE = os.path.join(HERE, "profiles", "traffic", "hess_flops.json")
HESS_SOURCES = ("pino-locoman_amd/csrc/k_hess.hip", "pino-locoman_amd/csrc/hess_tree.h", "pino-locoman_amd/csrc/rows.h",
                "pino-locoman_amd/csrc/rbd.h", "pino-locoman_amd/csrc/ad.h", "pino-locoman_amd/csrc/targets.h")
FP64_PEAK_TFLOPS = 78.6  # MI355X dense FP64 vector (MI355X_MICROARCH.md)


def hess_source_sha():
    h = hashlib.sha256()
    for rel in HESS_SOURCES:
        with open(os.path.join(HERE, rel), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def measured_hess_flops(batch, nodes, workload, mapping):
    """F64 flops per k_lag_hess launch from a committed PMC pass (SQ_INSTS_VALU_{FMA,MUL,ADD}_F64
    x 64 lanes, an FMA counted as 2), or None if taken on other sources / workload / mapping."""
    try:
        with open(HESS_FLOPS_FILE) as fh:
            tj = json.load(fh)
    except (OSError, ValueError):
        return None
    if (tj.get("src_sha") != hess_source_sha() or tj.get("batch") != batch or tj.get("nodes") != nodes
            or tj.get("workload") != workload or tj.get("mapping") != mapping):
        return None
    return tj


def traffic_source_sha():
    """sha256 of the k_admm sources: a PMC traffic measurement applies only to the
    kernel revision it was taken on."""
    h = hashlib.sha256()
    for rel in TRAFFIC_SOURCES:
        with open(os.path.join(HERE, rel), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def measured_traffic(batch, nodes, workload):
    """HBM bytes per problem-iteration of k_admm from the committed PMC passes
    (tools/pmc_traffic.py), or None if they were taken on another kernel revision
    or workload."""
    try:
        with open(TRAFFIC_FILE) as fh:
            tj = json.load(fh)
    except (OSError, ValueError):
        return None
    if (tj.get("src_sha") != traffic_source_sha() or tj.get("batch") != batch or tj.get("nodes") != nodes
            or tj.get("workload") != workload):
        return None
    return tj


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cgroup_cpu_quota():
    """CPUs granted by the cgroup CPU controller (v2 ``cpu.max`` or v1 cfs quota / period),
    or None when no quota is set: evidence for ``cores`` beside OMP_NUM_THREADS."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        return None if quota == "max" else int(quota) / int(period)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            quota = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            period = int(f.read())
        return None if quota <= 0 else quota / period
    except (OSError, ValueError):
        return None


def cpu_baseline(robot, dynamics, N, per_core=4, n_steps=2):
    """The compiled C++ restatement of the reference's CPU path (oracle/cpu/sqp_cpu.cpp:
    rows + dual Jacobians, OSQP 0.6 with the QDLDL LDL^T on the quasi-definite KKT,
    line search, MPC loop; -O3 -march=x86-64-v3, OpenMP over problems) on the host's
    CPU share, same workload and seeds as the GPU run.  Sample: per_core problems per
    thread x n_steps MPC steps, plus the single-thread latency of one problem.
    Runs before the GPU is initialised."""
    sys.path.insert(0, HERE)
    from oracle.cpu_baseline import CpuOCP  # noqa: E402  (baseline leg only)
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        avail = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    threads = max(1, min(avail, int(env))) if env else avail  # the box's CPU share is exported as OMP_NUM_THREADS
    R = robots.ROBOTS[robot]()
    R.set_gait_sequence("trot", 0.8)
    B = per_core * threads
    lay, P, X, XS, T0 = build_batch(R, dynamics, N, B, 0)
    c = CpuOCP(R, dynamics, N, gait_type="trot", gait_period=0.8)
    wall, _, _ = c.mpc(P, X, XS, T0, n_steps, threads=threads)
    w1, _, _ = c.mpc(P[:1], X[:1], XS[:1], T0[:1], n_steps, threads=1)
    return {"value": B * n_steps / wall, "unit": "solves/s", "cores": threads, "kind": "port",
            "sample": f"{B} problems x {n_steps} MPC steps of the same workload (seeds 0..{B - 1}) on {threads} OpenMP "
                      f"threads; compiled C++ restatement of the reference CPU path (oracle/cpu/sqp_cpu.cpp: OSQP 0.6 "
                      f"+ QDLDL LDL^T, Armijo/filter line search), g++ -O3 -march=x86-64-v3",
            "single_core_ms_per_solve": w1 / n_steps * 1e3, "cpu_model": _cpu_model(), "host_cpus_visible": avail,
            "omp_num_threads_env": env, "cgroup_cpu_quota": _cgroup_cpu_quota()}


def cpu_baseline_ip(robot, dynamics, N, per_core=1):
    """The compiled C++ restatement of the interior-point stand-in for the reference's Fatrop
    branch (oracle/cpu/sqp_cpu.cpp restating oracle/ip_ref.py: exact Lagrangian Hessian by
    hyper-dual node passes over the structurally non-zero pairs, QDLDL on the IP's
    quasi-definite KKT, inertia correction, filter line search; OpenMP over problems), same
    workload, seeds and driver branch as the GPU run (the reference's default compiled-solver
    driver: primal warm start, cold multipliers).  Not Fatrop (absent from the image and the
    reference).  Sample: per_core problems per thread; the time of MPC step 1 (the first
    warm-started solve, as the GPU line times warm steps) = the wall of steps 0-1 minus the wall
    of step 0 alone (the computation of step 0 is identical in both runs).  Runs before the GPU
    is initialised."""
    sys.path.insert(0, HERE)
    from oracle.cpu_baseline import CpuOCP  # noqa: E402  (baseline leg only)
    try:
        avail = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        avail = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    threads = max(1, min(avail, int(env))) if env else avail
    R = robots.ROBOTS[robot]()
    R.set_gait_sequence("trot", 0.8)
    B = per_core * threads
    lay, P, X, XS, T0 = build_batch(R, dynamics, N, B, 0)
    c = CpuOCP(R, dynamics, N, gait_type="trot", gait_period=0.8)
    pairs = c.hess_pairs()
    w1, _, _ = c.ip_mpc(P, X, XS, T0, 1, threads=threads)
    w2, _, st = c.ip_mpc(P, X, XS, T0, 2, threads=threads)
    wall = max(w2 - w1, 1e-9)
    return {"value": B / wall, "unit": "solves/s", "cores": threads, "kind": "port",
            "step0_s": w1, "step1_s": wall,
            "step1_status_counts": {int(k): int(v) for k, v in zip(*np.unique(st[:, 1, 0], return_counts=True))},
            "sample": f"{B} problems of the same workload (seeds 0..{B - 1}), MPC step 1 (the first warm-started solve: "
                      f"primal warm start, cold multipliers, the reference's default driver) timed as the wall of steps "
                      f"0-1 minus that of step 0, on {threads} OpenMP threads; compiled C++ restatement of the interior-point "
                      f"stand-in for the reference's Fatrop branch (oracle/cpu/sqp_cpu.cpp restating oracle/ip_ref.py: "
                      f"exact Lagrangian Hessian by hyper-dual passes over {pairs} column pairs, whole_body_rnea's "
                      f"(dq, a) / (dq, f_feet) blocks by dual passes as on the GPU, QDLDL LDL^T on the KKT, IPOPT "
                      f"inertia correction, filter line search), not Fatrop; g++ -O3 -march=x86-64-v3",
            "per_thread_s_per_solve": wall * threads / B, "mean_iter": float(st[:, 1, 1].mean()),
            "cpu_model": _cpu_model(), "host_cpus_visible": avail, "omp_num_threads_env": env,
            "cgroup_cpu_quota": _cgroup_cpu_quota()}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n):
    """Run this script as `n` ranks (one process per GPU) via torch.distributed.run in a
    child process; rank 0 prints the JSON line to the inherited stdout.  Called before
    any GPU work, so nothing is exec'ed from a process that initialised the GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.run(cmd, env=env).returncode


def dry_run(args, world, rank):
    """Rank / shard / gather plumbing over gloo on the CPU (no GPU, no solve)."""
    import torch
    dist = pdist.init("gloo")
    R = robots.ROBOTS[args.robot]()
    R.set_gait_sequence("trot", 0.8)
    B = args.batch
    first, count = shard(B * world, world, rank)
    lay, P, X, XS, T0 = build_batch(R, args.dynamics, args.nodes, count, first)
    t0 = time.perf_counter()
    elapsed = pdist.max_over_ranks(time.perf_counter() - t0, dist)
    allp = pdist.gather_rows(torch.from_numpy(np.concatenate([X[:, :lay.nu[0]], XS], 1)), dist)
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "unit": "solves/s", "n_gpus": world, "steps": 0,
                          "warmup": 0, "ms_per_step": elapsed * 1e3, "higher_is_better": True, "scaling": "weak",
                          "dry_run": True, "gathered_rows": int(allp.shape[0]),
                          "config": {"workload": f"{args.robot} {args.dynamics} N={args.nodes} MPC step",
                                     "batch_per_gpu": B, "global_batch": B * world}}), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=80)  # >= 10 s timed at the headline config
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--batch", type=int, default=1024, help="problems per GPU")
    ap.add_argument("--robot", default="b2g")
    ap.add_argument("--dynamics", default="whole_body_rnea")
    ap.add_argument("--nodes", type=int, default=50)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--solver", default="osqp", choices=["osqp", "fatrop"],
                    help="osqp: the headline SQP + OSQP path; fatrop: the interior-point restatement")
    ap.add_argument("--dry-run", action="store_true", help="gloo plumbing only, no GPU")
    ap.add_argument("--admm-kernel", default="auto", choices=["auto", "sweep", "sweep2", "chain"],
                    help="ADMM mapping (pl_ocp_set_admm_kernel); auto = the library's batch-size rule")
    ap.add_argument("--debug-paths", default="",
                    help="comma list of pl_ocp_desc.debug_paths names (earlier kernel paths, A/B runs only)")
    ap.add_argument("--host-io-steps", type=int, default=None,
                    help="extra steps timed with the per-step D2H of [u_0, x_state] (default min(steps, 10))")
    args = ap.parse_args()
    if args.host_io_steps is None:
        args.host_io_steps = min(args.steps, 10)

    world, rank, local_rank = pdist.env_ranks()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one rank per GPU")
    if args.dry_run:
        return dry_run(args, world, rank)
    base = None
    if not args.no_cpu_baseline and world == 1:  # before the GPU is initialised
        if args.solver == "osqp":
            base = cpu_baseline(args.robot, args.dynamics, args.nodes)
        else:
            base = cpu_baseline_ip(args.robot, args.dynamics, args.nodes)
    dist = pdist.init("nccl")

    R = robots.ROBOTS[args.robot]()
    R.set_gait_sequence("trot", 0.8)
    B = args.batch
    first, _ = shard(B * world, world, rank)
    lay, P, X, XS, T0 = build_batch(R, args.dynamics, args.nodes, B, first)
    paths = tuple(p for p in args.debug_paths.split(",") if p)
    bo = BatchedOCP(R, args.dynamics, args.nodes, batch=B, device=local_rank, gait_type="trot", gait_period=0.8,
                    debug_paths=paths)
    if args.solver == "fatrop":
        bo.set_solver("fatrop")
        bo.set_ip_settings()
    if args.admm_kernel != "auto":
        bo.set_admm_kernel(args.admm_kernel)
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

    # Per-launch HIP events on the ADMM launches (the roofline's avg_launch_ms) are taken
    # over the timed region itself for batches >= 64.  A latency-bound small batch replays
    # each MPC step as one HIP graph (pl_mpc_step), which per-launch events would disable:
    # there the ADMM launches are timed over the same number of profiled steps right after.
    prof_timed = args.batch >= 64
    for k in range(args.warmup):
        bo.mpc_step(k)
    barrier_sync()
    if prof_timed:
        bo.profile(1)
    barrier_sync()
    ip_steps = []
    if args.solver == "fatrop":
        # interior point (~0.5 s per step): each step timed between stream syncs, and its per-problem
        # outcome read after the clock stops (status counts of every timed step, outside the time)
        elapsed = 0.0
        for k in range(args.warmup, args.warmup + args.steps):
            t0 = time.perf_counter()
            bo.mpc_step(k)
            bo.sync()
            elapsed += time.perf_counter() - t0
            ist = bo.ip_stats()
            ip_steps.append({"step": k, "status_counts": {int(a): int(c) for a, c in
                                                          zip(*np.unique(ist["status"], return_counts=True))},
                             "mean_iter": float(np.mean(ist["iter"]))})
        barrier_sync()
    else:
        t0 = time.perf_counter()
        for k in range(args.warmup, args.warmup + args.steps):
            bo.mpc_step(k)
        barrier_sync()
        elapsed = time.perf_counter() - t0
    if not prof_timed:
        bo.profile(1)
        for k in range(args.warmup + args.steps, args.warmup + 2 * args.steps):
            bo.mpc_step(k)
        bo.sync()
    prof = bo.profile_read()
    hprof = bo.profile_read_hess() if args.solver == "fatrop" else None  # read before profile(0) clears
    bo.profile(0)
    elapsed = pdist.max_over_ranks(elapsed, dist)
    if dist is not None:
        # per-problem controller output [u_0, x_state] of the whole job, gathered over
        # RCCL after the timed region (no collective on the data path)
        import torch
        mine = torch.empty((B, lay.nu[0] + lay.nx), dtype=torch.float64, device=f"cuda:{local_rank}")
        bo.mpc_export(mine.data_ptr())
        bo.sync()
        allp = pdist.gather_rows(mine, dist)
        torch.cuda.synchronize()
        assert allp.shape[0] == B * world

    host_io = None
    if args.host_io_steps > 0:
        # PCIe-inclusive rate (never `value`): each step followed by the D2H of the per-problem
        # controller output [u_0, x_state] into host memory and a wait for it, as a real-time
        # loop reads it (run_mpc.py:138-141); SURVEY 8(d)
        buf = np.zeros((B, lay.nu[0] + lay.nx))
        k0 = args.warmup + 2 * args.steps
        barrier_sync()
        t1 = time.perf_counter()
        for k in range(k0, k0 + args.host_io_steps):
            bo.mpc_step(k)
            bo.mpc_download(buf)
        barrier_sync()
        e1 = pdist.max_over_ranks(time.perf_counter() - t1, dist)
        assert np.all(np.isfinite(buf))
        host_io = {"value": B * world * args.host_io_steps / e1, "unit": "solves/s",
                   "ms_per_step": e1 / args.host_io_steps * 1e3, "steps": args.host_io_steps,
                   "d2h_bytes_per_step": int(buf.nbytes),
                   "what": "per step: pl_mpc_step + pl_mpc_download ([u_0, x_state] of every problem to "
                           "host memory) + wait; inputs resident, the state stays on the device"}

    kernel = bo.admm_kernel()
    kname = {"sweep": "k_admm", "sweep2": "k_admm2", "chain": "k_admm_rc"}[kernel]
    sz = bo.sizes()
    ntab = bo.node_table()
    bytes_it = admm_bytes_per_problem_iter(sz, ntab, kernel=kernel, ndx=lay.ndx)
    bytes_it_padded = admm_bytes_per_problem_iter(sz, ntab, padded=True, kernel=kernel, ndx=lay.ndx)
    iters_per_launch = prof["problem_iters"] / max(1, prof["launches"])
    per_launch_bytes = bytes_it * iters_per_launch
    avg_launch_s = prof["admm_ms"] / max(1, prof["launches"]) / 1e3
    achieved = per_launch_bytes / avg_launch_s / 1e9 if avg_launch_s > 0 else 0.0
    workload = f"{args.robot} {args.dynamics} N={args.nodes} MPC step"
    tj = measured_traffic(B, args.nodes, workload) if kernel == "sweep" else None
    # PMC bytes per problem-iteration x this run's problem-iterations per launch
    traffic = tj["bytes_per_problem_iter"] * iters_per_launch if tj else None

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
            "config": {"workload": workload, "batch_per_gpu": B,
                       "global_batch": B * world, "nodes": args.nodes, "robot": args.robot,
                       "dynamics": args.dynamics,
                       "solver": ("osqp-sqp (1 SQP iteration, max_iter 100)" if args.solver == "osqp" else
                                  "fatrop-equivalent interior point (max_iter 10, tol 1e-3, mu_init 1e-4)"),
                       "parallelism": f"batch-sharded dp{world}", **({"debug_paths": list(paths)} if paths else {})},
            "roofline": {"bound": "hbm", "kernel": kname, "byte_model": kernel, "workgroups_per_problem": bo.admm_groups(),
                         "achieved": achieved,
                         "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "algorithmic_bytes_per_launch": per_launch_bytes,
                         "bytes_per_problem_iter": bytes_it, "bytes_per_problem_iter_padded": bytes_it_padded,
                         "problem_iters_per_launch": iters_per_launch, "avg_launch_ms": avg_launch_s * 1e3,
                         "launches": prof["launches"], "launch_timing": "timed region" if prof_timed else "profiled steps after the timed region (graph replay in it)",
                         "traffic_source": (f"profiles/traffic/admm_traffic.json (k_admm src {tj['src_sha']})"
                                            if tj else None)},
        }
        from pinoloco import _lib as plib
        from pinoloco import build as pbuild
        # provenance: the source hash compiled into the loaded library (pl_build_info) and
        # whether it is this tree's
        out["build"] = {"lib_src_sha256": plib.build_sha(), "tree_matches": plib.build_sha() == pbuild.source_sha()}
        if host_io is not None:
            out["host_io"] = host_io
        if base is not None:
            out["cpu_baseline"] = base
        if args.solver == "fatrop":
            # the IP step's dominant kernel is the Lagrangian Hessian (FP64 VALU-bound): its own
            # roofline; the ADMM sweeps' HBM line above moves to admm_roofline
            hp = hprof
            h_avg = hp["hess_ms"] / max(1, hp["launches"])
            hf = measured_hess_flops(B, args.nodes, workload, "sweep")
            # the PMC pass ran every problem in every evaluation; the kernels' waves follow the
            # active problems (k_ip_compact), so the flops of a launch scale with its lanes
            lane_frac = hp["lanes"] / (-(-B // 64) * 64) if hp.get("lanes") else 1.0
            flops = hf["flops_per_launch"] * lane_frac if hf else None
            ach = flops / (h_avg * 1e-3) / 1e12 if (hf and h_avg > 0) else None
            out["admm_roofline"] = out["roofline"]
            out["roofline"] = {"bound": "fp64_valu",
                               "kernel": "Lagrangian Hessian (k_lag_hess_col + _arm + _lin + _vv + _tree<true> + _cone; "
                                         "k_lag_hess_pb off the rnea family)",
                               "mapping": "sweep", "achieved": ach,
                               "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                               "frac": ach / FP64_PEAK_TFLOPS if ach is not None else None, "traffic": None,
                               "avg_launch_ms": h_avg, "launches": hp["launches"],
                               "flops_per_launch": flops,
                               "active_lane_fraction": lane_frac,
                               "flops_source": (f"profiles/traffic/hess_flops.json (PMC F64 instruction counts, "
                                                f"src {hf['src_sha']})" if hf else None)}
            tot = {}
            for st_ in ip_steps:
                for a, c in st_["status_counts"].items():
                    tot[a] = tot.get(a, 0) + c
            ok = tot.get(1, 0) + tot.get(-1, 0)  # converged or at the iteration cap (not -2 / -3)
            out["ip_stats"] = {"driver": "run_mpc.py default (compile_solver=True): primal warm start, cold multipliers",
                               "status_counts_timed": tot, "frac_ls_failed": tot.get(-2, 0) / max(1, sum(tot.values())),
                               "converged_or_max_iter_solves_per_s": ok * world / elapsed,
                               "per_step": ip_steps}
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
