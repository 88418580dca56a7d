"""Generate the golden vectors in tests/golden/ from the numpy oracle.

The reference holds no tests, fixtures or golden vectors and its native
dependencies (pinocchio, casadi, osqp) are absent from this image (SURVEY.md
section 8c), so these vectors are produced by our CPU restatement (oracle/) and
pin it against regressions; parity with the reference itself is unpinned.

Run from the repository root:  python tests/golden/make_golden.py
Writes  tests/golden/rbd_<robot>.npz  and  tests/golden/sqp_<config>.npz.
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.normpath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "pino-locoman_amd"))

from oracle import rbd  # noqa: E402
from oracle.ocp import OracleOCP  # noqa: E402
from pinoloco import robots  # noqa: E402
from pinoloco.synthetic import build_batch, problem_values  # noqa: E402

# (fixture name, robot, dynamics, N, problems, closed-loop steps for problem 0)
SQP_CONFIGS = [
    ("go2_rnea_n20", "go2", "whole_body_rnea", 20, 2, 4),
    ("b2_aba_n40", "b2", "whole_body_aba", 40, 1, 1),
    ("b2g_acc_n50", "b2g", "whole_body_acc", 50, 1, 1),
    ("b2g_rnea_n50", "b2g", "whole_body_rnea", 50, 1, 1),
]


def rbd_fixture(rname, seed=7, count=3):
    R = robots.ROBOTS[rname]()
    R.set_gait_sequence("trot", 0.8)
    M = rbd.ModelArrays(R.model)
    rng = np.random.default_rng(seed)
    frames = list(R.foot_frames) + ([R.ext_force_frame] if R.ext_force_frame is not None else [])
    out = {k: [] for k in ("q", "v", "a", "f", "tau", "aba", "M", "dq", "q_int", "foot_vel")}
    for _ in range(count):
        q = R.q0.copy()
        q[:3] += rng.normal(0, 0.1, 3)
        qu = rng.normal(size=4)
        q[3:7] = qu / np.linalg.norm(qu)
        q[7:] += rng.normal(0, 0.2, R.nj)
        v = rng.normal(0, 0.5, R.nv)
        a = rng.normal(0, 1.0, R.nv)
        f = rng.normal(0, 50.0, 3 * len(frames))
        dq = rng.normal(0, 0.3, R.nv)
        tau = rbd.rnea_dynamics(M, frames, q, v, a, f)
        out["q"].append(q)
        out["v"].append(v)
        out["a"].append(a)
        out["f"].append(f)
        out["tau"].append(tau)
        out["aba"].append(rbd.aba_dynamics(M, frames, q, v, tau[6:], f))
        out["M"].append(rbd.crba(M, q))
        out["dq"].append(dq)
        out["q_int"].append(rbd.integrate(M, q, dq))
        out["foot_vel"].append(np.concatenate([rbd.frame_velocity(M, q, v, fid) for fid in R.foot_frames]))
    arrs = {k: np.array(v) for k, v in out.items()}
    arrs["frames"] = np.array(frames)
    arrs["mass"] = np.array(R.mass)
    np.savez_compressed(os.path.join(HERE, f"rbd_{rname}.npz"), **arrs)


def sqp_fixture(name, rname, dyn, N, B, loop_steps):
    R = robots.ROBOTS[rname]()
    R.set_gait_sequence("trot", 0.8)
    lay, P, X, XS, T0 = build_batch(R, dyn, N, B, 0)
    rec = {"P": P, "X": X, "XS": XS, "T0": T0}
    keys = ("g", "lbg", "ubg", "grad", "f", "J_indptr", "J_indices", "J_data", "dx", "x_new", "xs_next", "status",
            "iters", "accepted", "alpha", "branch", "trials", "viol_max")
    per = {k: [] for k in keys}
    for b in range(B):
        o = OracleOCP(R, dyn, N)
        x, p = X[b], P[b]
        g, lbg, ubg = o.eval_g(x, p)
        f, grad = o.f_and_grad(x, p)
        J = o.eval_J(x, p).tocsr()
        o.init_solver(x, p)
        x_new, dx, st = o.sqp_step(x, p)
        DX, _ = o.split(x_new)
        for k, v in (("g", g), ("lbg", lbg), ("ubg", ubg), ("grad", grad), ("f", f), ("J_indptr", J.indptr),
                     ("J_indices", J.indices), ("J_data", J.data), ("dx", dx), ("x_new", x_new),
                     ("xs_next", o.integrate_state(XS[b], DX[1])), ("status", st["status"]), ("iters", st["iter"]),
                     ("accepted", int(st["accepted"])), ("alpha", st["alpha"]), ("branch", st["branch"]),
                     ("trials", st["trials"]), ("viol_max", st["viol_max"])):
            per[k].append(v)
    for k, v in per.items():
        if k.startswith("J_"):
            for b, a in enumerate(v):
                rec[f"{k}_{b}"] = np.asarray(a)
        else:
            rec[k] = np.array(v)
    # closed loop of problem 0 (run_mpc.py:127-143): per step gait at t0 + k dt_min,
    # warm start, one SQP iteration, x <- integrate(x, DX[1])
    if loop_steps > 1:
        o = OracleOCP(R, dyn, N)
        xs, x = XS[0].copy(), X[0].copy()
        states, u0s = [], []
        for k in range(loop_steps):
            vals, _, _ = problem_values(R, dyn, N, 0, lay, k)
            vals["x_init"] = xs
            p = lay.pack(vals)
            if k == 0:
                o.init_solver(x, p)
            else:
                x = o.warm_start(x, p)
            x, _, _ = o.sqp_step(x, p)
            DX, U = o.split(x)
            xs = o.integrate_state(xs, DX[1])
            states.append(xs)
            u0s.append(U[0])
        rec["loop_states"] = np.array(states)
        rec["loop_u0"] = np.array(u0s)
    np.savez_compressed(os.path.join(HERE, f"sqp_{name}.npz"), **rec)
    print(name, "status", per["status"], "iters", per["iters"], flush=True)


def main():
    for r in ("go2", "b2", "b2g"):
        rbd_fixture(r)
    only = sys.argv[1:]
    for cfg in SQP_CONFIGS:
        if not only or cfg[0] in only:
            sqp_fixture(*cfg)


if __name__ == "__main__":
    main()
