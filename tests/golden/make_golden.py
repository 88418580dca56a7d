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
from pinoloco.synthetic import problem_values  # noqa: E402
from oracle.osqp_ref import REFERENCE_SETTINGS  # noqa: E402
from pinoloco.gait import horizon_dts  # noqa: E402
from pinoloco.ocp import Layout, default_weights  # noqa: E402
from pinoloco.synthetic import DT_MAX, DT_MIN, SWING_HEIGHT, SWING_VEL_LIMITS, initial_guess  # noqa: E402

# Problems: ("syn", gidx) = synthetic problem gidx (pinoloco.synthetic); ("stand",) = the
# static standing equilibrium at the SRDF pose (a feasible point: violation ~1e-13);
# ("yaw", gidx, deg) = problem gidx with the base yawed by `deg` (the quaternion
# trace <= 0 branch of matrix->quaternion); ("beyond", gidx, joint, rad) = problem gidx
# with one joint `rad` past its upper limit (node-1 position bound unreachable: a
# primal-infeasible QP, NaN step, line search "didn't converge").
SYN8 = [("syn", k) for k in range(8)]
# name, robot, dynamics, N, problems, closed-loop steps of problem 0, gait, OSQP overrides, J stored for
SQP_CONFIGS = [
    ("go2_rnea_n20", "go2", "whole_body_rnea", 20, SYN8, 4, "trot", {}, 2),
    ("go2_cv_n20", "go2", "centroidal_vel", 20, SYN8, 4, "trot", {}, 2),
    ("b2_aba_n40", "b2", "whole_body_aba", 40, SYN8, 4, "trot", {}, 2),
    ("b2g_acc_n50", "b2g", "whole_body_acc", 50, SYN8, 4, "trot", {}, 1),
    ("b2g_rnea_n50", "b2g", "whole_body_rnea", 50, SYN8, 4, "trot", {}, 1),
    # edge cases of the reference's own code paths (reference settings)
    ("go2_rnea_n20_walk", "go2", "whole_body_rnea", 20, [("syn", 20), ("syn", 21), ("yaw", 22, 170.0)], 4, "walk",
     {}, 0),
    ("go2_rnea_n20_stand", "go2", "whole_body_rnea", 20, [("stand",), ("syn", 30), ("yaw", 31, -160.0)], 3, "stand",
     {}, 0),
    # OSQP termination at 25 / 50 / 75 / 100 iterations (eps 1e-2)
    ("go2_rnea_n20_eps2", "go2", "whole_body_rnea", 20, [("syn", k) for k in range(40, 48)], 1, "trot",
     {"eps_abs": 1e-2, "eps_rel": 1e-2}, 0),
    # primal-infeasible QPs (OSQP 0.6 certificate, status -3 -> NaN step -> line search
    # "didn't converge", ocp.py:478-480); detection needs more than 100 iterations
    ("go2_rnea_n20_infeas", "go2", "whole_body_rnea", 20, [("beyond", 23, 1, 10.0), ("beyond", 23, 0, 50.0),
                                                            ("syn", 24)], 1, "trot", {"max_iter": 400}, 0),
    # line-search branches 3 and 2 from the feasible standing point (tighter OSQP)
    ("go2_rnea_n20_eps5", "go2", "whole_body_rnea", 20, [("stand",)], 2, "stand",
     {"eps_abs": 1e-5, "eps_rel": 1e-5, "max_iter": 1000}, 0),
    ("go2_rnea_n20_eps6", "go2", "whole_body_rnea", 20, [("stand",)], 1, "stand",
     {"eps_abs": 1e-6, "eps_rel": 1e-6, "max_iter": 2000}, 0),
    # whole_body_acc / centroidal_acc without the base in u (ocp_whole_body_acc.py:124-135,
    # ocp_centroidal_acc.py:123-134) and centroidal_acc's gap A a + dA v - dh
    ("go2_acc_nb_n20", "go2", "whole_body_acc", 20, [("syn", k) for k in range(4)], 3, "trot", {}, 1,
     {"include_base": False}),
    ("go2_ca_n20", "go2", "centroidal_acc", 20, [("syn", k) for k in range(4)], 3, "trot", {}, 1,
     {"include_base": True}),
    ("go2_ca_nb_n20", "go2", "centroidal_acc", 20, [("syn", k) for k in range(2)], 1, "trot", {}, 1,
     {"include_base": False}),
    ("b2g_ca_n50", "b2g", "centroidal_acc", 50, [("syn", 0)], 1, "trot", {}, 1, {"include_base": True}),
    ("b2g_acc_nb_n50", "b2g", "whole_body_acc", 50, [("syn", 0)], 1, "trot", {}, 1, {"include_base": False}),
    # centroidal_vel without the base velocity in u (the OCPCentroidalVel default,
    # ocp_centroidal_vel.py:9-23, 119-129): v_b = A_b^-1 (m h - A_j v_j) inside the rows
    ("go2_cv_nb_n20", "go2", "centroidal_vel", 20, [("syn", k) for k in range(4)], 3, "trot", {}, 2,
     {"include_base": False}),
    # B2G centroidal_vel (ndx = 30: the factor sweeps with a 2-row identity pad)
    ("b2g_cv_n50", "b2g", "centroidal_vel", 50, [("syn", k) for k in range(4)], 3, "trot", {}, 1),
    # whole_body_rnea with finite-difference accelerations (include_acc = False,
    # ocp_whole_body_rnea.py:21-26, 157-159, 183-191): the RNEA rows of node i read dv_{i+1}
    ("go2_rnea_fd_n20", "go2", "whole_body_rnea", 20, [("syn", k) for k in range(4)] + [("stand",)], 3, "trot", {},
     2, {"include_acc": False}),
    ("b2g_rnea_fd_n50", "b2g", "whole_body_rnea", 50, [("syn", 0), ("syn", 1)], 1, "trot", {}, 1,
     {"include_acc": False}),
]

# Interior-point (Fatrop branch) fixtures: name, robot, dynamics, N, problems, closed-loop
# steps of problem 0, gait (oracle/ip_ref.py, reference settings ocp.py:254-262)
IP_CONFIGS = [
    ("ip_go2_rnea_n20", "go2", "whole_body_rnea", 20, [("syn", k) for k in range(4)], 3, "trot"),
    ("ip_go2_rnea_n20_stand", "go2", "whole_body_rnea", 20, [("stand",), ("syn", 30)], 2, "stand"),
    ("ip_go2_cv_n20", "go2", "centroidal_vel", 20, [("syn", 0), ("syn", 1)], 0, "trot"),
    ("ip_b2_aba_n40", "b2", "whole_body_aba", 40, [("syn", 0)], 0, "trot"),
    # the headline shapes: eight problems of the benchmark batch each (build_batch(..., 0) =
    # ("syn", k)), cold first solves: all stop at the iteration cap (status -1); the failed
    # line searches (-2) of the benchmark come at warm-started steps (IP_WARM_CONFIGS)
    ("ip_b2g_acc_n50", "b2g", "whole_body_acc", 50, [("syn", k) for k in (0, 1, 2, 7, 23, 29, 39, 43)], 0, "trot"),
    ("ip_b2g_rnea_n50", "b2g", "whole_body_rnea", 50, [("syn", k) for k in (0, 1, 2, 7, 10, 19, 44, 47)], 0, "trot"),
    # centroidal_vel from the feasible standing point (a well-conditioned trajectory beside the
    # chaotic cold starts of ip_go2_cv_n20), and the variants without the base in u and
    # centroidal_acc, each with a standing and a synthetic problem
    ("ip_go2_cv_n20_stand", "go2", "centroidal_vel", 20, [("stand",), ("syn", 2)], 0, "stand"),
    ("ip_go2_cv_nb_n20", "go2", "centroidal_vel", 20, [("stand",), ("syn", 2)], 0, "stand", {"include_base": False}),
    ("ip_go2_ca_n20", "go2", "centroidal_acc", 20, [("stand",), ("syn", 0)], 0, "stand", {"include_base": True}),
    ("ip_go2_acc_nb_n20", "go2", "whole_body_acc", 20, [("stand",), ("syn", 0)], 0, "stand",
     {"include_base": False}),
]


def _yaw_quat(deg):
    a = np.deg2rad(deg)
    return np.array([0.0, 0.0, np.sin(a / 2), np.cos(a / 2)])


def make_problem(R, lay, dyn, N, spec):
    """(p, x, x_state, t0) of one problem spec (see SQP_CONFIGS)."""
    kind = spec[0]
    if kind == "stand":
        Q, Rw, W = default_weights(R, dyn, lay)
        contact, swing = R.gait_sequence.get_gait_schedule(0.0, horizon_dts(DT_MIN, DT_MAX, N), N)
        xs = np.concatenate([R.q0, np.zeros(R.nv)])
        vals = dict(x_init=xs, dt_min=DT_MIN, dt_max=DT_MAX, n_contacts=R.gait_sequence.n_contacts,
                    swing_period=R.gait_sequence.swing_period, swing_height=SWING_HEIGHT,
                    swing_vel_limits=list(SWING_VEL_LIMITS), Q_diag=Q, R_diag=Rw, base_vel_des=np.zeros(6),
                    ext_force_des=np.zeros(3), arm_vel_des=np.zeros(3), tau_prev=np.zeros(R.nj), W_diag=W,
                    contact_schedule=contact, swing_schedule=swing)
        # contact forces balancing the gravity wrench (RNEA base rows = 0), joint torques
        # from RNEA: every row of the OCP holds to round-off
        M = rbd.ModelArrays(R.model)
        frames = list(R.foot_frames)
        z = np.zeros(R.nv)
        base = rbd.rnea_dynamics(M, frames, R.q0, z, z, np.zeros(12))
        Jb = np.stack([rbd.rnea_dynamics(M, frames, R.q0, z, z, np.eye(12)[k])[:6] - base[:6] for k in range(12)], 1)
        f = np.linalg.lstsq(Jb, -base[:6], rcond=None)[0]
        tau = rbd.rnea_dynamics(M, frames, R.q0, z, z, f)
        x = np.zeros(lay.n)
        for i in range(N):
            o = lay.x_off[i] + lay.ndx
            if dyn == "whole_body_rnea":
                u = np.concatenate([np.zeros(lay.na), f] + ([tau[6:]] if i < lay.tau_nodes else []))
            elif dyn == "whole_body_aba":  # u = [tau_j, f]
                u = np.concatenate([tau[6:], f])
            else:  # acc / centroidal families: zero accelerations / velocities, the same forces
                u = np.concatenate([np.zeros(lay.f_idx), f])
            x[o:o + lay.nu[i]] = u
        if dyn == "centroidal_vel":  # x = [h, q]: zero momentum
            xs = np.concatenate([np.zeros(6), R.q0])
            vals["x_init"] = xs
        return lay.pack(vals), x, xs, 0.0
    gidx = spec[1]
    vals, xs, t0 = problem_values(R, dyn, N, gidx, lay)
    xs = xs.copy()
    qo = 6 if dyn == "centroidal_vel" else 0
    if kind == "yaw":
        xs[qo + 3:qo + 7] = _yaw_quat(spec[2])
    elif kind == "beyond":
        xs[qo + 7 + spec[2]] = R.joint_pos_max[spec[2]] + spec[3]
    vals["x_init"] = xs
    return lay.pack(vals), initial_guess(R, lay, vals["n_contacts"]), xs, t0


def rbd_fixture(rname, seed=7, count=3):
    R = robots.ROBOTS[rname]()
    R.set_gait_sequence("trot", 0.8)
    M = rbd.ModelArrays(R.model)
    rng = np.random.default_rng(seed)
    frames = list(R.foot_frames) + ([R.ext_force_frame] if R.ext_force_frame is not None else [])
    out = {k: [] for k in ("q", "v", "a", "f", "tau", "aba", "M", "dq", "q_int", "foot_vel", "h", "a_j", "v_j",
                           "foot_pos", "foot_jac0", "nle", "com", "hg", "cmap", "com_dyn", "gaps_cv", "base_vel_cv",
                           "base_acc_cv", "base_acc_wb", "gaps_wb", "arm_vel_rel")}
    rng2 = np.random.default_rng(seed + 100)  # draws of the Dynamics-surface fixtures (the originals stay put)
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
        # Dynamics plugin surface (dynamics/*.py factories, pinoloco/dynamics.py)
        h = rng2.normal(0, 0.3, 6)
        a_j = rng2.normal(0, 1.0, R.nj)
        v_j = rng2.normal(0, 0.5, R.nj)
        _, oM = rbd.forward_kinematics(M, q)
        out["h"].append(h)
        out["a_j"].append(a_j)
        out["v_j"].append(v_j)
        out["foot_pos"].append(np.concatenate([rbd.frame_placement(M, oM, fid)[1] for fid in R.foot_frames]))
        out["foot_jac0"].append(rbd.frame_jacobian_lwa(M, q, R.foot_frames[0]))
        out["nle"].append(rbd.rnea(M, q, v, np.zeros(R.nv)))
        out["com"].append(rbd.center_of_mass(M, q))
        out["hg"].append(rbd.centroidal_momentum(M, q, v))
        out["cmap"].append(rbd.centroidal_map(M, q))
        out["com_dyn"].append(rbd.com_dynamics(M, frames, q, f, R.mass))
        out["gaps_cv"].append(rbd.centroidal_momentum(M, q, v) - R.mass * h)
        out["base_vel_cv"].append(rbd.base_vel_cv(M, h, q, v_j, R.mass))
        out["base_acc_cv"].append(rbd.base_acc_cv(M, frames, q, v, a_j, f, R.mass))
        out["base_acc_wb"].append(rbd.base_acc_wb(M, frames, q, v, a_j, f))
        out["gaps_wb"].append(tau[:6])
        base_fid = R.model.get_frame_id("base_link")
        out["arm_vel_rel"].append(rbd.frame_velocity(M, q, v, R.arm_ee_frame, True, base_fid)
                                  if R.arm_ee_frame is not None else np.zeros(6))
    arrs = {k: np.array(v) for k, v in out.items()}
    arrs["frames"] = np.array(frames)
    arrs["mass"] = np.array(R.mass)
    np.savez_compressed(os.path.join(HERE, f"rbd_{rname}.npz"), **arrs)


def sqp_fixture(name, rname, dyn, N, problems, loop_steps, gait, osqp, njac, kw=None):
    kw = kw or {}
    R = robots.ROBOTS[rname]()
    R.set_gait_sequence(gait, 0.8)
    lay = Layout(R, dyn, N, **kw)
    settings = dict(REFERENCE_SETTINGS)
    settings.update(osqp)
    B = len(problems)
    P, X, XS, T0 = (np.zeros((B, lay.np)), np.zeros((B, lay.n)), np.zeros((B, lay.nx)), np.zeros(B))
    for b, spec in enumerate(problems):
        P[b], X[b], XS[b], T0[b] = make_problem(R, lay, dyn, N, spec)
    rec = {"P": P, "X": X, "XS": XS, "T0": T0, "gait": np.array(gait), "kinds": np.array([s[0] for s in problems]),
           "osqp_eps": np.array([settings["eps_abs"], settings["eps_rel"]]), "osqp_max_iter": settings["max_iter"],
           "include_base": int(kw.get("include_base", True)), "include_acc": int(kw.get("include_acc", True))}
    keys = ("g", "lbg", "ubg", "grad", "f", "J_indptr", "J_indices", "J_data", "dx", "x_new", "xs_next", "status",
            "iters", "accepted", "alpha", "branch", "trials", "viol_max", "quat_trace_le0")
    per = {k: [] for k in keys}
    for b in range(B):
        o = OracleOCP(R, dyn, N, osqp_settings=settings, **kw)
        x, p = X[b], P[b]
        g, lbg, ubg = o.eval_g(x, p)
        f, grad = o.f_and_grad(x, p)
        J = o.eval_J(x, p).tocsr()
        o.init_solver(x, p)
        x_new, dx, st = o.sqp_step(x, p)
        DX, _ = o.split(x_new)
        qo = 6 if dyn == "centroidal_vel" else 0
        Rq = rbd.quat_to_matrix(XS[b][qo + 3:qo + 7])
        for k, v in (("g", g), ("lbg", lbg), ("ubg", ubg), ("grad", grad), ("f", f), ("J_indptr", J.indptr),
                     ("J_indices", J.indices), ("J_data", J.data), ("dx", dx), ("x_new", x_new),
                     ("xs_next", o.integrate_state(XS[b], DX[1])), ("status", st["status"]), ("iters", st["iter"]),
                     ("accepted", int(st["accepted"])), ("alpha", st["alpha"]), ("branch", st["branch"]),
                     ("trials", st["trials"]), ("viol_max", st["viol_max"]),
                     ("quat_trace_le0", int(np.trace(Rq) <= 0))):
            per[k].append(v)
    for k, v in per.items():
        if k.startswith("J_"):
            for b, a in enumerate(v[:njac]):
                rec[f"{k}_{b}"] = np.asarray(a)
        else:
            rec[k] = np.array(v)
    # closed loop of problem 0 (run_mpc.py:127-143): per step gait at t0 + k dt_min,
    # warm start, one SQP iteration, x <- integrate(x, DX[1]); per-step solver stats
    if loop_steps > 1:
        o = OracleOCP(R, dyn, N, osqp_settings=settings, **kw)
        xs, x = XS[0].copy(), X[0].copy()
        states, u0s, lst = [], [], []
        for k in range(loop_steps):
            p = P[0].copy()
            contact, swing = R.gait_sequence.get_gait_schedule(T0[0] + k * DT_MIN, horizon_dts(DT_MIN, DT_MAX, N), N)
            vals = {"x_init": xs, "contact_schedule": contact, "swing_schedule": swing}
            for key in vals:
                o_, s_ = lay.poff[key]
                p[o_:o_ + s_] = lay.pack(vals)[o_:o_ + s_]
            if k == 0:
                o.init_solver(x, p)
            else:
                x = o.warm_start(x, p)
            x, _, st = o.sqp_step(x, p)
            DX, U = o.split(x)
            xs = o.integrate_state(xs, DX[1])
            states.append(xs)
            u0s.append(U[0])
            lst.append([st["status"], st["iter"], st["branch"], st["trials"]])
        rec["loop_states"] = np.array(states)
        rec["loop_u0"] = np.array(u0s)
        rec["loop_stats"] = np.array(lst)
    np.savez_compressed(os.path.join(HERE, f"sqp_{name}.npz"), **rec)
    print(name, "status", per["status"], "iters", per["iters"], "branch", per["branch"], "trials", per["trials"],
          flush=True)


# (fixture, problem) whose per-iteration oracle states and Newton directions are stored for
# the GPU's teacher-forced directions (tests/test_ip.py); problems of ip_go2_rnea_n20 also
# get a lam_g warm-started solve from their own solution
IP_TF = {("ip_go2_cv_n20", 0), ("ip_go2_cv_n20", 1), ("ip_go2_rnea_n20", 0), ("ip_go2_acc_nb_n20", 1)}
IP_WARM = {"ip_go2_rnea_n20": 2}


def _ip_one(args):
    """One problem of an IP fixture (a worker process): the oracle's solve, its trace and,
    for problem 0, the Lagrangian Hessian at the solution."""
    from oracle.ip_ref import IPRef
    name, rname, dyn, N, gait, kw, b, x0, p = args
    R = robots.ROBOTS[rname]()
    R.set_gait_sequence(gait, 0.8)
    o = OracleOCP(R, dyn, N, **kw)
    ip = IPRef(o)
    x, lam, st = ip.solve(x0, p)
    out = dict(x=x, lam=lam, st=st, trace=ip.trace if (name, b) in IP_TF else None)
    if b == 0:
        out["hess"] = o.lag_hess(x, p, lam).tocsr()
    if b < IP_WARM.get(name, 0):
        out["warm"] = IPRef(o).solve(x, p, lam0=lam)
    g, lbg, ubg = o.eval_g(x, p)
    out["viol_max"] = o.violation_max(g, lbg, ubg)
    print(f"  {name} problem {b}: status {st['status']} iter {st['iter']}", flush=True)
    return out


def ip_fixture(name, rname, dyn, N, problems, loop_steps, gait, kw=None):
    from concurrent.futures import ProcessPoolExecutor
    from oracle.ip_ref import IP_SETTINGS, IPRef
    kw = kw or {}
    R = robots.ROBOTS[rname]()
    R.set_gait_sequence(gait, 0.8)
    lay = Layout(R, dyn, N, **kw)
    B = len(problems)
    P, X, XS, T0 = (np.zeros((B, lay.np)), np.zeros((B, lay.n)), np.zeros((B, lay.nx)), np.zeros(B))
    for b, spec in enumerate(problems):
        P[b], X[b], XS[b], T0[b] = make_problem(R, lay, dyn, N, spec)
    mi = IP_SETTINGS["max_iter"]
    rec = {"P": P, "X": X, "XS": XS, "T0": T0, "gait": np.array(gait), "kinds": np.array([s[0] for s in problems]),
           "include_base": int(kw.get("include_base", True))}
    per = {k: [] for k in ("x_out", "lam", "s", "zl", "zu", "status", "iter", "err", "mu", "f", "alphas", "trials",
                           "viol_max")}
    jobs = [(name, rname, dyn, N, gait, kw, b, X[b], P[b]) for b in range(B)]
    workers = min(B, int(os.environ.get("GOLDEN_WORKERS", "8")))
    if workers > 1:
        with ProcessPoolExecutor(workers) as ex:
            res = list(ex.map(_ip_one, jobs))
    else:
        res = [_ip_one(j) for j in jobs]
    for b, r in enumerate(res):
        x, lam, st = r["x"], r["lam"], r["st"]
        if r["trace"] is not None:
            for key in ("x", "s", "lam", "zl", "zu", "dx", "dl", "ds"):
                rec[f"tf{b}_{key}"] = np.array([t[key] for t in r["trace"]])
            for key in ("mu", "amax", "az", "dw_last", "dwi"):
                rec[f"tf{b}_{key}"] = np.array([float(t[key]) for t in r["trace"]])
        if "hess" in r:  # the Lagrangian Hessian at the solution (GPU k_lag_hess vs OracleOCP.lag_hess)
            Hl = r["hess"]
            rec["hess_data"], rec["hess_indices"], rec["hess_indptr"] = Hl.data, Hl.indices, Hl.indptr
        if "warm" in r:
            xw, lw, sw = r["warm"]
            for key, v in (("warm_x", xw), ("warm_lam", lw), ("warm_status", sw["status"]), ("warm_iter", sw["iter"])):
                rec.setdefault(key, []).append(v)
        al = np.zeros(mi)
        al[:len(st["alphas"])] = st["alphas"]
        for k, v in (("x_out", x), ("lam", lam), ("s", st["s"]), ("zl", st["zl"]), ("zu", st["zu"]),
                     ("status", st["status"]), ("iter", st["iter"]), ("err", st["err"]), ("mu", st["mu"]),
                     ("f", st["f"]), ("alphas", al), ("trials", int(np.sum(st["trials"]))),
                     ("viol_max", r["viol_max"])):
            per[k].append(v)
    rec.update({k: np.array(v) for k, v in per.items()})
    for key in ("warm_x", "warm_lam", "warm_status", "warm_iter"):
        if key in rec:
            rec[key] = np.array(rec[key])
    # closed loop of problem 0 (run_mpc.py:115-143 with the Fatrop solver): warm start,
    # one interior-point solve, x <- integrate(x, DX[1])
    if loop_steps > 1:
        o = OracleOCP(R, dyn, N, **kw)
        xs, x = XS[0].copy(), X[0].copy()
        states, stl = [], []
        lam_prev = None
        for k in range(loop_steps):
            p = P[0].copy()
            contact, swing = R.gait_sequence.get_gait_schedule(T0[0] + k * DT_MIN, horizon_dts(DT_MIN, DT_MAX, N), N)
            vals = {"x_init": xs, "contact_schedule": contact, "swing_schedule": swing}
            for key in vals:
                o_, s_ = lay.poff[key]
                p[o_:o_ + s_] = lay.pack(vals)[o_:o_ + s_]
            if k > 0:
                x = o.warm_start(x, p)
            # lam_g carried across solves (ocp_whole_body_rnea.py:234-235, ocp.py:373)
            x, lam_prev, st = IPRef(o).solve(x, p, lam0=lam_prev)
            DX, _ = o.split(x)
            xs = o.integrate_state(xs, DX[1])
            states.append(xs)
            stl.append([st["status"], st["iter"]])
        rec["loop_states"] = np.array(states)
        rec["loop_stats"] = np.array(stl)
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **rec)
    print(name, "status", per["status"], "iter", per["iter"], "err", np.round(per["err"], 4), flush=True)


def ip_compiled_fixture(steps=3):
    """The reference's default driver: run_mpc.py with solver = "fatrop", compile_solver =
    True, warm_start = True (run_mpc.py:13-37, 50-113): B2G standing_with_arm_up,
    whole_body_rnea, nodes 14, trot 0.8, x_init = x_nom.  Per step k: gait at k dt_min,
    the OCP warm start as the compiled function's x_warm_start, tau_prev = tau_j of node 1
    of the previous solution, one interior-point solve with cold multipliers (the compiled
    function has no lam_g input), x_init <- integrate(x_init, DX[1])."""
    from oracle.ip_ref import IPRef
    from pinoloco.synthetic import initial_guess
    R = robots.ROBOTS["b2g"]()
    R.set_gait_sequence("trot", 0.8)
    N = 14
    dyn = "whole_body_rnea"
    lay = Layout(R, dyn, N)
    o = OracleOCP(R, dyn, N)
    Q, Rw, W = default_weights(R, dyn, lay)
    x_init = np.concatenate([R.q0, np.zeros(R.nv)])
    tau_prev = np.zeros(R.nj)
    x = None
    rec = {k: [] for k in ("P", "X0", "x_out", "lam", "status", "iter", "alphas", "x_init_next")}
    for k in range(steps):
        contact, swing = R.gait_sequence.get_gait_schedule(k * DT_MIN, horizon_dts(DT_MIN, DT_MAX, N), N)
        vals = dict(x_init=x_init, dt_min=DT_MIN, dt_max=DT_MAX, contact_schedule=contact, swing_schedule=swing,
                    n_contacts=R.gait_sequence.n_contacts, swing_period=R.gait_sequence.swing_period,
                    swing_height=SWING_HEIGHT, swing_vel_limits=list(SWING_VEL_LIMITS), Q_diag=Q, R_diag=Rw,
                    base_vel_des=[0.2, 0, 0, 0, 0, 0], ext_force_des=np.zeros(3), arm_vel_des=np.zeros(3),
                    tau_prev=tau_prev, W_diag=W)
        p = lay.pack(vals)
        x0 = initial_guess(R, lay, vals["n_contacts"]) if x is None else o.warm_start(x, p)
        x, lam, st = IPRef(o).solve(x0, p)
        DX, U = o.split(x)
        x_init = o.integrate_state(x_init, DX[1])
        tau_prev = U[1][lay.tau_idx:].copy()
        al = np.zeros(10)
        al[:len(st["alphas"])] = st["alphas"]
        for key, v in (("P", p), ("X0", x0), ("x_out", x), ("lam", lam), ("status", st["status"]),
                       ("iter", st["iter"]), ("alphas", al), ("x_init_next", x_init)):
            rec[key].append(v)
        print(f"  compiled step {k}: status {st['status']} iter {st['iter']}", flush=True)
    np.savez_compressed(os.path.join(HERE, "ip_b2g_rnea_n14_compiled.npz"), **{k: np.array(v) for k, v in rec.items()})


# Warm-started interior-point solves of the benchmark loop (bench.py --solver fatrop): the cold
# first solves of the batch never fail the filter line search, the -2 exits come at MPC steps
# >= 2 (tools/gpu_ip_screen.py).  Problems of the benchmark batch ("syn" k), chosen from that
# screen: five that fail at step 2 and three that stop at the iteration cap.
IP_WARM_CONFIGS = [
    ("ip_b2g_rnea_n50_warm", "whole_body_rnea", [1, 8, 11, 14, 17, 0, 2, 3]),
    ("ip_b2g_acc_n50_warm", "whole_body_acc", [8, 11, 14, 17, 21, 0, 1, 2]),
]


def _ip_warm_one(args):
    """Steps 0 and 1 of the problem's MPC loop with the compiled restatement (oracle/cpu, the
    oracle's algorithm to <= 3e-12 on these shapes), then step 2 -- the fixture -- with the numpy
    oracle from the loop's warm start (x: OracleOCP.warm_start of step 1's solution; lam_g:
    step 1's multipliers, ocp_whole_body_rnea.py:207-235, ocp.py:373)."""
    from oracle.cpu_baseline import CpuOCP
    from oracle.ip_ref import IPRef
    dyn, gidx = args
    R = robots.ROBOTS["b2g"]()
    R.set_gait_sequence("trot", 0.8)
    N = 50
    lay = Layout(R, dyn, N)
    o = OracleOCP(R, dyn, N)
    c = CpuOCP(R, dyn, N)
    p, x, xs, t0 = make_problem(R, lay, dyn, N, ("syn", gidx))
    lam = None
    pre = []
    for k in range(3):
        if k > 0:
            contact, swing = R.gait_sequence.get_gait_schedule(t0 + k * DT_MIN, horizon_dts(DT_MIN, DT_MAX, N), N)
            vals = {"x_init": xs, "contact_schedule": contact, "swing_schedule": swing}
            for key in vals:
                o_, s_ = lay.poff[key]
                p[o_:o_ + s_] = lay.pack(vals)[o_:o_ + s_]
            x = o.warm_start(x, p)
        if k == 2:
            break
        x, lam, st = c.ip_solve(x, p, lam0=lam)
        pre.append([st["status"], st["iter"]])
        DX, _ = o.split(x)
        xs = o.integrate_state(xs, DX[1])
    ip = IPRef(o)
    xo, lo, st = ip.solve(x, p, lam0=lam)
    print(f"  {dyn} syn {gidx}: steps 0-1 {pre}, step 2 status {st['status']} iter {st['iter']}", flush=True)
    return dict(P=p.copy(), X=x.copy(), LAM0=np.array(lam), XS=xs.copy(), x_out=xo, lam=lo, st=st, pre=pre)


def ip_warm_fixture(name, dyn, gidx):
    from concurrent.futures import ProcessPoolExecutor
    from oracle.ip_ref import IP_SETTINGS
    workers = min(len(gidx), int(os.environ.get("GOLDEN_WORKERS", "8")))
    with ProcessPoolExecutor(workers) as ex:
        res = list(ex.map(_ip_warm_one, [(dyn, g) for g in gidx]))
    mi = IP_SETTINGS["max_iter"]
    rec = {"gidx": np.array(gidx), "step": 2, "gait": np.array("trot"), "include_base": 1}
    for key in ("P", "X", "LAM0", "XS", "x_out", "lam"):
        rec[key] = np.array([r[key] for r in res])
    for key in ("status", "iter", "err", "mu", "f"):
        rec[key] = np.array([r["st"][key] for r in res])
    for key in ("s", "zl", "zu"):
        rec[key] = np.array([r["st"][key] for r in res])
    al = np.zeros((len(res), mi))
    for b, r in enumerate(res):
        al[b, :len(r["st"]["alphas"])] = r["st"]["alphas"]
    rec["alphas"] = al
    rec["trials"] = np.array([int(np.sum(r["st"]["trials"])) for r in res])
    rec["pre_stats"] = np.array([r["pre"] for r in res])
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **rec)
    print(name, "status", rec["status"], "iter", rec["iter"], flush=True)


# Closed loops over every MPC step the benchmark runs (bench.py --warmup 5 --steps 20: steps
# 0-24) for problems of the benchmark batch (build_batch(..., 0) = ("syn", gidx)): per step the
# gait at t0 + k dt_min, x_init, the OCP warm start, one SQP iteration, x <- integrate(x, DX[1])
# (run_mpc.py:127-143).  tests/test_gpu.py checks these problems inside the B = 1024 / 256 batch.
# The aba loop also stores the trajectory of the reduced-form oracle (oracle/osqp_ref.py
# kkt="reduced_block": the GPU's algebra -- the reduced SPD system with block inverses -- in
# numpy): whole_body_aba's closed loop amplifies the two formulations' ~1e-9 per-step difference
# to ~1e-6 over 25 steps (tests/test_gpu.py LOOP_BENCH_TOL).
LOOP_CONFIGS = [
    ("loop_b2g_rnea_n50", "b2g", "whole_body_rnea", 50, [0, 1, 2, 3], 25),
    ("loop_b2g_acc_n50", "b2g", "whole_body_acc", 50, [0, 1, 2, 3], 25),
    ("loop_b2_aba_n40", "b2", "whole_body_aba", 40, [0, 1, 2, 3], 25, True),
]


def _loop_one(args):
    rname, dyn, N, gidx, steps, kkt = args
    R = robots.ROBOTS[rname]()
    R.set_gait_sequence("trot", 0.8)
    lay = Layout(R, dyn, N)
    o = OracleOCP(R, dyn, N, kkt=kkt)
    P0, X0, XS0, t0 = make_problem(R, lay, dyn, N, ("syn", gidx))
    xs, x = XS0.copy(), X0.copy()
    states, u0s, lst = [], [], []
    for k in range(steps):
        p = P0.copy()
        contact, swing = R.gait_sequence.get_gait_schedule(t0 + k * DT_MIN, horizon_dts(DT_MIN, DT_MAX, N), N)
        vals = {"x_init": xs, "contact_schedule": contact, "swing_schedule": swing}
        for key in vals:
            o_, s_ = lay.poff[key]
            p[o_:o_ + s_] = lay.pack(vals)[o_:o_ + s_]
        if k == 0:
            o.init_solver(x, p)
        else:
            x = o.warm_start(x, p)
        x, _, st = o.sqp_step(x, p)
        DX, U = o.split(x)
        xs = o.integrate_state(xs, DX[1])
        states.append(xs)
        u0s.append(U[0])
        lst.append([st["status"], st["iter"], st["branch"], st["trials"]])
    print(f"  {dyn} syn {gidx}: status {[s[0] for s in lst]}", flush=True)
    return dict(P=P0, X=X0, XS=XS0, T0=t0, states=np.array(states), u0=np.array(u0s), stats=np.array(lst))


def loop_fixture(name, rname, dyn, N, gidx, steps, reduced=False):
    from concurrent.futures import ProcessPoolExecutor
    workers = min(len(gidx), int(os.environ.get("GOLDEN_WORKERS", "4")))
    with ProcessPoolExecutor(workers) as ex:
        res = list(ex.map(_loop_one, [(rname, dyn, N, g, steps, "quasi_definite") for g in gidx]))
        red = list(ex.map(_loop_one, [(rname, dyn, N, g, steps, "reduced_block") for g in gidx])) if reduced else None
    rec = {"gidx": np.array(gidx), "gait": np.array("trot")}
    for key, out in (("P", "P"), ("X", "X"), ("XS", "XS"), ("T0", "T0"), ("states", "loop_states"),
                     ("u0", "loop_u0"), ("stats", "loop_stats")):
        rec[out] = np.array([r[key] for r in res])
    if red is not None:
        rec["loop_states_reduced"] = np.array([r["states"] for r in red])
        rec["loop_stats_reduced"] = np.array([r["stats"] for r in red])
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **rec)
    print(name, "statuses", sorted(set(rec["loop_stats"][:, :, 0].ravel().tolist())), flush=True)


# Interior-point closed loops of the reference's default driver (solver "fatrop", compile_solver
# = True, warm_start = True: run_mpc.py:34-37, 50-111): per step the gait at t0 + k dt_min,
# x_init, the OCP's primal warm start, one interior-point solve from COLD multipliers (the
# compiled solver function takes x only, ocp_whole_body_rnea.py:239-257), x <- integrate(x,
# DX[1]).  Problems of the benchmark batch (build_batch(..., 0) = ("syn", gidx)).  Go2 with the
# numpy oracle; the B2G headline shape with the compiled restatement oracle/cpu (the numpy
# oracle's algorithm to <= 3e-12 on these shapes, tests/test_cpu_baseline.py; a numpy B2G solve
# takes ~15 min), its first step checked against the numpy fixture ip_b2g_rnea_n50 by
# tests/test_ip.py.
IP_LOOP_CONFIGS = [
    ("ip_loop_go2_rnea_n20", "go2", "whole_body_rnea", 20, [0, 1, 2, 3], 5, "numpy"),
    ("ip_loop_b2g_rnea_n50", "b2g", "whole_body_rnea", 50, [0, 1, 2, 3], 10, "cpu"),
]


def _ip_loop_one(args):
    rname, dyn, N, gidx, steps, engine = args
    from oracle.ip_ref import IPRef
    R = robots.ROBOTS[rname]()
    R.set_gait_sequence("trot", 0.8)
    lay = Layout(R, dyn, N)
    o = OracleOCP(R, dyn, N)
    if engine == "cpu":
        from oracle.cpu_baseline import CpuOCP
        c = CpuOCP(R, dyn, N)
        solve = lambda x_, p_: c.ip_solve(x_, p_)  # noqa: E731
    else:
        solve = lambda x_, p_: IPRef(o).solve(x_, p_)  # noqa: E731
    P0, X0, XS0, t0 = make_problem(R, lay, dyn, N, ("syn", gidx))
    xs, x, p = XS0.copy(), X0.copy(), P0.copy()
    states, stl, xo = [], [], []
    for k in range(steps):
        if k > 0:
            contact, swing = R.gait_sequence.get_gait_schedule(t0 + k * DT_MIN, horizon_dts(DT_MIN, DT_MAX, N), N)
            vals = {"x_init": xs, "contact_schedule": contact, "swing_schedule": swing}
            for key in vals:
                o_, s_ = lay.poff[key]
                p[o_:o_ + s_] = lay.pack(vals)[o_:o_ + s_]
            x = o.warm_start(x, p)
        x, _, st = solve(x, p)
        DX, _ = o.split(x)
        xs = o.integrate_state(xs, DX[1])
        states.append(xs)
        stl.append([st["status"], st["iter"]])
        xo.append(x.copy())
    print(f"  {dyn} syn {gidx}: {stl}", flush=True)
    return dict(P=P0, X=X0, XS=XS0, T0=t0, states=np.array(states), stats=np.array(stl), x_out=np.array(xo))


def ip_loop_fixture(name, rname, dyn, N, gidx, steps, engine):
    from concurrent.futures import ProcessPoolExecutor
    workers = min(len(gidx), int(os.environ.get("GOLDEN_WORKERS", "4")))
    with ProcessPoolExecutor(workers) as ex:
        res = list(ex.map(_ip_loop_one, [(rname, dyn, N, g, steps, engine) for g in gidx]))
    rec = {"gidx": np.array(gidx), "gait": np.array("trot"), "engine": np.array(engine)}
    for key, out in (("P", "P"), ("X", "X"), ("XS", "XS"), ("T0", "T0"), ("states", "loop_states"),
                     ("stats", "loop_stats"), ("x_out", "loop_x")):
        rec[out] = np.array([r[key] for r in res])
    np.savez_compressed(os.path.join(HERE, f"{name}.npz"), **rec)
    print(name, "statuses", sorted(set(rec["loop_stats"][:, :, 0].ravel().tolist())), flush=True)


def main():
    only = sys.argv[1:]
    for cfg in IP_LOOP_CONFIGS:
        if cfg[0] in only:
            ip_loop_fixture(*cfg)
    for cfg in LOOP_CONFIGS:
        if cfg[0] in only:
            loop_fixture(*cfg)
    if only and all(o.startswith("loop_") or o.startswith("ip_loop_") for o in only):
        return
    for cfg in IP_WARM_CONFIGS:
        if cfg[0] in only:
            ip_warm_fixture(*cfg)
    if "ip_b2g_rnea_n14_compiled" in only:
        ip_compiled_fixture()
    for cfg in IP_CONFIGS:
        if cfg[0] in only:
            ip_fixture(*cfg)
    if only and all(o.startswith("ip_") for o in only):
        return
    if not only or "rbd" in only:
        for r in ("go2", "b2", "b2g"):
            rbd_fixture(r)
    for cfg in SQP_CONFIGS:
        if not only or cfg[0] in only:
            sqp_fixture(*cfg)


if __name__ == "__main__":
    main()
