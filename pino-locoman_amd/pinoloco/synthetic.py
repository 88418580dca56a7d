"""Synthetic MPC workloads.

The reference drives one robot from ``run_mpc.py:13-28`` targets (trot, period
0.8, dt_min 0.01, dt_max 0.08, swing height 0.07, swing velocity limits
[0.1, -0.2], base_vel_des = [0.2, 0, 0, 0, 0, 0]).  A batch of independent
problems is made by randomising the initial state, the gait phase and the
forward velocity target per problem, with ``numpy.random.default_rng(1234 +
global problem index)`` so a shard on rank r of G GPUs holds exactly the
problems the single-GPU run holds at the same global indices.
"""
from __future__ import annotations

import numpy as np

from .gait import horizon_dts
from .ocp import Layout, default_weights

DT_MIN, DT_MAX = 0.01, 0.08
SWING_HEIGHT = 0.07
SWING_VEL_LIMITS = (0.1, -0.2)
GAIT_PERIOD = 0.8
GRAV = 9.81


def random_state(robot, gidx, dynamics="whole_body_rnea"):
    """(x_state, t0, vx) of global problem ``gidx``.  x = [q, v]; for centroidal_vel
    x = [h, q] with the scaled momentum h = [v_base, 0.1 w_base] of the same draw."""
    rng = np.random.default_rng(1234 + gidx)
    q = robot.q0.copy()
    q[:3] += rng.normal(0.0, 0.01, 3)
    axis = rng.normal(size=3)
    axis /= np.linalg.norm(axis)
    ang = rng.uniform(0.0, 0.05)
    q[3:7] = np.concatenate([axis * np.sin(ang / 2), [np.cos(ang / 2)]])
    q[7:] = np.clip(q[7:] + rng.normal(0.0, 0.05, robot.nj), robot.joint_pos_min, robot.joint_pos_max)
    v = rng.normal(0.0, 0.1, robot.nv)
    t0 = rng.uniform(0.0, GAIT_PERIOD)
    vx = rng.uniform(0.0, 0.3)
    if dynamics == "centroidal_vel":
        return np.concatenate([v[:3], 0.1 * v[3:6], q]), t0, vx
    return np.concatenate([q, v]), t0, vx


def ext_force_target(robot, dynamics):
    """EE force target: [0, 0, -20] N for whole_body_acc, else 0."""
    if robot.ext_force_frame is None:
        return np.zeros(3)
    return np.array([0.0, 0.0, -20.0]) if dynamics == "whole_body_acc" else np.zeros(3)


def problem_values(robot, dynamics, N, gidx, lay=None, k=0):
    """Parameter values (Layout.pack keys) of problem ``gidx`` at MPC step ``k``
    (gait time t0 + k * dt_min), and its initial state."""
    lay = lay or Layout(robot, dynamics, N)
    xs, t0, vx = random_state(robot, gidx, dynamics)
    Q, Rw, W = default_weights(robot, dynamics, lay)
    contact, swing = robot.gait_sequence.get_gait_schedule(t0 + k * DT_MIN, horizon_dts(DT_MIN, DT_MAX, N), N)
    vals = dict(x_init=xs, dt_min=DT_MIN, dt_max=DT_MAX, n_contacts=robot.gait_sequence.n_contacts,
                swing_period=robot.gait_sequence.swing_period, swing_height=SWING_HEIGHT,
                swing_vel_limits=list(SWING_VEL_LIMITS), Q_diag=Q, R_diag=Rw, base_vel_des=[vx, 0, 0, 0, 0, 0],
                ext_force_des=ext_force_target(robot, dynamics), arm_vel_des=[0, 0, 0],
                tau_prev=np.zeros(robot.nj), W_diag=W, contact_schedule=contact, swing_schedule=swing)
    return vals, xs, t0


def u_des(robot, lay, n_contacts):
    """[0, f_des, 0] with f_des = 0.8 / 1.2 * m g / n_contacts front / rear
    (ocp_whole_body_rnea.py:96-106)."""
    fg = GRAV * robot.mass
    f = [0, 0, 0.8 * fg / n_contacts] * 2 + [0, 0, 1.2 * fg / n_contacts] * 2
    if robot.ext_force_frame is not None:
        f += [0, 0, 0]
    f = np.array(f, float)
    if lay.dynamics == "whole_body_aba":
        return np.concatenate([np.zeros(robot.nj), f])
    tail = [np.zeros(robot.nj)] if lay.dynamics == "whole_body_rnea" else []
    return np.concatenate([np.zeros(lay.f_idx), f] + tail)


def initial_guess(robot, lay, n_contacts):
    """Opti initial values: DX = 0, U_i = u_des truncated to nu_i (ocp.py:159-163, 193)."""
    x = np.zeros(lay.n)
    ud = u_des(robot, lay, n_contacts)
    for i in range(lay.N):
        o = lay.x_off[i] + lay.ndx
        x[o:o + lay.nu[i]] = ud[:lay.nu[i]]
    return x


def build_batch(robot, dynamics, N, B, first=0, include_base=True, include_acc=True):
    """Parameters P [B][np], initial guesses X [B][n], states XS [B][nx], gait offsets T0 [B]."""
    lay = Layout(robot, dynamics, N, include_base=include_base, include_acc=include_acc)
    P = np.zeros((B, lay.np))
    X = np.zeros((B, lay.n))
    XS = np.zeros((B, lay.nx))
    T0 = np.zeros(B)
    for b in range(B):
        vals, xs, t0 = problem_values(robot, dynamics, N, first + b, lay)
        P[b] = lay.pack(vals)
        X[b] = initial_guess(robot, lay, vals["n_contacts"])
        XS[b] = xs
        T0[b] = t0
    return lay, P, X, XS, T0


def shard(global_batch, world, rank):
    """Contiguous shard [first, first + count) of rank ``rank``."""
    base, rem = divmod(global_batch, world)
    first = rank * base + min(rank, rem)
    return first, base + (1 if rank < rem else 0)
