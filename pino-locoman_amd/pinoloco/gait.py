"""Gait tables and swing-height spline.

Restates ``utils/gait_sequence.py`` of the reference:
``GaitSequence`` (``:5-77``), ``get_spline_vel_z`` (``:96-107``) and the OCS2
``CubicSpline`` (``:110-133``).  The schedule is host work done once per MPC
step; the spline is evaluated again inside the HIP row kernels
(``csrc/rows.h``) on the same parameters.
"""
from __future__ import annotations

import numpy as np

FEET = ["FR_foot", "FL_foot", "RR_foot", "RL_foot"]  # gait_sequence.py:7


class GaitSequence:
    def __init__(self, gait_type="trot", gait_period=0.5):
        self.feet = list(FEET)
        self.gait_type = gait_type
        self.gait_period = gait_period
        if gait_type == "trot":
            self.n_contacts = 2
            self.swing_period = 0.5 * gait_period
        elif gait_type == "walk":
            self.n_contacts = 3
            self.swing_period = 0.25 * gait_period
        elif gait_type == "stand":
            self.n_contacts = 4
            self.swing_period = gait_period
        else:
            raise ValueError(f"Gait: {gait_type} not supported")

    def get_gait_schedule(self, t_current, dts, nodes):
        """Contact (0/1) and swing phase (0..1) over the horizon (gait_sequence.py:26-77)."""
        contact = np.ones((4, nodes))
        swing = np.zeros((4, nodes))
        if self.gait_type in ("trot", "walk"):
            t = t_current
            for i in range(nodes):
                if i > 0:
                    t += dts[i - 1]
                gait_phase = t % self.gait_period / self.gait_period
                swing_phase = t % self.swing_period / self.swing_period
                if self.gait_type == "trot":
                    feet = (0, 3) if gait_phase < 0.5 else (1, 2)
                else:
                    feet = (1,) if gait_phase < 0.25 else (2,) if gait_phase < 0.5 else \
                        (0,) if gait_phase < 0.75 else (3,)
                for f in feet:
                    contact[f, i] = 0
                    swing[f, i] = swing_phase
        return contact, swing


class CubicSpline:
    """OCS2 cubic spline (gait_sequence.py:110-133)."""

    def __init__(self, t0, t1, pos0, vel0, pos1, vel1):
        self.t0, self.t1 = t0, t1
        self.dt = t1 - t0
        dpos = pos1 - pos0
        dvel = vel1 - vel0
        self.c0 = pos0
        self.c1 = vel0 * self.dt
        self.c2 = -(3.0 * vel0 + dvel) * self.dt + 3.0 * dpos
        self.c3 = (2.0 * vel0 + dvel) * self.dt - 2.0 * dpos

    def position(self, t):
        tn = (t - self.t0) / self.dt
        return self.c3 * tn ** 3 + self.c2 * tn ** 2 + self.c1 * tn + self.c0

    def velocity(self, t):
        tn = (t - self.t0) / self.dt
        return (3.0 * self.c3 * tn ** 2 + 2.0 * self.c2 * tn + self.c1) / self.dt


def get_spline_vel_z(swing_phase, swing_period, h_max=0.1, v_liftoff=0.1, v_touchdown=-0.2):
    """Swing z-velocity target (gait_sequence.py:96-107); numpy-vectorised ``if_else``."""
    mid = swing_period / 2
    s1 = CubicSpline(0, mid, 0, v_liftoff, h_max, 0)
    s2 = CubicSpline(mid, swing_period, h_max, 0, 0, v_touchdown)
    t = swing_phase * swing_period
    return np.where(np.asarray(swing_phase) < 0.5, s1.velocity(t), s2.velocity(t))


def horizon_dts(dt_min, dt_max, nodes):
    """Geometric step growth (ocp.py:71-74)."""
    ratio = dt_max / dt_min
    gamma = ratio ** (1 / (nodes - 1))
    return [dt_min * gamma ** i for i in range(nodes)]
