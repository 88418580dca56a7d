"""Dynamics plugin surface of the reference (``dynamics/*.py``), batched on the C-ABI.

The reference's ``Dynamics`` classes are factories: each method builds a CasADi
point function from pinocchio.casadi and returns it (``dynamics/dynamics.py:23-118``,
``dynamics_whole_body_torque.py``, ``dynamics_whole_body_acc.py``,
``dynamics_centroidal_vel.py``).  The classes here keep those names and argument
orders; the returned callables take one point (1-D arrays) or a batch (arrays of
shape ``[B, len]``) and evaluate it with ``pl_dyn_eval`` (csrc/dyn.h, csrc/k_dyn.hip):
one GPU thread per point on ``device >= 0``, the library's host build of the same
code on ``device = -1`` (the default: these are per-point host calls in the
reference, e.g. in retract and the debug identity of ``run_mpc.py:186-241``).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib

FN = dict(rnea=0, aba=1, frame_pos=2, frame_vel=3, gaps_wb=4, base_acc_wb=5, com_dyn=6, base_vel_cv=7,
          base_acc_cv=8, gaps_cv=9, crba=10, nle=11, frame_jac=12, cmap=13, com=14, integrate_wb=15,
          difference_wb=16, integrate_cv=17, difference_cv=18, gaps_ca=19)


class _DynHandle:
    def __init__(self, robot, ext_force_frame, device):
        from .ocp import ModelCache
        self.model_h = ModelCache.get(robot.model)
        feet = np.ascontiguousarray(np.asarray(robot.foot_frames, dtype=np.int32))
        base = robot.model.get_frame_id("base_link")
        ext = -1 if ext_force_frame is None else int(ext_force_frame)
        h = C.c_void_p()
        _lib.check(_lib.lib().pl_dyn_create(self.model_h.h, _lib.iptr(feet), ext, int(base), int(device), C.byref(h)))
        self.h = h

    def __del__(self):
        try:
            if getattr(self, "h", None) and _lib._lib is not None:
                _lib._lib.pl_dyn_destroy(self.h)
        except Exception:  # noqa: BLE001
            pass


class PointFunction:
    """A batched point function (the role of the reference's ``ca.Function``)."""

    def __init__(self, handle, name, fn, frame=-1, flags=0, out_shape=None):
        self._h, self.name, self._fn, self._frame, self._flags = handle, name, fn, int(frame), int(flags)
        ins = (C.c_int * 4)()
        out = C.c_int()
        _lib.check(_lib.lib().pl_dyn_sizes(handle.h, fn, self._flags, ins, C.byref(out)))
        self.in_len = [int(v) for v in ins if v > 0]
        self.out_len = int(out.value)
        self.out_shape = out_shape

    def __call__(self, *args):
        if len(args) != len(self.in_len):
            raise ValueError(f"{self.name} takes {len(self.in_len)} inputs ({self.in_len})")
        arrs = [np.asarray(a, dtype=np.float64) for a in args]
        single = all(a.ndim <= 1 for a in arrs)
        B = 1 if single else max(a.shape[0] for a in arrs if a.ndim == 2)
        ins = []
        for a, n in zip(arrs, self.in_len):
            a = np.ascontiguousarray(np.broadcast_to(a.reshape(-1, n) if a.ndim <= 1 else a, (B, n)))
            ins.append(a)
        out = np.zeros((B, self.out_len))
        ptrs = [_lib.dptr(a) for a in ins] + [None] * (4 - len(ins))
        _lib.check(_lib.lib().pl_dyn_eval(self._h.h, self._fn, B, self._frame, self._flags, *ptrs, _lib.dptr(out)))
        if self.out_shape:
            out = out.reshape((B,) + self.out_shape)
        return out[0] if single else out


class Dynamics:
    """dynamics/dynamics.py:6-118 (base class)."""

    def __init__(self, robot, device=-1):
        self.robot = robot
        self.model = robot.model
        self.mass = robot.mass
        self.foot_frames = list(robot.foot_frames)
        self.base_frame = robot.model.get_frame_id("base_link")
        self.nq, self.nv = robot.nq, robot.nv
        self.nj = self.nq - 7
        self.device = device
        self._handles = {}

    def _h(self, ext_force_frame=None):
        key = None if ext_force_frame is None else int(ext_force_frame)
        if key not in self._handles:
            self._handles[key] = _DynHandle(self.robot, key, self.device)
        return self._handles[key]

    def _fn(self, name, ext_force_frame=None, frame=-1, flags=0, out_shape=None):
        flags |= 1 if ext_force_frame is not None else 0
        return PointFunction(self._h(ext_force_frame), name, FN[name], frame, flags, out_shape)

    # ---- state maps (whole-body state x = [q, v]; dynamics_whole_body_torque.py:11-40)
    def state_integrate(self):
        return self._fn("integrate_wb")

    def state_difference(self):
        return self._fn("difference_wb")

    # ---- factories of dynamics/dynamics.py
    def rnea_dynamics(self, ext_force_frame=None):
        """(q, v, a, forces) -> tau_rnea (nv)."""
        return self._fn("rnea", ext_force_frame)

    def get_frame_position(self, frame_id):
        return self._fn("frame_pos", frame=frame_id)

    def get_frame_velocity(self, frame_id, relative_to_base=False):
        return self._fn("frame_vel", frame=frame_id, flags=2 if relative_to_base else 0)

    # ---- pinocchio terms of the reference's debug identity (run_mpc.py:201-236)
    def crba(self):
        return self._fn("crba", out_shape=(self.nv, self.nv))

    def nonlinear_effects(self):
        return self._fn("nle")

    def frame_jacobian(self, frame_id):
        """computeFrameJacobian(..., LOCAL_WORLD_ALIGNED) -> 6 x nv."""
        return self._fn("frame_jac", frame=frame_id, out_shape=(6, self.nv))

    def centroidal_map(self):
        return self._fn("cmap", out_shape=(6, self.nv))

    def center_of_mass(self):
        return self._fn("com")


class DynamicsWholeBodyTorque(Dynamics):
    """dynamics/dynamics_whole_body_torque.py: RNEA (base class) and ABA."""

    def aba_dynamics(self, ext_force_frame=None):
        """(q, v, tau_j, forces) -> a (nv): ABA with tau = [0_6; tau_j]."""
        return self._fn("aba", ext_force_frame)


class DynamicsWholeBodyAcc(Dynamics):
    """dynamics/dynamics_whole_body_acc.py."""

    def base_acc_dynamics(self, ext_force_frame=None):
        """(q, v, a_j, forces) -> a_b = M_bb^-1 (-nle_b - M_bj a_j + sum J_c,b^T f)."""
        return self._fn("base_acc_wb", ext_force_frame)

    def dynamics_gaps(self, ext_force_frame=None):
        """(q, v, a, forces) -> RNEA base rows (6)."""
        return self._fn("gaps_wb", ext_force_frame)


class DynamicsCentroidalVel(Dynamics):
    """dynamics/dynamics_centroidal_vel.py: x = [h, q], dx = [dh, dq]."""

    def state_integrate(self):
        return self._fn("integrate_cv")

    def state_difference(self):
        return self._fn("difference_cv")

    def com_dynamics(self, ext_force_frame=None):
        """(q, forces) -> h_dot = [sum f + m g, sum (p_e - com) x f_e] / m."""
        return self._fn("com_dyn", ext_force_frame)

    def base_vel_dynamics(self):
        """(h, q, v_j) -> v_b = A_b^-1 (m h - A_j v_j)."""
        return self._fn("base_vel_cv")

    def base_acc_dynamics(self, ext_force_frame=None):
        """(q, v, a_j, forces) -> a_b = A_b^-1 (dh - dA v - A_j a_j) (pinocchio dccrba)."""
        return self._fn("base_acc_cv", ext_force_frame)

    def dynamics_gaps(self):
        """(h, q, v) -> A(q) v - m h."""
        return self._fn("gaps_cv")


class DynamicsCentroidalAcc(Dynamics):
    """dynamics/dynamics_centroidal_acc.py: x = [q, v]; the base equations in centroidal form."""

    def base_acc_dynamics(self, ext_force_frame=None):
        """(q, v, a_j, forces) -> a_b = A_b^-1 (dh - dA v - A_j a_j) (pinocchio dccrba)."""
        return self._fn("base_acc_cv", ext_force_frame)

    def dynamics_gaps(self, ext_force_frame=None):
        """(q, v, a, forces) -> A a + dA v - dh (6)."""
        return self._fn("gaps_ca", ext_force_frame)


DYNAMICS_CLASSES = {"whole_body_rnea": DynamicsWholeBodyTorque, "whole_body_aba": DynamicsWholeBodyTorque,
                    "whole_body_acc": DynamicsWholeBodyAcc, "centroidal_vel": DynamicsCentroidalVel,
                    "centroidal_acc": DynamicsCentroidalAcc}
