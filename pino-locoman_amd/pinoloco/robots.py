"""Robot definitions (Go2, B2, B2G) mirroring ``utils/robot.py`` of the reference.

The reference parses the URDF/SRDF with Pinocchio at construction time
(``utils/robot.py:10-42``).  Here the same parse is done by
:mod:`pinoloco.model` once, in the build container, and the resulting tables are
shipped as JSON in ``pinoloco/models/`` (``tools/gen_models.py``) so the GPU box
(which has no copy of the reference) loads identical numbers.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np

from . import model as mdl
from .gait import GaitSequence

MODELS_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "models")


def load_model(name: str) -> mdl.Model:
    return mdl.Model.load(os.path.join(MODELS_DIR, f"{name}.json"))


class Robot:
    """utils/robot.py:10-42 (free-flyer root, optional joint locking, SRDF pose)."""

    def __init__(self, model: mdl.Model, reference_pose: Optional[str]):
        self.model = model
        if reference_pose:
            self.q0 = model.reference_configurations[reference_pose].copy()
        else:
            self.q0 = model.neutral()
        self.nq = model.nq
        self.nv = model.nv
        self.nj = self.nq - 7
        self.nf = 12
        self.ext_force_frame = None
        self.arm_ee_frame = None
        self.gait_sequence = None
        self.foot_frames = None

    @property
    def mass(self):
        """``data.mass[0]`` after ``computeAllTerms`` (total mass), used at ocp.py:29."""
        return self.model.total_mass()

    def set_gait_sequence(self, gait_type, gait_period):
        self.gait_sequence = GaitSequence(gait_type, gait_period)
        self.foot_frames = [self.model.get_frame_id(f) for f in self.gait_sequence.feet]


class Go2(Robot):
    def __init__(self, reference_pose="standing"):
        super().__init__(load_model("go2"), reference_pose)
        self.joint_pos_min = np.tile([-1.0472, -1.5708, -2.7227], 4)
        self.joint_pos_max = np.tile([1.0472, 3.4907, -0.83776], 4)
        self.joint_vel_max = np.tile([30.1, 30.1, 15.70], 4)
        self.joint_torque_max = np.tile([23.7, 23.7, 45.43], 4)


class B2(Robot):
    def __init__(self, reference_pose="standing", payload=None):
        super().__init__(load_model("b2"), reference_pose)
        self.joint_pos_min = np.tile([-0.87, -0.94, -2.82], 4)
        self.joint_pos_max = np.tile([0.87, 4.69, -0.43], 4)
        self.joint_vel_max = np.tile([23.0, 23.0, 14.0], 4)
        self.joint_torque_max = np.tile([200, 200, 320], 4)
        if payload == "front":
            self.ext_force_frame = self.model.get_frame_id("payload_joint_front", mdl.FIXED_JOINT)
            self.nf += 3
        elif payload == "rear":
            self.ext_force_frame = self.model.get_frame_id("payload_joint_rear", mdl.FIXED_JOINT)
            self.nf += 3


class B2G(Robot):
    def __init__(self, reference_pose="standing_with_arm_up", ignore_arm=False):
        # utils/robot.py:79-118; the gripper (joint 20) is locked in b2g.json,
        # "ignore_arm" locks joints 14..20 (b2g_noarm.json).
        super().__init__(load_model("b2g_noarm" if ignore_arm else "b2g"), reference_pose)
        self.joint_pos_min = np.tile([-0.87, -0.94, -2.82], 4)
        self.joint_pos_max = np.tile([0.87, 4.69, -0.43], 4)
        self.joint_vel_max = np.tile([23.0, 23.0, 14.0], 4)
        self.joint_torque_max = np.tile([200, 200, 320], 4)
        if not ignore_arm:
            self.ext_force_frame = self.model.get_frame_id("gripperStator", mdl.FIXED_JOINT)
            self.arm_ee_frame = self.model.get_frame_id("gripperStator", mdl.FIXED_JOINT)
            self.nf += 3
            self.joint_pos_min = np.concatenate((self.joint_pos_min, [-2.62, 0.0, -2.88, -1.52, -1.34, -2.79]))
            self.joint_pos_max = np.concatenate((self.joint_pos_max, [2.62, 2.97, 0.0, 1.52, 1.34, 2.79]))
            self.joint_vel_max = np.concatenate((self.joint_vel_max, [3.14] * 6))
            self.joint_torque_max = np.concatenate((self.joint_torque_max, [30, 60, 30, 30, 30, 30]))


ROBOTS = {"go2": Go2, "b2": B2, "b2g": B2G}
