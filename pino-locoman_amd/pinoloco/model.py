"""Rigid-body model tables with Pinocchio's URDF/SRDF semantics.

The reference builds its model with ``RobotWrapper.BuildFromURDF(urdf, [dir],
JointModelFreeFlyer())`` (``utils/robot.py:13-20``), optionally reduces it with
``buildReducedRobot(lock_joints)`` (``utils/robot.py:21-22``; B2G locks the
gripper, joint id 20, ``utils/robot.py:83-86``) and reads the reference pose from
the SRDF (``utils/robot.py:26-28``).  Pinocchio is not available here, so this
module restates the parts of its URDF parser that decide the numbers the hot
path consumes:

* joint order = depth-first walk of the link tree where each link's children are
  visited in the order of their joint NAMES (urdfdom keeps joints in a
  ``std::map``);
* a free-flyer ``root_joint`` carries the root link;
* fixed joints are merged: the child link's inertia is appended to the parent
  joint at ``parent_frame.placement * joint_origin`` and a FIXED_JOINT frame plus
  a BODY frame are created at that placement;
* movable joints get ``jointPlacement = parent_frame.placement * joint_origin``;
* ``buildReducedModel`` turns a locked revolute joint into a fixed one at the
  locked configuration (the neutral value 0 here) and re-parents its frames.

The result is a plain-data :class:`Model` (numpy arrays) that serialises to the
JSON tables shipped in ``pinoloco/models/`` and that the C-ABI consumes through
``pl_model_desc`` (``include/pinoloco.h``).
"""
from __future__ import annotations

import json
import math
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import numpy as np

# Frame types (subset of pinocchio::FrameType values, same bit values).
OP_FRAME = 0x1
JOINT = 0x2
FIXED_JOINT = 0x4
BODY = 0x8
SENSOR = 0x10
ALL_FRAME_TYPES = OP_FRAME | JOINT | FIXED_JOINT | BODY | SENSOR

JT_UNIVERSE = 0
JT_FREEFLYER = 1
JT_REVOLUTE = 2


# --------------------------------------------------------------------------
# small SE3 / inertia helpers (host-side, numpy)
# --------------------------------------------------------------------------
def quat_xyzw_to_matrix(x, y, z, w):
    """Eigen ``Quaternion::toRotationMatrix`` (no renormalisation)."""
    tx, ty, tz = 2.0 * x, 2.0 * y, 2.0 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return np.array([
        [1.0 - (tyy + tzz), txy - twz, txz + twy],
        [txy + twz, 1.0 - (txx + tzz), tyz - twx],
        [txz - twy, tyz + twx, 1.0 - (txx + tyy)],
    ])


def rpy_to_matrix(roll, pitch, yaw):
    """urdfdom ``Rotation::setFromRPY`` (quaternion, normalised) -> Eigen matrix."""
    phi, the, psi = roll / 2.0, pitch / 2.0, yaw / 2.0
    x = math.sin(phi) * math.cos(the) * math.cos(psi) - math.cos(phi) * math.sin(the) * math.sin(psi)
    y = math.cos(phi) * math.sin(the) * math.cos(psi) + math.sin(phi) * math.cos(the) * math.sin(psi)
    z = math.cos(phi) * math.cos(the) * math.sin(psi) - math.sin(phi) * math.sin(the) * math.cos(psi)
    w = math.cos(phi) * math.cos(the) * math.cos(psi) + math.sin(phi) * math.sin(the) * math.sin(psi)
    n = math.sqrt(x * x + y * y + z * z + w * w)
    return quat_xyzw_to_matrix(x / n, y / n, z / n, w / n)


@dataclass
class SE3:
    R: np.ndarray = field(default_factory=lambda: np.eye(3))
    p: np.ndarray = field(default_factory=lambda: np.zeros(3))

    def __mul__(self, other: "SE3") -> "SE3":
        return SE3(self.R @ other.R, self.p + self.R @ other.p)

    def inverse(self) -> "SE3":
        return SE3(self.R.T.copy(), -self.R.T @ self.p)

    def to_list(self):
        return {"R": self.R.tolist(), "p": self.p.tolist()}

    @staticmethod
    def from_list(d):
        return SE3(np.array(d["R"], dtype=float), np.array(d["p"], dtype=float))


@dataclass
class Inertia:
    """Pinocchio ``InertiaTpl``: mass, lever (CoM in body frame), rotational inertia at CoM."""
    mass: float = 0.0
    lever: np.ndarray = field(default_factory=lambda: np.zeros(3))
    I: np.ndarray = field(default_factory=lambda: np.zeros((3, 3)))

    def is_zero(self):
        return self.mass == 0.0 and not np.any(self.lever) and not np.any(self.I)

    def act(self, M: SE3) -> "Inertia":
        """``M.act(Y)``: express the inertia in the frame M is placed in."""
        return Inertia(self.mass, M.p + M.R @ self.lever, M.R @ self.I @ M.R.T)

    def __iadd__(self, Yb: "Inertia"):
        # InertiaTpl::__pequ__ (pinocchio/spatial/inertia.hpp)
        eps = np.finfo(float).eps
        mab = self.mass + Yb.mass
        mab_inv = 1.0 / max(mab, eps)
        AB = self.lever - Yb.lever
        lever = self.lever * (self.mass * mab_inv) + (Yb.mass * mab_inv) * Yb.lever
        sk = np.array([[0, -AB[2], AB[1]], [AB[2], 0, -AB[0]], [-AB[1], AB[0], 0]])
        self.I = self.I + Yb.I - (self.mass * Yb.mass * mab_inv) * (sk @ sk)
        self.lever = lever
        self.mass = mab
        return self

    def matrix(self):
        """6x6 spatial inertia (linear first), Pinocchio convention."""
        m, c = self.mass, self.lever
        cx = np.array([[0, -c[2], c[1]], [c[2], 0, -c[0]], [-c[1], c[0], 0]])
        Y = np.zeros((6, 6))
        Y[:3, :3] = m * np.eye(3)
        Y[:3, 3:] = -m * cx
        Y[3:, :3] = m * cx
        Y[3:, 3:] = self.I - m * cx @ cx
        return Y

    def to_list(self):
        return {"mass": self.mass, "lever": self.lever.tolist(), "I": self.I.tolist()}

    @staticmethod
    def from_list(d):
        return Inertia(float(d["mass"]), np.array(d["lever"], dtype=float), np.array(d["I"], dtype=float))


@dataclass
class Joint:
    name: str
    jtype: int
    parent: int
    placement: SE3
    axis: np.ndarray
    idx_q: int
    idx_v: int
    nq: int
    nv: int
    lower: float = -np.inf
    upper: float = np.inf
    effort: float = np.inf
    velocity: float = np.inf


@dataclass
class Frame:
    name: str
    parent_joint: int
    parent_frame: int
    placement: SE3
    ftype: int
    inertia: Inertia = field(default_factory=Inertia)


class Model:
    """Plain-data restatement of the ``pinocchio.Model`` fields the hot path reads."""

    def __init__(self, name: str = ""):
        self.name = name
        self.joints: List[Joint] = [
            Joint("universe", JT_UNIVERSE, 0, SE3(), np.zeros(3), 0, 0, 0, 0)]
        self.inertias: List[Inertia] = [Inertia()]
        self.frames: List[Frame] = [Frame("universe", 0, 0, SE3(), FIXED_JOINT)]
        self.reference_configurations: Dict[str, np.ndarray] = {}
        self.gravity = np.array([0.0, 0.0, -9.81])
        self.nq = 0
        self.nv = 0

    # ------------------------------------------------------------------ build
    @property
    def njoints(self):
        return len(self.joints)

    def add_joint(self, parent, jtype, placement, name, axis=None, limits=None):
        nq, nv = (7, 6) if jtype == JT_FREEFLYER else (1, 1)
        j = Joint(name, jtype, parent, placement,
                  np.zeros(3) if axis is None else np.asarray(axis, dtype=float),
                  self.nq, self.nv, nq, nv)
        if limits is not None:
            j.lower, j.upper, j.effort, j.velocity = limits
        self.joints.append(j)
        self.inertias.append(Inertia())
        self.nq += nq
        self.nv += nv
        return len(self.joints) - 1

    def add_frame(self, frame: Frame, append_inertia=True):
        # Model::addFrame (pinocchio 3): appends the frame's inertia to its parent joint.
        if append_inertia and not frame.inertia.is_zero():
            self.inertias[frame.parent_joint] += frame.inertia.act(frame.placement)
        self.frames.append(frame)
        return len(self.frames) - 1

    def append_body_to_joint(self, joint_id, Y: Inertia, placement: SE3):
        self.inertias[joint_id] += Y.act(placement)

    # ------------------------------------------------------------------ query
    def get_frame_id(self, name, ftype=ALL_FRAME_TYPES):
        for i, f in enumerate(self.frames):
            if f.name == name and (f.ftype & ftype):
                return i
        return len(self.frames)  # pinocchio returns nframes when not found

    def exist_frame(self, name, ftype=ALL_FRAME_TYPES):
        return self.get_frame_id(name, ftype) < len(self.frames)

    def get_joint_id(self, name):
        for i, j in enumerate(self.joints):
            if j.name == name:
                return i
        return len(self.joints)

    def neutral(self):
        q = np.zeros(self.nq)
        for j in self.joints[1:]:
            if j.jtype == JT_FREEFLYER:
                q[j.idx_q + 6] = 1.0
        return q

    def total_mass(self):
        return float(sum(Y.mass for Y in self.inertias))

    # ------------------------------------------------------------------ io
    def to_dict(self):
        return {
            "name": self.name,
            "gravity": self.gravity.tolist(),
            "nq": self.nq,
            "nv": self.nv,
            "joints": [{
                "name": j.name, "type": j.jtype, "parent": j.parent,
                "placement": j.placement.to_list(), "axis": j.axis.tolist(),
                "idx_q": j.idx_q, "idx_v": j.idx_v, "nq": j.nq, "nv": j.nv,
                "limits": [_finite(j.lower), _finite(j.upper), _finite(j.effort), _finite(j.velocity)],
            } for j in self.joints],
            "inertias": [Y.to_list() for Y in self.inertias],
            "frames": [{
                "name": f.name, "parent_joint": f.parent_joint, "parent_frame": f.parent_frame,
                "placement": f.placement.to_list(), "type": f.ftype,
            } for f in self.frames],
            "reference_configurations": {k: v.tolist() for k, v in self.reference_configurations.items()},
        }

    @staticmethod
    def from_dict(d) -> "Model":
        m = Model(d["name"])
        m.gravity = np.array(d["gravity"], dtype=float)
        m.nq, m.nv = int(d["nq"]), int(d["nv"])
        m.joints = []
        for jd in d["joints"]:
            lim = [(_unfinite(x) if x is not None else np.inf) for x in jd["limits"]]
            j = Joint(jd["name"], int(jd["type"]), int(jd["parent"]), SE3.from_list(jd["placement"]),
                      np.array(jd["axis"], dtype=float), int(jd["idx_q"]), int(jd["idx_v"]),
                      int(jd["nq"]), int(jd["nv"]), *lim)
            m.joints.append(j)
        m.inertias = [Inertia.from_list(x) for x in d["inertias"]]
        m.frames = [Frame(f["name"], int(f["parent_joint"]), int(f["parent_frame"]),
                          SE3.from_list(f["placement"]), int(f["type"])) for f in d["frames"]]
        m.reference_configurations = {k: np.array(v, dtype=float)
                                      for k, v in d["reference_configurations"].items()}
        return m

    def save(self, path):
        with open(path, "w") as fh:
            json.dump(self.to_dict(), fh, indent=1)

    @staticmethod
    def load(path) -> "Model":
        with open(path) as fh:
            return Model.from_dict(json.load(fh))


def _finite(x):
    return None if not np.isfinite(x) else float(x)


def _unfinite(x):
    return float(x)


# --------------------------------------------------------------------------
# URDF parsing (urdfdom data model + pinocchio's tree walk)
# --------------------------------------------------------------------------
def _floats(s, n, default=0.0):
    if s is None:
        return [default] * n
    v = [float(t) for t in s.split()]
    assert len(v) == n, s
    return v


def _origin(el) -> SE3:
    o = el.find("origin") if el is not None else None
    if o is None:
        return SE3()
    xyz = _floats(o.get("xyz"), 3)
    rpy = _floats(o.get("rpy"), 3)
    return SE3(rpy_to_matrix(*rpy), np.array(xyz))


def _inertial(link_el) -> Inertia:
    """pinocchio ``convertFromUrdf(inertial)``: I expressed at the CoM in link axes."""
    ie = link_el.find("inertial")
    if ie is None:
        return Inertia()
    M = _origin(ie)
    mass = float(ie.find("mass").get("value"))
    it = ie.find("inertia")
    g = {k: float(it.get(k, 0.0)) for k in ("ixx", "ixy", "ixz", "iyy", "iyz", "izz")}
    I = np.array([[g["ixx"], g["ixy"], g["ixz"]],
                  [g["ixy"], g["iyy"], g["iyz"]],
                  [g["ixz"], g["iyz"], g["izz"]]])
    return Inertia(mass, M.p.copy(), M.R @ I @ M.R.T)


def build_model_from_urdf(urdf_path: str, root_joint_name: str = "root_joint") -> Model:
    """``pinocchio.buildModelFromUrdf(path, JointModelFreeFlyer())`` restated."""
    tree = ET.parse(urdf_path)
    robot = tree.getroot()
    links = {l.get("name"): l for l in robot.findall("link")}
    joints = {}
    for j in robot.findall("joint"):
        joints[j.get("name")] = j
    # urdfdom initTree: iterate joints in std::map (name) order
    children: Dict[str, List[str]] = {name: [] for name in links}
    parent_joint_of: Dict[str, str] = {}
    for jname in sorted(joints.keys()):
        j = joints[jname]
        p = j.find("parent").get("link")
        c = j.find("child").get("link")
        children[p].append(jname)
        parent_joint_of[c] = jname
    roots = [l for l in links if l not in parent_joint_of]
    assert len(roots) == 1, roots
    root = roots[0]

    model = Model(robot.get("name", ""))
    # addRootJoint
    jid = model.add_joint(0, JT_FREEFLYER, SE3(), root_joint_name)
    jf = model.add_frame(Frame(root_joint_name, jid, 0, SE3(), JOINT))
    _append_body(model, jf, _inertial(links[root]), SE3(), root)

    def body_id(link_name):
        fid = model.get_frame_id(link_name, BODY)
        assert fid < len(model.frames), link_name
        return fid

    def parse_tree(link_name):
        for jname in children[link_name]:
            j = joints[jname]
            child = j.find("child").get("link")
            parent_fid = body_id(link_name)
            pf = model.frames[parent_fid]
            jpl = _origin(j)
            Y = _inertial(links[child])
            jt = j.get("type")
            if jt in ("revolute", "continuous"):
                assert jt == "revolute", "continuous joints are not used by the reference robots"
                axis = np.array(_floats(j.find("axis").get("xyz") if j.find("axis") is not None else "1 0 0", 3))
                lim = j.find("limit")
                limits = (float(lim.get("lower", 0.0)), float(lim.get("upper", 0.0)),
                          float(lim.get("effort", 0.0)), float(lim.get("velocity", 0.0)))
                new_j = model.add_joint(pf.parent_joint, JT_REVOLUTE, pf.placement * jpl, jname,
                                        axis=axis, limits=limits)
                jfid = model.add_frame(Frame(jname, new_j, parent_fid, SE3(), JOINT))
                _append_body(model, jfid, Y, SE3(), child)
            elif jt == "fixed":
                placement = pf.placement * jpl
                fid = model.add_frame(Frame(jname, pf.parent_joint, parent_fid, placement, FIXED_JOINT, Y))
                model.frames.append(Frame(child, pf.parent_joint, fid, placement, BODY))
            else:
                raise NotImplementedError(f"joint type {jt}")
            parse_tree(child)

    parse_tree(root)
    return model


def _append_body(model: Model, fid: int, Y: Inertia, placement: SE3, body_name: str):
    f = model.frames[fid]
    p = f.placement * placement
    if not Y.is_zero():
        model.append_body_to_joint(f.parent_joint, Y, p)
    model.frames.append(Frame(body_name, f.parent_joint, fid, p, BODY))


# --------------------------------------------------------------------------
# SRDF reference configurations and joint locking
# --------------------------------------------------------------------------
def load_reference_configurations(model: Model, srdf_path: str):
    """``pinocchio.loadReferenceConfigurations`` restated (group_state -> q)."""
    root = ET.parse(srdf_path).getroot()
    for gs in root.findall("group_state"):
        q = model.neutral()
        for je in gs.findall("joint"):
            jid = model.get_joint_id(je.get("name"))
            if jid >= model.njoints:
                continue
            j = model.joints[jid]
            vals = [float(t) for t in je.get("value").split()]
            if len(vals) != j.nq:
                continue
            q[j.idx_q:j.idx_q + j.nq] = vals
        model.reference_configurations[gs.get("name")] = q


def _joint_transform(j: Joint, qj: np.ndarray) -> SE3:
    if j.jtype == JT_REVOLUTE:
        a = j.axis / np.linalg.norm(j.axis)
        th = float(qj[0])
        K = np.array([[0, -a[2], a[1]], [a[2], 0, -a[0]], [-a[1], a[0], 0]])
        R = np.eye(3) + math.sin(th) * K + (1 - math.cos(th)) * K @ K
        return SE3(R, np.zeros(3))
    raise NotImplementedError


def build_reduced_model(model: Model, lock_joint_ids, q_ref: Optional[np.ndarray] = None) -> Model:
    """``pinocchio.buildReducedModel`` restated for locked revolute joints.

    A locked joint becomes a FIXED_JOINT frame at ``jointPlacement * jMi(q_ref)``;
    its body inertia is appended to its parent joint and every frame it supported
    is re-parented with the composed placement.
    """
    if q_ref is None:
        q_ref = model.neutral()
    lock = sorted(set(int(i) for i in lock_joint_ids))
    for jid in lock:
        assert 0 < jid < model.njoints
        assert model.joints[jid].jtype == JT_REVOLUTE
    red = Model(model.name)
    red.gravity = model.gravity.copy()
    new_index = {0: 0}
    # placement of the (locked) joint frame w.r.t. the nearest kept ancestor joint
    extra = {0: SE3()}
    for jid in range(1, model.njoints):
        j = model.joints[jid]
        par = j.parent
        kept_parent = new_index[par]
        base = extra[par]
        if jid in lock:
            M = base * j.placement * _joint_transform(j, q_ref[j.idx_q:j.idx_q + 1])
            new_index[jid] = kept_parent
            extra[jid] = M
            red.inertias[kept_parent] += model.inertias[jid].act(M)
        else:
            nj = red.add_joint(kept_parent, j.jtype, base * j.placement, j.name, axis=j.axis,
                               limits=(j.lower, j.upper, j.effort, j.velocity))
            red.inertias[nj] = Inertia(model.inertias[jid].mass, model.inertias[jid].lever.copy(),
                                       model.inertias[jid].I.copy())
            new_index[jid] = nj
            extra[jid] = SE3()
    # frames: keep order, re-parent frames attached to locked joints
    for f in model.frames[1:]:
        M = extra[f.parent_joint] * f.placement
        ftype = f.ftype
        if f.ftype == JOINT and model.get_joint_id(f.name) in lock:
            ftype = FIXED_JOINT
        red.frames.append(Frame(f.name, new_index[f.parent_joint], f.parent_frame, M, ftype))
    for k, q in model.reference_configurations.items():
        red.reference_configurations[k] = _reduce_q(model, red, q)
    return red


def _reduce_q(model, red, q):
    out = red.neutral()
    for j in red.joints[1:]:
        src = model.joints[model.get_joint_id(j.name)]
        out[j.idx_q:j.idx_q + j.nq] = q[src.idx_q:src.idx_q + src.nq]
    return out
