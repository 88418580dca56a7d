"""ORACLE (test infrastructure only) -- numpy fp64 restatement of Pinocchio's algorithms.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this package, and only as the checker.  The product path
(``pino-locoman_amd/``) never imports it.

PARITY UNPINNED: the reference's algorithms live in Pinocchio (unpinned,
``README.md:12``), which is neither vendored in ``/root/reference`` nor installed
here.  This file restates Pinocchio's published conventions and is pinned only by
physical identities (EOM == RNEA, ABA(RNEA(a)) == a, difference(integrate) == id,
total mass) that the reference's own debug block checks (``run_mpc.py:186-241``).

Conventions (Pinocchio): Motion = [linear; angular], Force = [force; torque];
free-flyer q = [p, qx, qy, qz, qw], v = [v_local; w_local]; gravity (0, 0, -9.81).
Every function accepts a leading batch shape and complex inputs (complex-step
differentiation): branches test ``.real`` only and no ``abs`` is taken on values.
"""
from __future__ import annotations

import numpy as np

JT_FREEFLYER = 1
JT_REVOLUTE = 2


# ---------------------------------------------------------------- 3-vectors
def cross(a, b):
    return np.stack([a[..., 1] * b[..., 2] - a[..., 2] * b[..., 1],
                     a[..., 2] * b[..., 0] - a[..., 0] * b[..., 2],
                     a[..., 0] * b[..., 1] - a[..., 1] * b[..., 0]], axis=-1)


def skew(a):
    z = np.zeros_like(a[..., 0])
    return np.stack([np.stack([z, -a[..., 2], a[..., 1]], -1),
                     np.stack([a[..., 2], z, -a[..., 0]], -1),
                     np.stack([-a[..., 1], a[..., 0], z], -1)], axis=-2)


def mv(R, x):
    return np.einsum("...ij,...j->...i", R, x)


def mtv(R, x):
    return np.einsum("...ji,...j->...i", R, x)


def mm(A, B):
    return np.matmul(A, B)


def mtm(A, B):
    return np.matmul(np.swapaxes(A, -1, -2), B)


# ---------------------------------------------------------------- spatial algebra
def act_motion(R, p, v):          # M.act(v)
    w = mv(R, v[..., 3:])
    return np.concatenate([mv(R, v[..., :3]) + cross(p, w), w], -1)


def act_inv_motion(R, p, v):      # M.actInv(v)
    w = v[..., 3:]
    return np.concatenate([mtv(R, v[..., :3] - cross(p, w)), mtv(R, w)], -1)


def act_force(R, p, f):           # M.act(f)
    fl = mv(R, f[..., :3])
    return np.concatenate([fl, mv(R, f[..., 3:]) + cross(p, fl)], -1)


def motion_cross_motion(v1, v2):  # v1 x v2
    return np.concatenate([cross(v1[..., 3:], v2[..., :3]) + cross(v1[..., :3], v2[..., 3:]),
                           cross(v1[..., 3:], v2[..., 3:])], -1)


def motion_cross_force(v, f):     # v x* f
    return np.concatenate([cross(v[..., 3:], f[..., :3]),
                           cross(v[..., 3:], f[..., 3:]) + cross(v[..., :3], f[..., :3])], -1)


def inertia_mul(m, c, Ic, v):     # Y * v  (Pinocchio InertiaTpl::__mult__)
    fl = m * (v[..., :3] - cross(c, v[..., 3:]))
    return np.concatenate([fl, mv(Ic, v[..., 3:]) + cross(c, fl)], -1)


def inertia_matrix(m, c, Ic):
    cx = skew(np.asarray(c, dtype=float))
    Y = np.zeros((6, 6))
    Y[:3, :3] = m * np.eye(3)
    Y[:3, 3:] = -m * cx
    Y[3:, :3] = m * cx
    Y[3:, 3:] = Ic - m * cx @ cx
    return Y


def X_actinv(R, p):
    """6x6 motion transform implementing M.actInv (parent coords -> child coords)."""
    shp = R.shape[:-2]
    X = np.zeros(shp + (6, 6), dtype=np.result_type(R, p))
    Rt = np.swapaxes(R, -1, -2)
    X[..., :3, :3] = Rt
    X[..., :3, 3:] = -mm(Rt, skew(p))
    X[..., 3:, 3:] = Rt
    return X


# ---------------------------------------------------------------- SO3 / SE3
PREC3 = np.finfo(float).eps ** (1.0 / 4.0)   # TaylorSeriesExpansion<double>::precision<3>()


def exp3(w):
    t2 = np.sum(w * w, -1)
    small = t2.real < PREC3 ** 2
    t2s = np.where(small, 1.0, t2)
    t = np.sqrt(t2s)
    st, ct = np.sin(t), np.cos(t)
    a_v = np.where(small, 1 - t2 / 6, st / t)
    a_wxv = np.where(small, 0.5 - t2 / 24, (1 - ct) / t2s)
    diag = np.where(small, 1 - t2 / 2, ct)
    R = a_wxv[..., None, None] * (w[..., :, None] * w[..., None, :])
    R = R + a_v[..., None, None] * skew(w)
    R = R + diag[..., None, None] * np.eye(3)
    return R


def exp6(nu):
    """pinocchio exp6: SE3 exponential of a twist [v; w]."""
    v, w = nu[..., :3], nu[..., 3:]
    t2 = np.sum(w * w, -1)
    small = t2.real < PREC3 ** 2
    t2s = np.where(small, 1.0, t2)
    t = np.sqrt(t2s)
    st, ct = np.sin(t), np.cos(t)
    a_wxv = np.where(small, 0.5 - t2 / 24, (1 - ct) / t2s)
    a_v = np.where(small, 1 - t2 / 6, st / t)
    a_w = np.where(small, 1.0 / 6 - t2 / 120, (1 - a_v) / t2s)
    diag = np.where(small, 1 - t2 / 2, ct)
    trans = a_v[..., None] * v + (a_w * np.sum(w * v, -1))[..., None] * w + a_wxv[..., None] * cross(w, v)
    R = a_wxv[..., None, None] * (w[..., :, None] * w[..., None, :]) + a_v[..., None, None] * skew(w) \
        + diag[..., None, None] * np.eye(3)
    return R, trans


def quat_to_matrix(qv):
    x, y, z, w = qv[..., 0], qv[..., 1], qv[..., 2], qv[..., 3]
    tx, ty, tz = 2 * x, 2 * y, 2 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    return np.stack([np.stack([1 - (tyy + tzz), txy - twz, txz + twy], -1),
                     np.stack([txy + twz, 1 - (txx + tzz), tyz - twx], -1),
                     np.stack([txz - twy, tyz + twx, 1 - (txx + tyy)], -1)], -2)


def matrix_to_quat(R):
    """Eigen quaternionbase_assign_impl (matrix -> quaternion [x, y, z, w])."""
    shp = R.shape[:-2]
    out = np.zeros(shp + (4,), dtype=R.dtype)
    t = R[..., 0, 0] + R[..., 1, 1] + R[..., 2, 2]
    # branch t > 0
    tp = np.sqrt(np.where(t.real > 0, t + 1.0, 1.0))
    inv = 0.5 / tp
    pos = np.stack([(R[..., 2, 1] - R[..., 1, 2]) * inv, (R[..., 0, 2] - R[..., 2, 0]) * inv,
                    (R[..., 1, 0] - R[..., 0, 1]) * inv, 0.5 * tp], -1)
    # branch t <= 0 (evaluated per element; rare)
    neg = np.zeros_like(out)
    flat_R = R.reshape((-1, 3, 3))
    flat_n = neg.reshape((-1, 4))
    for k in range(flat_R.shape[0]):
        M = flat_R[k]
        if (M[0, 0] + M[1, 1] + M[2, 2]).real > 0:
            continue
        i = 0
        if M[1, 1].real > M[0, 0].real:
            i = 1
        if M[2, 2].real > M[i, i].real:
            i = 2
        j, kk = (i + 1) % 3, (i + 2) % 3
        tt = np.sqrt(M[i, i] - M[j, j] - M[kk, kk] + 1.0)
        qv = np.zeros(4, dtype=R.dtype)
        qv[i] = 0.5 * tt
        tt = 0.5 / tt
        qv[3] = (M[kk, j] - M[j, kk]) * tt
        qv[j] = (M[j, i] + M[i, j]) * tt
        qv[kk] = (M[kk, i] + M[i, kk]) * tt
        flat_n[k] = qv
    return np.where((t.real > 0)[..., None], pos, neg)


def log3(R):
    """pinocchio log3 (value path used by ``difference``; real inputs)."""
    tr = R[..., 0, 0] + R[..., 1, 1] + R[..., 2, 2]
    theta = np.where(tr >= 3, 0.0, np.where(tr <= -1, np.pi, np.arccos(np.clip((tr - 1) / 2, -1.0, 1.0))))
    small = theta < PREC3
    ths = np.where(small, 1.0, theta)
    t = np.where(small, 1 + theta * theta / 6, ths / np.sin(ths))
    axis = np.stack([R[..., 2, 1] - R[..., 1, 2], R[..., 0, 2] - R[..., 2, 0], R[..., 1, 0] - R[..., 0, 1]], -1)
    return (t / 2)[..., None] * axis, theta


def log6(R, p):
    w, theta = log3(R)
    t2 = theta * theta
    small = theta.real < PREC3
    ths = np.where(small, 1.0, theta)
    st, ct = np.sin(ths), np.cos(ths)
    alpha = np.where(small, 1 - t2 / 12 - t2 * t2 / 720, ths * st / (2 * (1 - ct)))
    beta = np.where(small, 1.0 / 12 + t2 / 720, 1 / (ths * ths) - st / (2 * ths * (1 - ct)))
    lin = alpha[..., None] * p - 0.5 * cross(w, p) + (beta * np.sum(w * p, -1))[..., None] * w
    return np.concatenate([lin, w], -1)


# ---------------------------------------------------------------- model tables
class ModelArrays:
    """numpy view of pinoloco.model.Model for the oracle."""

    def __init__(self, model):
        self.model = model
        self.nj = model.njoints
        self.nq, self.nv = model.nq, model.nv
        self.parent = [j.parent for j in model.joints]
        self.jtype = [j.jtype for j in model.joints]
        self.idx_q = [j.idx_q for j in model.joints]
        self.idx_v = [j.idx_v for j in model.joints]
        self.jR = [j.placement.R for j in model.joints]
        self.jp = [j.placement.p for j in model.joints]
        self.axis = [j.axis for j in model.joints]
        self.mass = [Y.mass for Y in model.inertias]
        self.lever = [Y.lever for Y in model.inertias]
        self.Ic = [Y.I for Y in model.inertias]
        self.Y6 = [inertia_matrix(Y.mass, Y.lever, Y.I) for Y in model.inertias]
        self.gravity = model.gravity
        self.total_mass = model.total_mass()

    def frame(self, fid):
        f = self.model.frames[fid]
        return f.parent_joint, f.placement.R, f.placement.p


def _rev_rot(axis, qj):
    s, c = np.sin(qj), np.cos(qj)
    a = axis
    if a[0] == 1 and a[1] == 0 and a[2] == 0:
        o, z = np.ones_like(s), np.zeros_like(s)
        return np.stack([np.stack([o, z, z], -1), np.stack([z, c, -s], -1), np.stack([z, s, c], -1)], -2)
    if a[0] == 0 and a[1] == 1 and a[2] == 0:
        o, z = np.ones_like(s), np.zeros_like(s)
        return np.stack([np.stack([c, z, s], -1), np.stack([z, o, z], -1), np.stack([-s, z, c], -1)], -2)
    if a[0] == 0 and a[1] == 0 and a[2] == 1:
        o, z = np.ones_like(s), np.zeros_like(s)
        return np.stack([np.stack([c, -s, z], -1), np.stack([s, c, z], -1), np.stack([z, z, o], -1)], -2)
    K = skew(np.broadcast_to(np.asarray(a, float), s.shape + (3,)))
    return np.eye(3) + s[..., None, None] * K + (1 - c)[..., None, None] * mm(K, K)


def joint_transforms(M: ModelArrays, q):
    """liMi for every joint (R, p), batch-leading."""
    out = [None] * M.nj
    for i in range(1, M.nj):
        iq = M.idx_q[i]
        if M.jtype[i] == JT_FREEFLYER:
            R = quat_to_matrix(q[..., iq + 3:iq + 7])
            p = q[..., iq:iq + 3]
        else:
            Rj = _rev_rot(M.axis[i], q[..., iq])
            R = mm(np.broadcast_to(M.jR[i], Rj.shape), Rj)
            p = np.broadcast_to(M.jp[i], Rj.shape[:-2] + (3,)).astype(Rj.dtype)
        out[i] = (R, p)
    return out


def forward_kinematics(M: ModelArrays, q):
    li = joint_transforms(M, q)
    oM = [None] * M.nj
    for i in range(1, M.nj):
        R, p = li[i]
        par = M.parent[i]
        if par == 0:
            oM[i] = (R, p)
        else:
            Ro, po = oM[par]
            oM[i] = (mm(Ro, R), po + mv(Ro, p))
    return li, oM


def _S(M, i, shape, dtype):
    """Motion subspace of joint i as a (6 x nv_i) matrix."""
    if M.jtype[i] == JT_FREEFLYER:
        return np.eye(6)
    S = np.zeros((6, 1))
    S[3:, 0] = M.axis[i]
    return S


def joint_vel(M, i, x):
    iv = M.idx_v[i]
    if M.jtype[i] == JT_FREEFLYER:
        return x[..., iv:iv + 6]
    z = np.zeros_like(x[..., iv])
    a = M.axis[i]
    return np.stack([z, z, z, a[0] * x[..., iv], a[1] * x[..., iv], a[2] * x[..., iv]], -1)


def rnea(M: ModelArrays, q, v, a, fext=None, gravity=True):
    """pinocchio::rnea(model, data, q, v, a, fext) -- fext[i] in joint-i local frame
    (gravity=False: the same recursion with a zero gravity field)."""
    li, _ = forward_kinematics(M, q)
    nb = M.nj
    vs, as_, fs = [None] * nb, [None] * nb, [None] * nb
    shape = q.shape[:-1]
    dt = np.result_type(q, v, a)
    g = np.zeros(shape + (6,), dtype=dt)
    if gravity:
        g[..., :3] = -M.gravity
    for i in range(1, nb):
        R, p = li[i]
        par = M.parent[i]
        vJ = joint_vel(M, i, v)
        aJ = joint_vel(M, i, a)
        if par == 0:
            vi = vJ
            ai = act_inv_motion(R, p, g) + aJ
        else:
            vi = act_inv_motion(R, p, vs[par]) + vJ
            ai = act_inv_motion(R, p, as_[par]) + aJ + motion_cross_motion(vi, vJ)
        fi = inertia_mul(M.mass[i], M.lever[i], M.Ic[i], ai) + \
            motion_cross_force(vi, inertia_mul(M.mass[i], M.lever[i], M.Ic[i], vi))
        if fext is not None and fext[i] is not None:
            fi = fi - fext[i]
        vs[i], as_[i], fs[i] = vi, ai, fi
    tau = np.zeros(shape + (M.nv,), dtype=np.result_type(dt, fs[1]))
    for i in range(nb - 1, 0, -1):
        iv = M.idx_v[i]
        if M.jtype[i] == JT_FREEFLYER:
            tau[..., iv:iv + 6] = fs[i]
        else:
            tau[..., iv] = np.einsum("...k,k->...", fs[i][..., 3:], M.axis[i])
        par = M.parent[i]
        if par > 0:
            R, p = li[i]
            fs[par] = fs[par] + act_force(R, p, fs[i])
    return tau


def aba(M: ModelArrays, q, v, tau, fext=None):
    """pinocchio::aba(model, data, q, v, tau, fext) (articulated-body algorithm)."""
    li, _ = forward_kinematics(M, q)
    nb = M.nj
    shape = q.shape[:-1]
    dt = np.result_type(q, v, tau)
    vs, cs, pA, Ya = [None] * nb, [None] * nb, [None] * nb, [None] * nb
    for i in range(1, nb):
        R, p = li[i]
        par = M.parent[i]
        vJ = joint_vel(M, i, v)
        vi = vJ if par == 0 else act_inv_motion(R, p, vs[par]) + vJ
        ci = motion_cross_motion(vi, vJ)
        Yi = np.broadcast_to(M.Y6[i], shape + (6, 6)).astype(dt)
        pi = motion_cross_force(vi, mv(Yi, vi))
        if fext is not None and fext[i] is not None:
            pi = pi - fext[i]
        vs[i], cs[i], pA[i], Ya[i] = vi, ci, pi, Yi
    U, Dinv, u = [None] * nb, [None] * nb, [None] * nb
    for i in range(nb - 1, 0, -1):
        S = _S(M, i, shape, dt)
        iv = M.idx_v[i]
        nvi = S.shape[1]
        Ui = np.einsum("...ij,jk->...ik", Ya[i], S)
        Di = np.einsum("ji,...jk->...ik", S, Ui)
        Dinvi = np.linalg.inv(Di)
        ui = tau[..., iv:iv + nvi] - np.einsum("ji,...j->...i", S, pA[i])
        U[i], Dinv[i], u[i] = Ui, Dinvi, ui
        par = M.parent[i]
        if par > 0:
            Ia = Ya[i] - mm(mm(Ui, Dinvi), np.swapaxes(Ui, -1, -2))
            pa = pA[i] + mv(Ia, cs[i]) + mv(Ui, mv(Dinvi, ui))
            R, p = li[i]
            X = X_actinv(R, p)
            Ya[par] = Ya[par] + mtm(X, mm(Ia, X))
            pA[par] = pA[par] + act_force(R, p, pa)
    g = np.zeros(shape + (6,), dtype=dt)
    g[..., :3] = -M.gravity
    ddq = np.zeros(shape + (M.nv,), dtype=np.result_type(dt, pA[1]))
    acc = [None] * nb
    for i in range(1, nb):
        R, p = li[i]
        par = M.parent[i]
        S = _S(M, i, shape, dt)
        iv = M.idx_v[i]
        nvi = S.shape[1]
        ai = act_inv_motion(R, p, g if par == 0 else acc[par]) + cs[i]
        qdd = mv(Dinv[i], u[i] - np.einsum("...ji,...j->...i", U[i], ai))
        ddq[..., iv:iv + nvi] = qdd
        acc[i] = ai + np.einsum("ij,...j->...i", S, qdd)
    return ddq


def crba(M: ModelArrays, q):
    """Composite-rigid-body algorithm (joint-space mass matrix), independent of rnea()."""
    li, _ = forward_kinematics(M, q)
    shape = q.shape[:-1]
    Yc = [np.broadcast_to(M.Y6[i], shape + (6, 6)).copy() for i in range(M.nj)]
    Mq = np.zeros(shape + (M.nv, M.nv), dtype=q.dtype)  # complex under the complex-step Jacobian
    for i in range(M.nj - 1, 0, -1):
        Si = _S(M, i, shape, float)
        iv, nvi = M.idx_v[i], Si.shape[1]
        F = np.einsum("...ij,jk->...ik", Yc[i], Si)
        Mq[..., iv:iv + nvi, iv:iv + nvi] = np.einsum("ji,...jk->...ik", Si, F)
        j = i
        while M.parent[j] > 0:
            R, p = li[j]
            F = mtm(X_actinv(R, p), F)
            j = M.parent[j]
            Sj = _S(M, j, shape, float)
            jv, nvj = M.idx_v[j], Sj.shape[1]
            blk = np.einsum("ji,...jk->...ik", Sj, F)
            Mq[..., jv:jv + nvj, iv:iv + nvi] = blk
            Mq[..., iv:iv + nvi, jv:jv + nvj] = np.swapaxes(blk, -1, -2)
        par = M.parent[i]
        if par > 0:
            R, p = li[i]
            X = X_actinv(R, p)
            Yc[par] = Yc[par] + mtm(X, mm(Yc[i], X))
    return Mq


def joint_velocities(M: ModelArrays, q, v):
    li, oM = forward_kinematics(M, q)
    vs = [None] * M.nj
    for i in range(1, M.nj):
        R, p = li[i]
        par = M.parent[i]
        vJ = joint_vel(M, i, v)
        vs[i] = vJ if par == 0 else act_inv_motion(R, p, vs[par]) + vJ
    return li, oM, vs


def frame_placement(M: ModelArrays, oM, fid):
    j, Rf, pf = M.frame(fid)
    Ro, po = oM[j]
    return mm(Ro, np.broadcast_to(Rf, Ro.shape)), po + mv(Ro, np.broadcast_to(pf, po.shape))


def frame_velocity_lwa(M: ModelArrays, oM, vs, fid):
    """getFrameVelocity(..., LOCAL_WORLD_ALIGNED) (dynamics/dynamics.py:82-84)."""
    j, Rf, pf = M.frame(fid)
    Ro, _ = oM[j]
    vj = vs[j]
    lin = mv(Ro, vj[..., :3] + cross(vj[..., 3:], np.broadcast_to(pf, vj[..., :3].shape)))
    return np.concatenate([lin, mv(Ro, vj[..., 3:])], -1)


def frame_velocity(M: ModelArrays, q, v, fid, relative_to_base=False, base_fid=None):
    """Dynamics.get_frame_velocity (dynamics/dynamics.py:77-118)."""
    li, oM, vs = joint_velocities(M, q, v)
    fv = frame_velocity_lwa(M, oM, vs, fid)
    if not relative_to_base:
        return fv
    bv = frame_velocity_lwa(M, oM, vs, base_fid)
    Rb, pb = frame_placement(M, oM, base_fid)
    _, pfw = frame_placement(M, oM, fid)
    rel = pfw - pb
    corr = cross(bv[..., 3:], rel)
    rl = fv[..., :3] - bv[..., :3] - corr
    ra = fv[..., 3:] - bv[..., 3:]
    rlb = mtv(Rb, rl)
    rab = mtv(Rb, ra)
    return np.stack([rlb[..., 0], rlb[..., 1], fv[..., 2], rab[..., 0], rab[..., 1], fv[..., 5]], -1)


def contact_fext(M: ModelArrays, oM, frames, forces):
    """World-frame point forces -> joint-local f_ext (dynamics_whole_body_torque.py:55-69).

    A later frame on the same joint overwrites an earlier one, as in the reference.
    """
    fext = [None] * M.nj
    for idx, fid in enumerate(frames):
        j, _, pf = M.frame(fid)
        Ro, _ = oM[j]
        fw = forces[..., 3 * idx:3 * idx + 3]
        flin = mtv(Ro, fw)
        fang = cross(np.broadcast_to(pf, flin.shape), flin)
        fext[j] = np.concatenate([flin, fang], -1)
    return fext


def rnea_dynamics(M, frames, q, v, a, forces):
    _, oM = forward_kinematics(M, q)
    return rnea(M, q, v, a, contact_fext(M, oM, frames, forces))


def aba_dynamics(M, frames, q, v, tau_j, forces):
    _, oM = forward_kinematics(M, q)
    tau = np.concatenate([np.zeros(q.shape[:-1] + (6,), dtype=tau_j.dtype), tau_j], -1)
    return aba(M, q, v, tau, contact_fext(M, oM, frames, forces))


def frame_jacobian_lwa(M: ModelArrays, q, fid):
    """computeFrameJacobian(LOCAL_WORLD_ALIGNED) via the linear map v -> frame velocity."""
    cols = [frame_velocity(M, q, np.eye(M.nv)[k], fid) for k in range(M.nv)]
    return np.stack(cols, -1)


def integrate(M: ModelArrays, q, dq):
    """pinocchio::integrate for free-flyer + revolute joints (LieGroup SE3 / R)."""
    out = np.zeros(np.broadcast(q, dq[..., :1]).shape[:-1] + (M.nq,), dtype=np.result_type(q, dq))
    for i in range(1, M.nj):
        iq, iv = M.idx_q[i], M.idx_v[i]
        if M.jtype[i] == JT_FREEFLYER:
            quat0 = q[..., iq + 3:iq + 7]
            R0 = quat_to_matrix(quat0)
            p0 = q[..., iq:iq + 3]
            Rx, tx = exp6(dq[..., iv:iv + 6])
            R1 = mm(R0, Rx)
            p1 = p0 + mv(R0, tx)
            qu = matrix_to_quat(R1)
            dot = np.sum(qu * quat0, -1)
            qu = np.where((dot.real < 0)[..., None], -qu, qu)
            n2 = np.sum(qu * qu, -1)
            qu = qu * ((3.0 - n2) / 2.0)[..., None]
            out[..., iq:iq + 3] = p1
            out[..., iq + 3:iq + 7] = qu
        else:
            out[..., iq] = q[..., iq] + dq[..., iv]
    return out


def difference(M: ModelArrays, q0, q1):
    out = np.zeros(np.broadcast(q0, q1).shape[:-1] + (M.nv,), dtype=np.result_type(q0, q1))
    for i in range(1, M.nj):
        iq, iv = M.idx_q[i], M.idx_v[i]
        if M.jtype[i] == JT_FREEFLYER:
            R0 = quat_to_matrix(q0[..., iq + 3:iq + 7])
            R1 = quat_to_matrix(q1[..., iq + 3:iq + 7])
            p0, p1 = q0[..., iq:iq + 3], q1[..., iq:iq + 3]
            R = mtm(R0, R1)
            p = mtv(R0, p1 - p0)
            out[..., iv:iv + 6] = log6(R, p)
        else:
            out[..., iv] = q1[..., iq] - q0[..., iq]
    return out


def center_of_mass(M: ModelArrays, q):
    _, oM = forward_kinematics(M, q)
    acc = 0.0
    for i in range(1, M.nj):
        Ro, po = oM[i]
        acc = acc + M.mass[i] * (po + mv(Ro, np.broadcast_to(M.lever[i], po.shape)))
    return acc / M.total_mass


def centroidal_momentum(M: ModelArrays, q, v):
    """h_G = A_G(q) v (linear first, world axes, about the CoM)."""
    li, oM, vs = joint_velocities(M, q, v)
    com = center_of_mass(M, q)
    h = 0.0
    for i in range(1, M.nj):
        Ro, po = oM[i]
        hl = inertia_mul(M.mass[i], M.lever[i], M.Ic[i], vs[i])
        h = h + act_force(Ro, po - com, hl)
    return h


def centroidal_map(M: ModelArrays, q):
    """computeCentroidalMap: A_G(q) (6 x nv), columns h_G(q, e_k)."""
    return np.stack([centroidal_momentum(M, q, np.eye(M.nv)[k]) for k in range(M.nv)], -1)


def dccrba_v(M: ModelArrays, q, v, h=1e-30):
    """pinocchio dccrba(q, v) applied to v: d/dt A_G(q(t)) v along q(t) = q (+) t v,
    by complex step through the Lie-group integrate (dynamics_centroidal_vel.py:110)."""
    qc = integrate(M, q.astype(complex), 1j * h * v.astype(complex))
    return (centroidal_map(M, qc) @ v).imag / h


def com_dynamics(M: ModelArrays, frames, q, forces, mass, scale=True):
    """DynamicsCentroidalVel.com_dynamics (dynamics_centroidal_vel.py:43-71):
    [sum f + (0, 0, -9.81 m), sum (p_e - com) x f_e] (/ m when scale)."""
    _, oM = forward_kinematics(M, q)
    com = center_of_mass(M, q)
    fs = [forces[..., 3 * k:3 * k + 3] for k in range(len(frames))]
    dp = sum(fs) + np.array([0, 0, -9.81 * mass])
    dl = 0
    for k, fid in enumerate(frames):
        _, pf = frame_placement(M, oM, fid)
        dl = dl + cross(pf - com, fs[k])
    out = np.concatenate([dp, dl], -1)
    return out / mass if scale else out


def base_vel_cv(M: ModelArrays, h, q, v_j, mass):
    """base_vel_dynamics (dynamics_centroidal_vel.py:73-89): A_b^-1 (m h - A_j v_j)."""
    A = centroidal_map(M, q)  # (..., 6, nv); h, v_j may carry the same leading dims
    rhs = h * mass - (A[..., :, 6:] @ np.asarray(v_j)[..., None])[..., 0]
    return np.linalg.solve(A[..., :, :6], rhs[..., None])[..., 0]


def base_acc_cv(M: ModelArrays, frames, q, v, a_j, forces, mass):
    """base_acc_dynamics (dynamics_centroidal_vel.py:91-134): A_b^-1 (dh - dA v - A_j a_j)."""
    A = centroidal_map(M, q)
    dh = com_dynamics(M, frames, q, forces, mass, scale=False)
    return np.linalg.solve(A[:, :6], dh - dccrba_v(M, q, v) - A[:, 6:] @ a_j)


def base_acc_wb(M: ModelArrays, frames, q, v, a_j, forces):
    """DynamicsWholeBodyAcc.base_acc_dynamics (dynamics_whole_body_acc.py:43-83):
    M_bb^-1 (-nle_b - M_bj a_j + sum_k J_c,k[:3, :6]^T f_k) with crba, nonLinearEffects
    and computeFrameJacobian(LOCAL_WORLD_ALIGNED)."""
    Mq = crba(M, q)
    nle = rnea(M, q, v, np.zeros_like(v))
    tb = sum(np.einsum("...ji,...j->...i", frame_jacobian_lwa(M, q, fid)[..., :3, :6], forces[..., 3 * k:3 * k + 3])
             for k, fid in enumerate(frames))
    rhs = -nle[..., :6] - np.einsum("...ij,...j->...i", Mq[..., :6, 6:], a_j) + tb
    return np.linalg.solve(Mq[..., :6, :6], rhs[..., None])[..., 0]


def ab_inv_ocs2(Ab):
    """OCS2 closed form of A_b^-1 (DynamicsCentroidalVel._compute_Ab_inv,
    dynamics_centroidal_vel.py:150-159)."""
    m = Ab[0, 0]
    A22i = np.linalg.inv(Ab[3:, 3:])
    out = np.zeros((6, 6))
    out[:3, :3] = np.eye(3) / m
    out[:3, 3:] = -Ab[:3, 3:] @ A22i / m
    out[3:, 3:] = A22i
    return out


def momentum_rate(M: ModelArrays, q, v, a):
    """A_G(q) a + dA_G(q, v) v (computeCentroidalMap, dccrba): the rate of the centroidal
    momentum, as the Newton-Euler sum of the body wrenches without gravity: the root's
    subtree force of a zero-gravity RNEA, moved to world axes and then to the CoM.
    Arithmetic only (safe under the complex-step Jacobian); pinned against
    centroidal_map(q) a + dccrba_v(q, v) in tests/test_oracle.py."""
    f_root = rnea(M, q, v, a, gravity=False)[..., :6]
    li, oM = forward_kinematics(M, q)
    R, p = oM[1]
    f = act_force(R, p, f_root)  # world axes, about the world origin
    com = center_of_mass(M, q)
    return np.concatenate([f[..., :3], f[..., 3:] - cross(com, f[..., :3])], -1)


def base_acc_ca(M: ModelArrays, frames, q, v, a_j, forces, mass):
    """DynamicsCentroidalAcc.base_acc_dynamics (dynamics_centroidal_acc.py:43-90):
    A_b^-1 (dh - dA v - A_j a_j), with A [0; a_j] + dA v as momentum_rate(q, v, [0; a_j])."""
    A = centroidal_map(M, q)
    dh = com_dynamics(M, frames, q, forces, mass, scale=False)
    a0 = np.concatenate([np.zeros(a_j.shape[:-1] + (6,), dtype=a_j.dtype), a_j], -1)
    rhs = dh - momentum_rate(M, q, v, a0)
    return np.linalg.solve(A[..., :, :6], rhs[..., None])[..., 0]


def gaps_ca(M: ModelArrays, frames, q, v, a, forces, mass):
    """DynamicsCentroidalAcc.dynamics_gaps (dynamics_centroidal_acc.py:92-119):
    A a + dA v - dh."""
    return momentum_rate(M, q, v, a) - com_dynamics(M, frames, q, forces, mass, scale=False)
