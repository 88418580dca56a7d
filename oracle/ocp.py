"""ORACLE (test infrastructure only) -- the reference's OCP/SQP(OSQP) path restated in numpy.

Restates, node by node and row by row, what the reference builds symbolically with
CasADi Opti and evaluates with its MX virtual machine:

* decision vector ``[dx_0, u_0, ..., dx_{N-1}, u_{N-1}, dx_N]``
  (``ocp_whole_body_rnea.py:79-84``);
* parameter vector in Opti declaration order (``ocp.py:54-69``,
  ``ocp_whole_body_rnea.py:88-89``), matrices column-major;
* constraint rows in ``subject_to`` order (``ocp.py:103-190`` and each subclass's
  ``setup_dynamics_constraints``);
* objective (``ocp.py:80-101``, ``ocp_whole_body_rnea.py:108-136``), constant
  Hessian diagonal (``ocp.py:293-296``);
* one SQP iteration with OSQP and the Armijo/filter line search
  (``ocp.py:375-480``), retract (``ocp_whole_body_rnea.py:293-324``), warm start
  (``ocp_whole_body_rnea.py:207-235``) and the MPC loop (``run_mpc.py:115-143``).

Jacobians are complex-step derivatives of the row functions (exact to round-off),
an independent technique from the forward-mode duals the HIP kernels use.

Row canonicalisation: an inequality ``a >= b`` is kept as ``g = b - a <= 0`` only
when both sides depend on x, otherwise as ``lb <= g`` with the parameter side as
the bound.  CasADi's own canonical form may flip a row's sign or move a parameter
between g and its bounds; the QP (l - g, u - g, rows of A up to sign) and the
violation metrics are invariant to both, so parity is checked at the QP level.
PARITY UNPINNED (no CasADi/Pinocchio/OSQP in this container, no reference fixtures).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

from . import rbd
from .osqp_ref import OSQPRef, REFERENCE_SETTINGS

INF = np.inf
GRAV = 9.81


def spline_vel_z(phase, period, h_max, v_lo, v_td):
    """get_spline_vel_z / CubicSpline (utils/gait_sequence.py:96-133)."""
    mid = period / 2

    def coeffs(t0, t1, p0, v0, p1, v1):
        dt = t1 - t0
        dpos, dvel = p1 - p0, v1 - v0
        return t0, dt, v0 * dt, -(3.0 * v0 + dvel) * dt + 3.0 * dpos, (2.0 * v0 + dvel) * dt - 2.0 * dpos

    def vel(c, t):
        t0, dt, c1, c2, c3 = c
        tn = (t - t0) / dt
        return (3.0 * c3 * tn ** 2 + 2.0 * c2 * tn + c1) / dt

    s1 = coeffs(0, mid, 0, v_lo, h_max, 0)
    s2 = coeffs(mid, period, h_max, 0, 0, v_td)
    t = phase * period
    return np.where(np.asarray(phase).real < 0.5, vel(s1, t), vel(s2, t))


class OracleOCP:
    """One OCP instance (= one problem) with the reference's semantics."""

    def __init__(self, robot, dynamics, nodes, tau_nodes=3, include_acc=True, include_base=True, mu=0.7,
                 osqp_settings=None, kkt="quasi_definite"):
        self.robot = robot
        self.dynamics = dynamics
        self.N = nodes
        self.mu = mu
        self.M = rbd.ModelArrays(robot.model)
        self.nq, self.nv, self.nj, self.nf = robot.nq, robot.nv, robot.nj, robot.nf
        self.mass = robot.model.total_mass()
        self.feet = list(robot.foot_frames)
        self.ext = robot.ext_force_frame
        self.arm = robot.arm_ee_frame
        self.base_fid = robot.model.get_frame_id("base_link")
        self.ee_frames = self.feet + ([self.ext] if self.ext is not None else [])
        self.tau_nodes = tau_nodes if dynamics == "whole_body_rnea" else 0
        self.include_acc = include_acc
        self.include_base = include_base
        nv, nj, nf = self.nv, self.nj, self.nf
        if dynamics == "whole_body_rnea":
            self.nx, self.ndx = self.nq + nv, 2 * nv
            na = nv if include_acc else 0
            self.na = na
            self.nu = [na + nf + nj] * tau_nodes + [na + nf] * (nodes - tau_nodes)
        elif dynamics in ("whole_body_acc", "centroidal_acc"):
            # u = [a | f] (include_base) or [a_j | f] with the base acceleration from the
            # dynamics (ocp_whole_body_acc.py:56-63, 124-135; ocp_centroidal_acc.py:15-19)
            self.nx, self.ndx = self.nq + nv, 2 * nv
            self.na = nv if include_base else nj
            self.nu = [self.na + nf] * nodes
        elif dynamics == "whole_body_aba":
            self.nx, self.ndx = self.nq + nv, 2 * nv
            self.nu = [nj + nf] * nodes
        elif dynamics == "centroidal_vel":
            # u = [v | f] (include_base) or [v_j | f] (ocp_centroidal_vel.py:19-23, 56-57)
            self.nx, self.ndx = 6 + self.nq, 6 + nv
            self.nv_opt = nv if include_base else nj
            self.nu = [self.nv_opt + nf] * nodes
        else:
            raise ValueError(f"Unknown dynamics type: {dynamics}")
        self.x_off = []
        off = 0
        for i in range(nodes):
            self.x_off.append(off)
            off += self.ndx + self.nu[i]
        self.x_off.append(off)
        self.n = off + self.ndx
        self._pinfo = self._param_layout()
        self.osqp_settings = dict(REFERENCE_SETTINGS if osqp_settings is None else osqp_settings)
        self.kkt = kkt  # "reduced_block": the GPU's linear algebra (osqp_ref.BlockReduced), a diagnostic
        self.pattern = None
        self.osqp = None
        self.hess_diag = None

    # ------------------------------------------------------------------ params
    def _param_layout(self):
        N, ndx = self.N, self.ndx
        items = [("x_init", self.nx), ("dt_min", 1), ("dt_max", 1), ("contact", 4 * N), ("swing", 4 * N),
                 ("n_contacts", 1), ("swing_period", 1), ("swing_height", 1), ("swing_vel_limits", 2),
                 ("Q_diag", ndx), ("R_diag", self.nu[0]), ("base_vel_des", 6), ("ext_force_des", 3),
                 ("arm_vel_des", 3)]
        if self.dynamics == "whole_body_rnea":
            items += [("tau_prev", self.nj), ("W_diag", self.nj)]
        lay, off = {}, 0
        for k, s in items:
            lay[k] = (off, s)
            off += s
        self.np_ = off
        return lay

    def pack_params(self, **kw):
        p = np.zeros(self.np_)
        for k, (o, s) in self._pinfo.items():
            if k in kw and kw[k] is not None:
                v = np.asarray(kw[k], dtype=float)
                if k in ("contact", "swing"):
                    v = v.reshape(4, self.N).T.ravel()  # column-major 4xN
                p[o:o + s] = v.ravel()
        return p

    def unpack(self, p):
        d = {k: p[o:o + s] for k, (o, s) in self._pinfo.items()}
        d["contact"] = d["contact"].reshape(self.N, 4).T
        d["swing"] = d["swing"].reshape(self.N, 4).T
        d["dt_min"], d["dt_max"] = float(d["dt_min"][0]), float(d["dt_max"][0])
        for k in ("n_contacts", "swing_period", "swing_height"):
            d[k] = float(d[k][0])
        ratio = d["dt_max"] / d["dt_min"]
        gamma = ratio ** (1 / (self.N - 1))
        d["dts"] = [d["dt_min"] * gamma ** i for i in range(self.N)]
        return d

    def default_weights(self):
        """set_weights of each subclass (ocp_whole_body_rnea.py:28-63 etc.)."""
        nj, nf = self.nj, self.nf
        Qb = [0, 0, 1000, 10000, 10000, 0]
        Qj = list(np.tile([1000, 500, 500], 4))
        if self.arm is not None:
            Qj += [100] * 6
        Qv = [2000, 2000, 1000, 1000, 1000, 2000] + [1] * nj
        if self.dynamics == "centroidal_vel":
            Q = [1000] * 6 + Qb + Qj
            R = [1] * self.nv_opt + [1e-3] * nf
        else:
            Q = Qb + Qj + Qv
            if self.dynamics == "whole_body_rnea":
                R = [1e-3] * self.na + [1e-3] * nf + [1e-4] * nj
            elif self.dynamics in ("whole_body_acc", "centroidal_acc"):
                R = [1e-3] * self.na + [1e-3] * nf
            else:
                R = [1e-3] * nj + [1e-3] * nf
        W = [0.0] * nj
        return np.array(Q, float), np.array(R, float), np.array(W, float)

    # ------------------------------------------------------------------ targets
    def f_des(self, P):
        fg = GRAV * self.mass
        fr = 0.8 * fg / P["n_contacts"]
        rr = 1.2 * fg / P["n_contacts"]
        v = [0, 0, fr, 0, 0, fr, 0, 0, rr, 0, 0, rr]
        if self.ext is not None:
            v += [0, 0, 0]
        return np.array(v, float)

    def u_des(self, P):
        fd = self.f_des(P)
        if self.dynamics == "whole_body_rnea":
            return np.concatenate([np.zeros(self.na), fd, np.zeros(self.nj)])
        if self.dynamics in ("whole_body_acc", "centroidal_acc"):
            return np.concatenate([np.zeros(self.na), fd])
        if self.dynamics == "whole_body_aba":
            return np.concatenate([np.zeros(self.nj), fd])
        return np.concatenate([np.zeros(self.nv_opt), fd])

    def dx_des(self, P):
        xi = P["x_init"]
        nq, nv, nj = self.nq, self.nv, self.nj
        q0 = self.robot.q0
        if self.dynamics == "centroidal_vel":
            h_des = P["base_vel_des"]
            dq = rbd.difference(self.M, xi[6:], q0)
            return np.concatenate([h_des - xi[:6], dq])
        dq = rbd.difference(self.M, xi[:nq], q0)
        v_des = np.concatenate([P["base_vel_des"], np.zeros(nj)])
        return np.concatenate([dq, v_des - xi[nq:]])

    # ------------------------------------------------------------------ x helpers
    def split(self, x):
        DX, U = [], []
        for i in range(self.N):
            o = self.x_off[i]
            DX.append(x[..., o:o + self.ndx])
            U.append(x[..., o + self.ndx:o + self.ndx + self.nu[i]])
        DX.append(x[..., self.x_off[self.N]:self.x_off[self.N] + self.ndx])
        return DX, U

    def state(self, dx, P):
        """get_q / get_v (or get_h / get_q for centroidal_vel)."""
        xi = P["x_init"]
        if self.dynamics == "centroidal_vel":
            h = xi[:6] + dx[..., :6]
            q = rbd.integrate(self.M, xi[6:], dx[..., 6:])
            return h, q
        q = rbd.integrate(self.M, xi[:self.nq], dx[..., :self.nv])
        v = xi[self.nq:] + dx[..., self.nv:]
        return q, v

    # ------------------------------------------------------------------ rows
    def node_rows(self, i, dx, u, dx_next, P):
        """Rows of node i in subject_to order -> list of (g, lb, ub) with leading batch dims."""
        nv, nj, nf, nq = self.nv, self.nj, self.nf, self.nq
        shp = dx.shape[:-1]
        dt = P["dts"][i]
        rows = []

        def add(g, lb, ub):
            g = np.asarray(g)
            if g.ndim == len(shp):
                g = g[..., None]
            k = g.shape[-1]
            rows.append((g, np.broadcast_to(np.asarray(lb, float), (k,)).copy(),
                         np.broadcast_to(np.asarray(ub, float), (k,)).copy()))

        dyn = self.dynamics
        if dyn == "centroidal_vel":
            h, q = self.state(dx, P)
            if self.include_base:
                v = u[..., :nv]
            else:  # get_v: v_b = base_vel_dynamics(h, q, v_j) (ocp_centroidal_vel.py:119-129)
                v_j = u[..., :nj]
                v = np.concatenate([rbd.base_vel_cv(self.M, h, q, v_j, self.mass), v_j], -1)
            forces = u[..., self.nv_opt:]
        else:
            q, v = self.state(dx, P)
        if dyn == "whole_body_rnea":
            forces = u[..., self.na:self.na + nf]
            tau_j = u[..., self.na + nf:]
            add(dx_next[..., :nv] - (dx[..., :nv] + v * dt), 0, 0)
            if self.include_acc:
                a = u[..., :nv]
                add(dx_next[..., nv:] - (dx[..., nv:] + a * dt), 0, 0)
            else:  # get_a: finite difference, no dv row (ocp_whole_body_rnea.py:157-159, 183-191)
                _, v_next = self.state(dx_next, P)
                a = (v_next - v) / dt
            tau = rbd.rnea_dynamics(self.M, self.ee_frames, q, v, a, forces)
            add(tau[..., :6], 0, 0)
            if i < self.tau_nodes:
                add(tau[..., 6:] - tau_j, 0, 0)
                tmax = self.robot.joint_torque_max
                add(tau_j, -tmax, tmax)
        elif dyn in ("whole_body_acc", "centroidal_acc"):
            forces = u[..., self.na:]
            if self.include_base:
                a = u[..., :nv]
            else:  # get_a (ocp_whole_body_acc.py:124-135, ocp_centroidal_acc.py:123-134)
                a_j = u[..., :nj]
                if dyn == "whole_body_acc":
                    a_b = rbd.base_acc_wb(self.M, self.ee_frames, q, v, a_j, forces)
                else:
                    a_b = rbd.base_acc_ca(self.M, self.ee_frames, q, v, a_j, forces, self.mass)
                a = np.concatenate([a_b, a_j], -1)
            add(dx_next[..., :nv] - (dx[..., :nv] + v * dt), 0, 0)
            add(dx_next[..., nv:] - (dx[..., nv:] + a * dt), 0, 0)
            if self.include_base:
                if dyn == "whole_body_acc":  # dynamics_gaps = RNEA base rows
                    tau = rbd.rnea_dynamics(self.M, self.ee_frames, q, v, a, forces)
                    add(tau[..., :6], 0, 0)
                else:  # A a + dA v - dh (dynamics_centroidal_acc.py:92-119)
                    add(rbd.gaps_ca(self.M, self.ee_frames, q, v, a, forces, self.mass), 0, 0)
        elif dyn == "whole_body_aba":
            tau_j = u[..., :nj]
            forces = u[..., nj:]
            a = rbd.aba_dynamics(self.M, self.ee_frames, q, v, tau_j, forces)
            add(dx_next[..., :nv] - (dx[..., :nv] + v * dt), 0, 0)
            add(dx_next[..., nv:] - (dx[..., nv:] + a * dt), 0, 0)
        else:  # centroidal_vel
            hdot = self._com_dynamics(q, forces)
            add(dx_next[..., :6] - (dx[..., :6] + hdot * dt), 0, 0)
            add(dx_next[..., 6:] - (dx[..., 6:] + v * dt), 0, 0)
            if self.include_base:  # dynamics_gaps (ocp_centroidal_vel.py:104-107)
                hg = rbd.centroidal_momentum(self.M, q, v)
                add(hg - h * self.mass, 0, 0)

        skip_state = (i == 0 and dyn != "centroidal_vel")
        fvel = None
        if not skip_state:
            li, oM, vs = rbd.joint_velocities(self.M, q, v)
        mu2 = self.mu ** 2
        for k, fid in enumerate(self.feet):
            fe = forces[..., 3 * k:3 * k + 3]
            c = P["contact"][k, i]
            ph = P["swing"][k, i]
            add(c * fe[..., 2], 0, INF)
            add(c * (fe[..., 0] ** 2 + fe[..., 1] ** 2) - c * mu2 * fe[..., 2] ** 2, -INF, 0)
            add((1 - c) * fe, 0, 0)
            if skip_state:
                continue
            vel = rbd.frame_velocity_lwa(self.M, oM, vs, fid)
            add(c * vel[..., :2], 0, 0)
            vz_des = spline_vel_z(ph, P["swing_period"], P["swing_height"],
                                  P["swing_vel_limits"][0], P["swing_vel_limits"][1])
            add(c * vel[..., 2] + (1 - c) * (vel[..., 2] - vz_des), 0, 0)
        if self.ext is not None:
            fe = forces[..., 3 * len(self.feet):]
            add(fe - P["ext_force_des"], 0, 0)
        if skip_state:
            return rows
        if self.arm is not None:
            vel = rbd.frame_velocity(self.M, q, v, self.arm, relative_to_base=True, base_fid=self.base_fid)
            add(vel[..., :3] - P["arm_vel_des"], 0, 0)
        add(q[..., 7:], self.robot.joint_pos_min, self.robot.joint_pos_max)
        add(v[..., 6:], -self.robot.joint_vel_max, self.robot.joint_vel_max)
        return rows

    def _com_dynamics(self, q, forces):
        """DynamicsCentroidalVel.com_dynamics (dynamics_centroidal_vel.py:43-71)."""
        _, oM = rbd.forward_kinematics(self.M, q)
        com = rbd.center_of_mass(self.M, q)
        nfe = len(self.ee_frames)
        fs = [forces[..., 3 * k:3 * k + 3] for k in range(nfe)]
        dp = sum(fs) + np.array([0, 0, -GRAV * self.mass])
        dl = 0
        for k, fid in enumerate(self.ee_frames):
            _, pf = rbd.frame_placement(self.M, oM, fid)
            dl = dl + rbd.cross(pf - com, fs[k])
        return np.concatenate([dp, dl], -1) / self.mass

    def _node_io(self, x, i):
        DX, U = self.split(x)
        return DX[i], U[i], DX[i + 1]

    def eval_g(self, x, p):
        """g_data(x, p) -> g, lbg, ubg (ocp.py:290)."""
        P = self.unpack(p)
        DX, U = self.split(x)
        gs, ls, us = [DX[0]], [np.zeros(self.ndx)], [np.zeros(self.ndx)]
        for i in range(self.N):
            for g, lb, ub in self.node_rows(i, DX[i], U[i], DX[i + 1], P):
                gs.append(g)
                ls.append(lb)
                us.append(ub)
        return np.concatenate(gs, -1), np.concatenate(ls), np.concatenate(us)

    def node_row_count(self, i, P):
        z = np.zeros(self.ndx)
        return sum(r[0].shape[-1] for r in self.node_rows(i, z, np.zeros(self.nu[i]), z, P))

    def eval_J(self, x, p, h=1e-30):
        """Constraint Jacobian by complex step, node block by node block -> csc (m x n)."""
        P = self.unpack(p)
        DX, U = self.split(x)
        rows, cols, vals = [], [], []
        ndx = self.ndx
        for k in range(ndx):
            rows.append(k)
            cols.append(k)
            vals.append(1.0)
        r0 = ndx
        for i in range(self.N):
            nu = self.nu[i]
            nin = ndx + nu + ndx
            base = np.concatenate([DX[i], U[i], DX[i + 1]])
            pert = np.broadcast_to(base, (nin, nin)).astype(complex) + 1j * h * np.eye(nin)
            out = self.node_rows(i, pert[:, :ndx], pert[:, ndx:ndx + nu], pert[:, ndx + nu:], P)
            G = np.concatenate([np.broadcast_to(g, (nin, g.shape[-1])) for g, _, _ in out], -1)
            Jn = G.imag.T / h  # (rows_i x nin)
            colmap = np.concatenate([np.arange(self.x_off[i], self.x_off[i] + ndx + nu),
                                     np.arange(self.x_off[i + 1], self.x_off[i + 1] + ndx)])
            rr, cc = np.nonzero(Jn)
            rows.extend((rr + r0).tolist())
            cols.extend(colmap[cc].tolist())
            vals.extend(Jn[rr, cc].tolist())
            r0 += Jn.shape[0]
        return sp.csc_matrix((vals, (rows, cols)), shape=(r0, self.n))

    def lag_hess(self, x, p, lam, delta=1e-3):
        """Lagrangian Hessian sum_r lam_r d^2 g_r / dx^2 (csr, n x n) -- the constraint part of
        the exact Hessian CasADi gives the reference's Opti/Fatrop solve (ocp.py:248-263).
        The rows of node i are linear in dx_{i+1} (the integration rows), so it is block
        diagonal over the w_i = [dx_i, u_i].  Entry (j, k) of block i: the complex-step
        derivative of lam_i^T g_i along w_j, differentiated along w_k by the fourth-order
        central difference [-f(+2d) + 8 f(+d) - 8 f(-d) + f(-2d)] / (12 d) (an independent
        technique from the GPU's hyper-dual numbers; ~1e-12 relative).  The rnea tau_j
        columns enter linearly and are skipped."""
        P = self.unpack(p)
        DX, U = self.split(x)
        h = 1e-30
        ndx = self.ndx
        rows, cols, vals = [], [], []
        r0 = ndx
        for i in range(self.N):
            nu = self.nu[i]
            nw = ndx + nu
            nr = self.node_row_count(i, P)
            li = lam[r0:r0 + nr]
            r0 += nr
            lin = nw
            if self.dynamics == "whole_body_rnea":
                lin = ndx + self.na + self.nf
            jj, kk = np.tril_indices(lin)  # j <= k pairs (kk >= jj after the swap below)
            jj, kk = kk, jj
            jj, kk = np.minimum(jj, kk), np.maximum(jj, kk)
            base = np.concatenate([DX[i], U[i], DX[i + 1]])
            npair = jj.size
            steps = np.array([2.0, 1.0, -1.0, -2.0]) * delta
            wts = np.array([-1.0, 8.0, -8.0, 1.0]) / (12.0 * delta)
            pert = np.broadcast_to(base, (4, npair, base.size)).astype(complex).copy()
            ar = np.arange(npair)
            for s in range(4):
                pert[s, ar, jj] += 1j * h
                pert[s, ar, kk] += steps[s]
            pert = pert.reshape(4 * npair, base.size)
            out = self.node_rows(i, pert[:, :ndx], pert[:, ndx:nw], pert[:, nw:], P)
            G = np.concatenate([np.broadcast_to(g, (4 * npair, g.shape[-1])) for g, _, _ in out], -1)
            dphi = (G.imag @ li / h).reshape(4, npair)
            Hjk = wts @ dphi
            off = self.x_off[i]
            rows.extend((off + kk).tolist())
            cols.extend((off + jj).tolist())
            vals.extend(Hjk.tolist())
            low = jj != kk
            rows.extend((off + jj[low]).tolist())
            cols.extend((off + kk[low]).tolist())
            vals.extend(Hjk[low].tolist())
        return sp.csr_matrix((vals, (rows, cols)), shape=(self.n, self.n))

    def structural_pattern(self, p):
        """Jacobian pattern from randomised inputs (contacts toggled) -- superset of
        every numeric pattern the solve can produce.  Used as the OSQP A pattern."""
        rng = np.random.default_rng(7)
        P = self.unpack(p)
        pats = []
        for trial in range(2):
            pp = p.copy()
            lay = self._pinfo
            o, s = lay["contact"]
            pp[o:o + s] = 0.5 + 0.1 * trial
            x = rng.normal(size=self.n) * 0.1
            for i in range(self.N):
                o = self.x_off[i] + self.ndx
                x[o:o + self.nu[i]] += self.u_des(P)[:self.nu[i]]
            J = self.eval_J(x, pp)
            J.data[:] = 1.0
            pats.append(J)
        pat = (pats[0] + pats[1]).tocsc()
        pat.data[:] = 1.0
        return pat

    # ------------------------------------------------------------------ objective
    def f_and_grad(self, x, p):
        P = self.unpack(p)
        DX, U = self.split(x)
        Q, R = P["Q_diag"], P["R_diag"]
        dxd = self.dx_des(P)
        ud = self.u_des(P)
        f = 0.0
        grad = np.zeros(self.n)
        nu0 = self.nu[0]
        for i in range(self.N):
            e = DX[i] - dxd
            f += e @ (Q * e)
            grad[self.x_off[i]:self.x_off[i] + self.ndx] = 2 * Q * e
            ui = U[i]
            upad = np.concatenate([ui, np.zeros(nu0 - ui.size)])
            eu = upad - ud
            f += eu @ (R * eu)
            o = self.x_off[i] + self.ndx
            grad[o:o + ui.size] = (2 * R * eu)[:ui.size]
        if self.dynamics == "whole_body_rnea":
            ti = self.na + self.nf
            t0 = U[0][ti:]
            et = t0 - P["tau_prev"]
            f += et @ (P["W_diag"] * et)
            o = self.x_off[0] + self.ndx + ti
            grad[o:o + self.nj] += 2 * P["W_diag"] * et
        e = DX[self.N] - dxd
        f += e @ (Q * e)
        grad[self.x_off[self.N]:] = 2 * Q * e
        return f, grad

    def compute_hess_diag(self, p):
        P = self.unpack(p)
        h = np.zeros(self.n)
        for i in range(self.N + 1):
            h[self.x_off[i]:self.x_off[i] + self.ndx] = 2 * P["Q_diag"]
            if i < self.N:
                o = self.x_off[i] + self.ndx
                h[o:o + self.nu[i]] = 2 * P["R_diag"][:self.nu[i]]
        if self.dynamics == "whole_body_rnea":
            o = self.x_off[0] + self.ndx + self.na + self.nf
            h[o:o + self.nj] += 2 * P["W_diag"]
        return h

    # ------------------------------------------------------------------ solver
    def init_solver(self, x, p):
        """ocp.py:265-313 (OSQP branch): constant Hessian diagonal + A pattern."""
        self.hess_diag = self.compute_hess_diag(p)
        self.pattern = self.structural_pattern(p)
        blocks = [(self.x_off[i], (self.x_off[i + 1] if i < self.N else self.n) - self.x_off[i], self.ndx)
                  for i in range(self.N + 1)]
        self.osqp = OSQPRef(self.hess_diag, self.pattern, self.osqp_settings, kkt=self.kkt, blocks=blocks)

    def jacobian_values(self, x, p):
        J = self.eval_J(x, p)
        Jp = self.pattern.copy().tocsc()
        Jp.data[:] = 0.0
        Jd = (Jp + J).tocsc()
        Jd.sort_indices()
        # values on the fixed pattern, CSC order
        pat = self.pattern.tocsc()
        pat.sort_indices()
        vals = np.zeros(pat.nnz)
        for col in range(pat.shape[1]):
            a, b = pat.indptr[col], pat.indptr[col + 1]
            ra = pat.indices[a:b]
            ca, cb = Jd.indptr[col], Jd.indptr[col + 1]
            m = dict(zip(Jd.indices[ca:cb], Jd.data[ca:cb]))
            extra = set(m) - set(ra.tolist())
            # entries that vanish in exact arithmetic may carry round-off (|v| ~ 1e-17)
            assert not any(abs(m[r]) > 1e-10 for r in extra), "Jacobian entry outside the structural pattern"
            vals[a:b] = [m.get(r, 0.0) for r in ra]
        return vals

    @staticmethod
    def violation_metric(g, lbg, ubg):
        lb = np.maximum(0, lbg - g)
        ub = np.maximum(0, g - ubg)
        return float(np.linalg.norm(np.concatenate([lb, ub])))

    @staticmethod
    def violation_max(g, lbg, ubg):
        lb = np.maximum(0, lbg - g)
        ub = np.maximum(0, g - ubg)
        return float(np.max(np.abs(np.concatenate([lb, ub]))))

    def line_search(self, dx, x, p):
        """_armijo_line_search (ocp.py:430-480). Returns (x_new, accepted, alpha, branch, trials)."""
        armijo_factor, a, a_min, a_decay = 1e-4, 1.0, 1e-4, 0.5
        g_max, g_min, gamma = 1e-3, 1e-5, 1e-5
        f, grad = self.f_and_grad(x, p)
        g, lbg, ubg = self.eval_g(x, p)
        g_metric = self.violation_metric(g, lbg, ubg)
        armijo_metric = float(grad @ dx)
        accepted = False
        branch = 0
        trials = 0
        new_x = x
        while not accepted and a > a_min:
            new_x = x + a * dx
            new_f, _ = self.f_and_grad(new_x, p)
            new_g, lbg, ubg = self.eval_g(new_x, p)
            new_gm = self.violation_metric(new_g, lbg, ubg)
            trials += 1
            if new_gm > g_max:
                if new_gm < (1 - gamma) * g_metric:
                    accepted, branch = True, 1
            elif max(new_gm, g_metric) < g_min and armijo_metric < 0:
                if new_f <= f + armijo_factor * armijo_metric:
                    accepted, branch = True, 2
            elif new_f <= f - gamma * new_gm or new_gm < (1 - gamma) * g_metric:
                accepted, branch = True, 3
            a *= a_decay
            f = new_f
            g_metric = new_gm
        if accepted:
            return new_x, True, a / a_decay, branch, trials
        return x, False, 0.0, 0, trials

    def sqp_step(self, x, p):
        """ocp.solve() OSQP branch (ocp.py:375-422) minus retract. Returns x_new and stats."""
        f, grad = self.f_and_grad(x, p)
        g, lbg, ubg = self.eval_g(x, p)
        Ax = self.jacobian_values(x, p)
        dx, info = self.osqp.update_and_solve(grad, Ax, lbg - g, ubg - g)
        stats = dict(status=info["status"], iter=info["iter"], pri_res=info["pri_res"], dua_res=info["dua_res"])
        if np.any(np.isnan(dx)):
            # NaN step: every trial compares False -> "didn't converge" (ocp.py:478-480)
            x_new, acc, alpha, branch, trials = x, False, 0.0, 0, 14
        else:
            x_new, acc, alpha, branch, trials = self.line_search(dx, x, p)
        g2, l2, u2 = self.eval_g(x_new, p)
        stats.update(accepted=acc, alpha=alpha, branch=branch, trials=trials,
                     viol_max=self.violation_max(g2, l2, u2))
        return x_new, dx, stats

    # ------------------------------------------------------------------ MPC glue
    def initial_guess(self, P_setup):
        """Opti initial values after setup_constraints (ocp.py:159-163,193)."""
        x = np.zeros(self.n)
        ud = self.u_des(P_setup)
        for i in range(self.N):
            o = self.x_off[i] + self.ndx
            x[o:o + self.nu[i]] = ud[:self.nu[i]]
        return x

    def warm_start(self, x_prev_solution, p):
        """warm_start (ocp_whole_body_rnea.py:207-235 and siblings): DX <- DX_prev,
        inputs <- [previous a / tau / v, f_des masked by the contact schedule, tau]."""
        P = self.unpack(p)
        DX, U = self.split(x_prev_solution)
        x = np.array(x_prev_solution, copy=True)
        fd = self.f_des(P)
        for i in range(self.N):
            f = fd.copy()
            for j in range(4):
                if P["contact"][j, i] == 0:
                    f[3 * j:3 * j + 3] = 0
            o = self.x_off[i] + self.ndx
            if self.dynamics == "whole_body_rnea":
                a_prev = U[i][:self.na]
                uw = np.concatenate([a_prev, f] + ([U[i][self.na + self.nf:]] if i < self.tau_nodes else []))
            elif self.dynamics == "whole_body_aba":
                uw = np.concatenate([U[i][:self.nj], f])
            elif self.dynamics in ("whole_body_acc", "centroidal_acc"):
                uw = np.concatenate([U[i][:self.na], f])
            else:
                uw = np.concatenate([U[i][:self.nv_opt], f])
            x[o:o + self.nu[i]] = uw
        return x

    def integrate_state(self, x_state, dx):
        """dyn.state_integrate()(x, dx)."""
        if self.dynamics == "centroidal_vel":
            return np.concatenate([x_state[:6] + dx[:6], rbd.integrate(self.M, x_state[6:], dx[6:])])
        return np.concatenate([rbd.integrate(self.M, x_state[:self.nq], dx[:self.nv]),
                               x_state[self.nq:] + dx[self.nv:]])
