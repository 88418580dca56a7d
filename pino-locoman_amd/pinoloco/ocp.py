"""make_ocp / OCP surface of the reference, backed by the HIP solve path.

Mirrors ``optimization/ocp_factory.py:8-27`` and the methods of
``optimization/ocp.py`` / ``ocp_whole_body_{rnea,acc,aba}.py`` that the drivers
use (``run_mpc.py:72-143``, ``run_ocp.py:48-99``): parameter setters, gait update,
warm start, ``init_solver``, ``solve(retract_all)``, ``retract_stacked_sol``,
``DX_prev`` / ``U_prev`` / ``q_sol`` ... / ``solve_time``.  Solver ``"osqp"`` runs
the OSQP-SQP path on the GPU through libpinoloco (one problem = batch of 1);
:class:`BatchedOCP` exposes the same path for a batch of independent problems.
"""
from __future__ import annotations

import ctypes as C
import time

import numpy as np

from . import _lib
from .dynamics import DYNAMICS_CLASSES, Dynamics  # noqa: F401  (Dynamics: plugin base class)
from .gait import horizon_dts

DYN_CODES = {"whole_body_rnea": 0, "whole_body_acc": 1, "whole_body_aba": 2, "centroidal_vel": 3,
             "centroidal_acc": 4}
GAIT_CODES = {"trot": 0, "walk": 1, "stand": 2}
SOLVER_CODES = {"osqp": 0, "fatrop": 1}

# ocp.py:267-273 plus the OSQP 0.6 library defaults it leaves untouched.
OSQP_SETTINGS = dict(max_iter=100, alpha=1.4, rho=2e-2, warm_start=True, adaptive_rho=False,
                     sigma=1e-6, eps_abs=1e-3, eps_rel=1e-3, eps_prim_inf=1e-4, eps_dual_inf=1e-4,
                     scaling=10, check_termination=25)

# ocp.py:254-262 (the reference's Fatrop options) plus the restatement's constants
# (oracle/ip_ref.py IP_SETTINGS: bound_frac, regularisation, line-search trials)
# hessian: 0 = the exact Lagrangian Hessian (CasADi / Fatrop), 1 = the objective's diagonal
FATROP_SETTINGS = dict(max_iter=10, tol=1e-3, mu_init=1e-4, bound_push=1e-7, bound_frac=1e-2, delta_w=1e-8,
                       delta_c=1e-4, ls_max=12, n_refine=8, hessian=0)
IP_HESSIAN = {"exact": 0, "gauss_newton": 1}

# ocp_args.py:2-19
OCP_ARGS = {
    "centroidal_vel": {"include_base": True},
    "centroidal_acc": {"include_base": True},
    "whole_body_acc": {"include_base": True},
    "whole_body_aba": {},
    "whole_body_rnea": {"tau_nodes": 3, "include_acc": True},
}

STATUS_NAMES = {1: "solved", 2: "solved inaccurate", -2: "maximum iterations reached", -3: "primal infeasible",
                3: "primal infeasible inaccurate", -4: "dual infeasible", 4: "dual infeasible inaccurate",
                -7: "problem non convex", -10: "unsolved"}


class Layout:
    """Variable / parameter bookkeeping (setup_variables / setup_parameters)."""

    def __init__(self, robot, dynamics, nodes, tau_nodes=3, include_base=True, include_acc=True):
        self.dynamics = dynamics
        self.include_base = include_base
        self.include_acc = include_acc
        self.N = nodes
        self.nq, self.nv, self.nj, self.nf = robot.nq, robot.nv, robot.nj, robot.nf
        self.nx = self.nq + self.nv
        self.ndx = 2 * self.nv
        nv, nj, nf = self.nv, self.nj, self.nf
        if dynamics == "centroidal_vel":
            # x = [h (6), q], dx = [dh, dq], u = [v | f] or, without the base, [v_j | f]
            # (ocp_centroidal_vel.py:19-23, 49-66)
            self.nx, self.ndx = 6 + self.nq, 6 + nv
            self.tau_nodes = 0
            self.na = 0
            self.nv_opt = nv if include_base else nj
            self.nu = [self.nv_opt + nf] * nodes
            self.f_idx, self.tau_idx = self.nv_opt, None
        elif dynamics == "whole_body_rnea":
            # na_opt = nv, or 0 with finite-difference accelerations (ocp_whole_body_rnea.py:21-26, 69-76)
            self.tau_nodes = tau_nodes
            self.na = nv if include_acc else 0
            self.nu = [self.na + nf + nj] * tau_nodes + [self.na + nf] * (nodes - tau_nodes)
            self.f_idx, self.tau_idx = self.na, self.na + nf
        elif dynamics in ("whole_body_acc", "centroidal_acc"):
            # u = [a | f] or, without the base, [a_j | f] (ocp_whole_body_acc.py:56-63,
            # ocp_centroidal_acc.py:15-19, 57-59)
            self.tau_nodes = 0
            self.na = nv if include_base else nj
            self.nu = [self.na + nf] * nodes
            self.f_idx, self.tau_idx = self.na, self.na + nf
        elif dynamics == "whole_body_aba":
            self.tau_nodes = 0
            self.na = 0
            self.nu = [nj + nf] * nodes
            self.f_idx, self.tau_idx = nj, None
        else:
            raise ValueError(f"Unknown dynamics type: {dynamics}")
        self.x_off = [0]
        for i in range(nodes):
            self.x_off.append(self.x_off[-1] + self.ndx + self.nu[i])
        self.n = self.x_off[-1] + self.ndx
        items = [("x_init", self.nx), ("dt_min", 1), ("dt_max", 1), ("contact_schedule", 4 * nodes),
                 ("swing_schedule", 4 * nodes), ("n_contacts", 1), ("swing_period", 1), ("swing_height", 1),
                 ("swing_vel_limits", 2), ("Q_diag", self.ndx), ("R_diag", self.nu[0]), ("base_vel_des", 6),
                 ("ext_force_des", 3), ("arm_vel_des", 3)]
        if dynamics == "whole_body_rnea":
            items += [("tau_prev", nj), ("W_diag", nj)]
        self.poff = {}
        off = 0
        for k, s in items:
            self.poff[k] = (off, s)
            off += s
        self.np = off

    def pack(self, values: dict) -> np.ndarray:
        p = np.zeros(self.np)
        for k, (o, s) in self.poff.items():
            v = values.get(k)
            if v is None:
                continue
            v = np.asarray(v, dtype=np.float64)
            if k in ("contact_schedule", "swing_schedule"):
                v = v.reshape(4, self.N).T  # column-major 4xN (CasADi parameter vectorisation)
            p[o:o + s] = v.ravel()
        return p

    def split(self, x):
        DX, U = [], []
        for i in range(self.N):
            o = self.x_off[i]
            DX.append(x[o:o + self.ndx])
            U.append(x[o + self.ndx:o + self.ndx + self.nu[i]])
        DX.append(x[self.x_off[self.N]:self.x_off[self.N] + self.ndx])
        return DX, U


def default_weights(robot, dynamics, layout):
    """set_weights (ocp_whole_body_rnea.py:28-63, ocp_whole_body_acc.py:26-54, ocp_whole_body_aba.py:22-50)."""
    nj, nf = robot.nj, robot.nf
    Qb = [0, 0, 1000, 10000, 10000, 0]
    Qj = list(np.tile([1000, 500, 500], 4))
    if robot.arm_ee_frame is not None:
        Qj += [100] * 6
    Qv = [2000, 2000, 1000, 1000, 1000, 2000] + [1] * nj
    Q = np.array(Qb + Qj + Qv, float)
    if dynamics == "centroidal_vel":  # ocp_centroidal_vel.py:23-47
        Q = np.array([1000] * 6 + Qb + Qj, float)
        R = np.array([1] * layout.nv_opt + [1e-3] * nf, float)
    elif dynamics == "whole_body_rnea":
        R = np.array([1e-3] * layout.na + [1e-3] * nf + [1e-4] * nj, float)
    elif dynamics in ("whole_body_acc", "centroidal_acc"):
        R = np.array([1e-3] * layout.na + [1e-3] * nf, float)
    else:
        R = np.array([1e-3] * nj + [1e-3] * nf, float)
    W = np.zeros(nj)
    return Q, R, W


class BatchedOCP:
    """A batch of independent OCPs of one (robot, dynamics, N) on one GPU."""

    def __init__(self, robot, dynamics, nodes, batch=1, device=0, tau_nodes=3, include_acc=True,
                 include_base=True, gait_type="trot", gait_period=0.8, osqp_settings=None, mu=0.7, debug_paths=()):
        """debug_paths: names of _lib.PATHS (the reference paths of the regression tests and the
        phase timing); empty in production."""
        if dynamics not in DYN_CODES:
            raise ValueError(f"Unknown dynamics type: {dynamics}")
        L = _lib.lib()
        self.robot = robot
        self.dynamics = dynamics
        self.batch = batch
        self.layout = Layout(robot, dynamics, nodes, tau_nodes, include_base, include_acc)
        self.model_h = ModelCache.get(robot.model)
        s = dict(OSQP_SETTINGS)
        if osqp_settings:
            s.update(osqp_settings)
        self.settings = s
        model = robot.model
        feet = robot.foot_frames if robot.foot_frames is not None else [model.get_frame_id(f) for f in
                                                                         ("FR_foot", "FL_foot", "RR_foot", "RL_foot")]
        base = model.get_frame_id("base_link")
        self._keep = []

        def arr(x):
            a = np.ascontiguousarray(np.asarray(x, dtype=np.float64))
            self._keep.append(a)
            return _lib.dptr(a)

        d = _lib.OcpDesc()
        d.dynamics = DYN_CODES[dynamics]
        d.nodes = nodes
        d.tau_nodes = tau_nodes if dynamics == "whole_body_rnea" else 0
        d.include_acc = int(include_acc)
        d.include_base = int(include_base)
        d.n_feet = 4
        for k in range(4):
            d.foot_frames[k] = int(feet[k])
        d.ext_force_frame = -1 if robot.ext_force_frame is None else int(robot.ext_force_frame)
        d.arm_ee_frame = -1 if robot.arm_ee_frame is None else int(robot.arm_ee_frame)
        d.base_frame = base if base < len(model.frames) else -1
        d.mu = mu
        d.q0 = arr(robot.q0)
        d.joint_pos_min = arr(robot.joint_pos_min)
        d.joint_pos_max = arr(robot.joint_pos_max)
        d.joint_vel_max = arr(robot.joint_vel_max)
        d.joint_torque_max = arr(robot.joint_torque_max)
        for k in ("rho", "sigma", "alpha", "eps_abs", "eps_rel", "eps_prim_inf", "eps_dual_inf"):
            setattr(d, k, float(s[k]))
        d.max_iter, d.scaling, d.check_termination = int(s["max_iter"]), int(s["scaling"]), int(
            s["check_termination"])
        d.warm_start = int(bool(s["warm_start"]))
        d.gait_type = GAIT_CODES[gait_type]
        d.gait_period = float(gait_period)
        bits = 0
        for name in debug_paths:
            if name not in _lib.PATHS:
                raise ValueError(f"unknown debug path {name} (choose from {sorted(_lib.PATHS)})")
            bits |= _lib.PATHS[name]
        d.debug_paths = bits
        h = C.c_void_p()
        _lib.check(L.pl_ocp_create(self.model_h.h, C.byref(d), batch, device, C.byref(h)))
        self.h = h
        self.device = device
        n, m, np_, nnz = C.c_int(), C.c_int(), C.c_int(), C.c_int()
        _lib.check(L.pl_ocp_dims(h, C.byref(n), C.byref(m), C.byref(np_), C.byref(nnz)))
        self.n, self.m, self.np, self.nnz = n.value, m.value, np_.value, nnz.value
        assert self.n == self.layout.n and self.np == self.layout.np, (self.n, self.layout.n, self.np, self.layout.np)

    # ---------------------------------------------------------------- queries
    def pattern(self):
        rows = np.zeros(self.nnz, dtype=np.int32)
        cols = np.zeros(self.nnz, dtype=np.int32)
        _lib.check(_lib.lib().pl_ocp_pattern(self.h, _lib.iptr(rows), _lib.iptr(cols)))
        return rows, cols

    def node_table(self):
        out = np.zeros(12 * (self.layout.N + 1), dtype=np.int32)
        _lib.check(_lib.lib().pl_debug_nodes(self.h, _lib.iptr(out)))
        return out.reshape(-1, 12)

    # ---------------------------------------------------------------- data
    def set_params(self, P):
        P = np.ascontiguousarray(np.broadcast_to(np.asarray(P, dtype=np.float64), (self.batch, self.np)))
        _lib.check(_lib.lib().pl_ocp_set_params(self.h, _lib.dptr(P)))

    def get_params(self):
        P = np.zeros((self.batch, self.np))
        _lib.check(_lib.lib().pl_ocp_get_params(self.h, _lib.dptr(P)))
        return P

    def set_x(self, X):
        X = np.ascontiguousarray(np.broadcast_to(np.asarray(X, dtype=np.float64), (self.batch, self.n)))
        _lib.check(_lib.lib().pl_ocp_set_x(self.h, _lib.dptr(X)))

    def get_x(self):
        X = np.zeros((self.batch, self.n))
        _lib.check(_lib.lib().pl_ocp_get_x(self.h, _lib.dptr(X)))
        return X

    def get_step(self):
        X = np.zeros((self.batch, self.n))
        _lib.check(_lib.lib().pl_ocp_get_step(self.h, _lib.dptr(X)))
        return X

    def init_solver(self):
        _lib.check(_lib.lib().pl_ocp_init_solver(self.h))

    def set_sqp_iters(self, k):
        """SQP iterations per solve / MPC step (reference: 1, ocp.py:382-383)."""
        _lib.check(_lib.lib().pl_ocp_set_sqp_iters(self.h, int(k)))

    ADMM_KERNELS = {"auto": 0, "sweep": 1, "sweep2": 2, "chain": 3}

    def set_admm_kernel(self, kind):
        """GPU mapping of the ADMM linear solve inside osqp.solve() (ocp.py:401): "sweep"
        (one wave per problem, node-by-node block sweeps), "sweep2" (two waves per problem),
        "chain" (reduced chain, one workgroup per problem) or "auto" (by batch size).  All
        run the same OSQP iteration on the same factor and agree to round-off."""
        if kind not in self.ADMM_KERNELS:
            raise ValueError(f"ADMM kernel {kind} unknown (choose from {sorted(self.ADMM_KERNELS)})")
        _lib.check(_lib.lib().pl_ocp_set_admm_kernel(self.h, self.ADMM_KERNELS[kind]))

    def admm_kernel(self):
        code = _lib.lib().pl_ocp_get_admm_kernel(self.h)
        return {v: k for k, v in self.ADMM_KERNELS.items()}[code]

    def admm_groups(self):
        """Workgroups per problem of the next ADMM launch (k_admm_rc spreads its node phases
        over several; the sweep kernels use 1)."""
        return _lib.lib().pl_ocp_get_admm_groups(self.h)

    def set_solver(self, solver):
        """"osqp" (SQP + OSQP, ocp.py:265-313 / 375-422) or "fatrop" (the interior-point
        restatement of the Fatrop branch, ocp.py:248-263 / 360-373)."""
        if solver not in SOLVER_CODES:
            raise ValueError(f"Solver {solver} not supported (choose from {sorted(SOLVER_CODES)})")
        _lib.check(_lib.lib().pl_ocp_set_solver(self.h, SOLVER_CODES[solver]))
        self.solver = solver

    def set_ip_settings(self, **kw):
        """Interior-point settings (defaults: FATROP_SETTINGS, the reference's ocp.py:254-262)."""
        s = dict(FATROP_SETTINGS)
        s.update(kw)
        if isinstance(s["hessian"], str):
            s["hessian"] = IP_HESSIAN[s["hessian"]]
        st = _lib.IpSettings(**{k: s[k] for k, _ in _lib.IpSettings._fields_})
        _lib.check(_lib.lib().pl_ocp_set_ip_settings(self.h, C.byref(st)))

    def ip_stats(self):
        stats = (_lib.IpStats * self.batch)()
        _lib.check(_lib.lib().pl_ocp_ip_stats(self.h, stats))
        return {k: np.array([np.array(getattr(s, k)) for s in stats]) for k, _ in _lib.IpStats._fields_}

    def set_lam(self, lam):
        """lam_g warm start of the next interior-point solves ([batch][m] or None for the
        cold start), the OCPs' opti.set_initial(opti.lam_g, lam_g) (ocp_whole_body_rnea.py:234-235)."""
        if lam is None:
            _lib.check(_lib.lib().pl_ocp_set_lam(self.h, None))
            return
        lam = np.ascontiguousarray(np.broadcast_to(np.asarray(lam, dtype=np.float64), (self.batch, self.m)))
        _lib.check(_lib.lib().pl_ocp_set_lam(self.h, _lib.dptr(lam)))

    def get_lam(self):
        lam = np.zeros((self.batch, self.m))
        _lib.check(_lib.lib().pl_ocp_get_lam(self.h, _lib.dptr(lam)))
        return lam

    def ip_direction(self, X, S, LAM, ZL, ZU, MU):
        """Teacher-forced interior-point Newton direction (parity aid): (dx, dlam, ds,
        alpha_max, alpha_z) from the given iterate, slacks and multipliers."""
        self.set_x(X)
        arrs = [np.ascontiguousarray(np.broadcast_to(np.asarray(a, dtype=np.float64), (self.batch, self.m)))
                for a in (S, LAM, ZL, ZU)]
        mu = np.ascontiguousarray(np.broadcast_to(np.asarray(MU, dtype=np.float64), (self.batch,)))
        _lib.check(_lib.lib().pl_debug_ip_direction(self.h, *[_lib.dptr(a) for a in arrs], _lib.dptr(mu)))
        B = self.batch
        st = self.ip_stats()
        return (self.debug("ip_dx", B * self.n).reshape(B, self.n), self.debug("ip_dl", B * self.m).reshape(B, self.m),
                self.debug("ip_ds", B * self.m).reshape(B, self.m), st["alpha"], st["alpha_z"])

    def solve(self, timed=False):
        stats = (_lib.Stats * self.batch)()
        phase = np.zeros(4)
        _lib.check(_lib.lib().pl_ocp_solve(self.h, stats, _lib.dptr(phase) if timed else None))
        out = {k: np.array([getattr(s, k) for s in stats]) for k, _ in _lib.Stats._fields_ if k != "pad"}
        if timed:
            out["phase_ms"] = phase
        return out

    def eval_sqp_data(self):
        B = self.batch
        grad, J = np.zeros((B, self.n)), np.zeros((B, self.nnz))
        g, lbg, ubg = np.zeros((B, self.m)), np.zeros((B, self.m)), np.zeros((B, self.m))
        _lib.check(_lib.lib().pl_eval_sqp_data(self.h, _lib.dptr(grad), _lib.dptr(J), _lib.dptr(g), _lib.dptr(lbg),
                                               _lib.dptr(ubg)))
        return grad, J, g, lbg, ubg

    def eval_f(self):
        f = np.zeros(self.batch)
        _lib.check(_lib.lib().pl_eval_f(self.h, _lib.dptr(f)))
        return f

    def debug(self, name, length):
        out = np.zeros(length)
        _lib.check(_lib.lib().pl_debug_get(self.h, name.encode(), _lib.dptr(out), length))
        return out

    def debug_set(self, name, values):
        v = np.ascontiguousarray(np.asarray(values, dtype=np.float64).ravel())
        _lib.check(_lib.lib().pl_debug_set(self.h, name.encode(), _lib.dptr(v), v.size))

    def lag_hess(self):
        """The interior point's Lagrangian Hessian blocks of the last Newton system (tests):
        [batch] list of csr n x n matrices (k_lag_hess, packed lower per node)."""
        import scipy.sparse as sp
        nodes = self.node_table()
        B = self.batch
        offs, o = [], 0
        for nd in nodes:
            offs.append(o)
            o += nd[0] * (nd[0] + 1) // 2
        stride = (o + 1) & ~1
        raw = self.debug("Hlag", B * stride).reshape(B, stride)
        out = []
        for b in range(B):
            rows, cols, vals = [], [], []
            for i, nd in enumerate(nodes):
                nw, xo = nd[0], nd[2]
                kk, jj = np.tril_indices(nw)
                v = raw[b, offs[i] + kk * (kk + 1) // 2 + jj]
                rows += (xo + kk).tolist() + (xo + jj[kk != jj]).tolist()
                cols += (xo + jj).tolist() + (xo + kk[kk != jj]).tolist()
                vals += v.tolist() + v[kk != jj].tolist()
            out.append(sp.csr_matrix((vals, (rows, cols)), shape=(self.n, self.n)))
        return out

    # ---------------------------------------------------------------- MPC
    def mpc_setup(self, x_state, t0):
        xs = np.ascontiguousarray(np.asarray(x_state, dtype=np.float64).reshape(self.batch, -1))
        t = np.ascontiguousarray(np.asarray(t0, dtype=np.float64).reshape(self.batch))
        _lib.check(_lib.lib().pl_mpc_setup(self.h, _lib.dptr(xs), _lib.dptr(t)))

    def mpc_step(self, k):
        _lib.check(_lib.lib().pl_mpc_step(self.h, int(k)))

    def mpc_state(self):
        xs = np.zeros((self.batch, self.layout.nx))
        _lib.check(_lib.lib().pl_mpc_get_state(self.h, _lib.dptr(xs)))
        return xs

    def mpc_stats(self):
        stats = (_lib.Stats * self.batch)()
        _lib.check(_lib.lib().pl_mpc_get_stats(self.h, stats))
        return {k: np.array([getattr(s, k) for s in stats]) for k, _ in _lib.Stats._fields_ if k != "pad"}

    def mpc_export(self, device_ptr):
        _lib.check(_lib.lib().pl_mpc_export(self.h, C.c_void_p(device_ptr)))

    def mpc_download(self, out=None):
        """[u_0, x_state] per problem into host memory ([batch][nu_0 + nx]); returns after the copy."""
        if out is None:
            out = np.zeros((self.batch, self.layout.nu[0] + self.layout.nx))
        _lib.check(_lib.lib().pl_mpc_download(self.h, _lib.dptr(out)))
        return out

    def mpc_set_ip_lam(self, carry):
        """Interior-point MPC loop: carry=False (default) the reference's default driver
        (compile_solver=True: primal warm start, cold multipliers, run_mpc.py:34-37, 50-111);
        carry=True the Opti branch (lam_g passed back, ocp_whole_body_rnea.py:234-235)."""
        _lib.check(_lib.lib().pl_mpc_set_ip_lam(self.h, int(bool(carry))))

    def mpc_graph_info(self):
        out = (C.c_longlong * 3)()
        _lib.check(_lib.lib().pl_mpc_graph_info(self.h, out))
        return {"captures": int(out[0]), "replays": int(out[1]), "eager_fallback": int(out[2])}

    def sync(self):
        _lib.check(_lib.lib().pl_ocp_sync(self.h))

    def profile(self, enable):
        _lib.check(_lib.lib().pl_ocp_profile(self.h, int(enable)))

    def profile_read(self):
        out = np.zeros(3)
        _lib.check(_lib.lib().pl_ocp_profile_read(self.h, _lib.dptr(out)))
        return {"admm_ms": out[0], "launches": int(out[1]), "problem_iters": int(out[2])}

    def profile_read_hess(self):
        out = np.zeros(3)
        _lib.check(_lib.lib().pl_ocp_profile_read_hess(self.h, _lib.dptr(out)))
        return {"hess_ms": out[0], "launches": int(out[1]), "lanes": out[2]}

    def sizes(self):
        out = (C.c_longlong * 13)()
        _lib.check(_lib.lib().pl_ocp_sizes(self.h, out))
        return dict(zip(("n", "m", "nnz", "S_stride", "nw_max", "N", "admm_prog", "admm_ppw", "admm_lds_bytes",
                         "admm_asr", "admm_asb_cap", "nent_max", "debug_paths"), [int(v) for v in out]))

    def close(self):
        if getattr(self, "h", None):
            _lib.lib().pl_ocp_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


class ModelCache:
    _cache = {}

    @classmethod
    def get(cls, model):
        key = id(model)
        if key not in cls._cache:
            cls._cache[key] = (model, _lib.ModelHandle(model))
        return cls._cache[key][1]


class ParamSym:
    """An Opti parameter (or decision) symbol of the reference (``opti.parameter`` /
    ``opti.x``, ocp.py:54-69): a name that :meth:`Opti.value` reads back and that
    :class:`CompiledSolver` accepts as an argument slot."""

    def __init__(self, name):
        self.name = name

    def __repr__(self):
        return f"ParamSym({self.name!r})"


# Parameters the drivers read through ocp.opti.value (run_mpc.py:64-77) or pass to the
# compiled solver (ocp.py:326-335, ocp_whole_body_rnea.py:239-250)
OPTI_PARAMS = ("x_init", "dt_min", "dt_max", "contact_schedule", "swing_schedule", "n_contacts", "swing_period",
               "swing_height", "swing_vel_limits", "Q_diag", "R_diag", "base_vel_des", "ext_force_des", "arm_vel_des",
               "tau_prev", "W_diag")


class Opti:
    """The part of the reference's ``ca.Opti`` its drivers read (run_mpc.py:56-77, 176):
    ``value(parameter)``, ``value(opti.x, opti.initial())`` (the warm-start point),
    ``value(opti.x)`` / ``value(opti.lam_g)`` after a solve, and plain numbers (the
    geometric ``dts``) returned unchanged."""

    x = ParamSym("x")
    lam_g = ParamSym("lam_g")

    def __init__(self, ocp):
        self._ocp = ocp

    @staticmethod
    def initial():
        return "initial"

    def value(self, sym, initial=None):
        o = self._ocp
        if not isinstance(sym, ParamSym):
            return np.asarray(sym, float) if np.ndim(sym) else float(sym)
        if sym.name == "x":
            if initial is not None:
                return o._x_initial.copy()
            if o._x_sol is None:
                raise RuntimeError("opti.value(opti.x): no solution yet (solve first)")
            return o._x_sol.copy()
        if sym.name == "lam_g":
            if o.lam_g is None:
                raise RuntimeError("opti.value(opti.lam_g): no solution yet (solve first)")
            return o.lam_g.copy()
        if sym.name not in o.p:
            raise RuntimeError(f"opti.value({sym.name}): parameter not set")
        v = o.p[sym.name]
        return np.array(v, float) if np.ndim(v) else float(v)


class CompiledSolver:
    """The Fatrop branch's compiled solver (``opti.to_function("compiled_solver", params,
    [opti.x])``, ocp.py:324-342 and ocp_whole_body_rnea.py:237-258; called as
    ``sol_x = solver_function(*params)`` at run_mpc.py:100 with the parameter list of
    run_mpc.py:84-96).  One call is one interior-point solve of this OCP on the GPU from
    the given parameters and primal warm start (``x_warm_start`` when compiled with
    ``warm_start``, else the initial guess at compile time).  The function has no lam_g
    input, so the multipliers start cold, as the reference's generated function does
    (its lam_g initial is the one baked in at ``to_function`` time, before any solve).
    A solve that stops at the iteration cap or on a failed line search returns its last
    iterate (the reference's function returns the solver's output; ``opti.debug``,
    ocp.py:362-365, in the uncompiled branch).  Returns x as a flat float64 vector."""

    def __init__(self, ocp, names):
        self._ocp = ocp
        self.names = list(names)
        self._x0 = None if "x" in self.names else ocp._x_initial.copy()

    def n_in(self):
        return len(self.names)

    def name_in(self, i):
        return self.names[i]

    def _pack(self, args):
        """(p, x0) of one call: the OCP's current parameters overridden by the arguments."""
        if len(args) != len(self.names):
            raise TypeError(f"compiled_solver takes {len(self.names)} arguments ({', '.join(self.names)}), "
                            f"got {len(args)}")
        o = self._ocp
        vals = dict(o.p)
        x0 = self._x0
        for name, a in zip(self.names, args):
            if name == "x":
                x0 = np.asarray(a, float).ravel()
                if x0.size != o.layout.n:
                    raise ValueError(f"x_warm_start has {x0.size} entries, the OCP {o.layout.n}")
            else:
                vals[name] = a
        return o.layout.pack(vals), np.array(x0, float)

    def __call__(self, *args):
        o = self._ocp
        p, x0 = self._pack(args)
        be = o._backend
        be.set_params(p)
        be.init_solver()  # the objective's Hessian diagonal from these parameters (ocp.py:293-296)
        be.set_x(x0)
        be.set_lam(None)
        start = time.time()
        st = be.solve()
        o.solve_time = time.time() - start
        o.stats = {k: v[0] for k, v in st.items()}
        o.stats.update({"ip_" + k: v[0] for k, v in be.ip_stats().items()})
        x = be.get_x()[0]
        o._x_sol = x.copy()
        return x


class OCP:
    """Single-problem OCP with the reference's method surface (ocp.py:11-480)."""

    def __init__(self, robot, solver, nodes, dynamics, tau_nodes=3, include_acc=True, include_base=True, device=0):
        if solver not in SOLVER_CODES:
            raise ValueError(f"Solver {solver} not supported (ocp.py:248, 265: 'fatrop' or 'osqp')")
        self.robot = robot
        self.model = robot.model
        self.gait_sequence = robot.gait_sequence
        self.foot_frames = robot.foot_frames
        self.ext_force_frame = robot.ext_force_frame
        self.arm_ee_frame = robot.arm_ee_frame
        self.n_feet = len(self.foot_frames)
        self.nq, self.nv, self.nf, self.nj = robot.nq, robot.nv, robot.nf, robot.nj
        self.solver = solver
        self.nodes = nodes
        self.mass = robot.mass
        self.dynamics = dynamics
        self.dyn = DYNAMICS_CLASSES[dynamics](robot, device=device)
        self.layout = Layout(robot, dynamics, nodes, tau_nodes, include_base, include_acc)
        L = self.layout
        self.nx, self.ndx_opt, self.nu_opt = L.nx, L.ndx, L.nu
        self.f_idx, self.tau_idx = L.f_idx, L.tau_idx
        self.tau_nodes = L.tau_nodes
        self.na_opt = L.na
        self.include_acc, self.include_base = include_acc, include_base
        if dynamics == "centroidal_vel":
            self.x_nom = np.concatenate(([0] * 6, robot.q0))  # CoM momentum + joint pos (ocp_centroidal_vel.py:16)
        else:
            self.x_nom = np.concatenate((robot.q0, [0] * self.nv))
        self.q_sol, self.v_sol, self.a_sol, self.forces_sol, self.tau_sol = [], [], [], [], []
        self.DX_prev = None
        self.U_prev = None
        self.lam_g = None
        self.solve_time = None
        self.stats = None
        self.solver_function = None
        self._x_sol = None
        # the Opti view and its parameter symbols (ocp.opti.value(ocp.Q_diag), run_mpc.py:64-77)
        self.opti = Opti(self)
        for name in OPTI_PARAMS:
            setattr(self, name, ParamSym(name))
        self._backend = BatchedOCP(robot, dynamics, nodes, batch=1, device=device, tau_nodes=tau_nodes,
                                   include_acc=include_acc, include_base=include_base,
                                   gait_type=self.gait_sequence.gait_type if self.gait_sequence else "trot",
                                   gait_period=self.gait_sequence.gait_period if self.gait_sequence else 0.8)
        if solver == "fatrop" and device >= 0:  # a host-only handle (device < 0) never solves
            self._backend.set_solver("fatrop")
            self._backend.set_ip_settings()
        self.p = {"tau_prev": np.zeros(self.nj), "W_diag": np.zeros(self.nj), "ext_force_des": np.zeros(3),
                  "arm_vel_des": np.zeros(3), "x_init": self.x_nom.copy()}
        if self.gait_sequence is not None:
            self.p["n_contacts"] = self.gait_sequence.n_contacts
        # initial guess: DX = 0, U = u_des (ocp.py:159-163, 193)
        self._x_initial = np.zeros(L.n)
        for i in range(nodes):
            o = L.x_off[i] + L.ndx
            self._x_initial[o:o + L.nu[i]] = self._u_des()[:L.nu[i]]

    # ------------------------------------------------------------------ params
    def _f_des(self):
        fg = 9.81 * self.mass
        nc = float(np.asarray(self.p["n_contacts"]).ravel()[0])
        f = [0, 0, 0.8 * fg / nc] * 2 + [0, 0, 1.2 * fg / nc] * 2
        if self.ext_force_frame is not None:
            f += [0, 0, 0]
        return np.array(f, float)

    def _u_des(self):
        f = self._f_des()
        if self.dynamics == "whole_body_rnea":
            return np.concatenate([np.zeros(self.na_opt), f, np.zeros(self.nj)])
        if self.dynamics in ("whole_body_acc", "centroidal_acc"):
            return np.concatenate([np.zeros(self.na_opt), f])
        if self.dynamics == "centroidal_vel":
            return np.concatenate([np.zeros(self.layout.nv_opt), f])
        return np.concatenate([np.zeros(self.nj), f])

    def set_weights(self):
        Q, R, W = default_weights(self.robot, self.dynamics, self.layout)
        self.p["Q_diag"], self.p["R_diag"], self.p["W_diag"] = Q, R, W

    def set_time_params(self, dt_min, dt_max):
        self.p["dt_min"], self.p["dt_max"] = dt_min, dt_max

    def set_swing_params(self, swing_height, swing_vel_limits):
        self.p["swing_height"], self.p["swing_vel_limits"] = swing_height, np.asarray(swing_vel_limits, float)

    def set_tracking_targets(self, base_vel_des, ext_force_des=None, arm_vel_des=None):
        self.p["base_vel_des"] = np.asarray(base_vel_des, float)
        if self.ext_force_frame is not None:
            self.p["ext_force_des"] = np.asarray(ext_force_des, float)
        if self.arm_ee_frame is not None:
            self.p["arm_vel_des"] = np.asarray(arm_vel_des, float)

    def update_initial_state(self, x_init):
        self.p["x_init"] = np.asarray(x_init, float).ravel()

    def update_previous_torques(self, tau_prev):
        self.p["tau_prev"] = np.asarray(tau_prev, float)

    @property
    def dts(self):
        return horizon_dts(self.p["dt_min"], self.p["dt_max"], self.nodes)

    def update_gait_sequence(self, t_current):
        contact, swing = self.gait_sequence.get_gait_schedule(t_current, self.dts, self.nodes)
        self.p["contact_schedule"], self.p["swing_schedule"] = contact, swing
        self.p["n_contacts"] = self.gait_sequence.n_contacts
        self.p["swing_period"] = self.gait_sequence.swing_period

    def param_vector(self):
        return self.layout.pack(self.p)

    # ------------------------------------------------------------------ warm start
    def warm_start(self):
        """ocp_whole_body_rnea.py:207-235 (and the acc / aba variants)."""
        L = self.layout
        x = self._x_initial
        if self.DX_prev is not None:
            for i in range(self.nodes + 1):
                x[L.x_off[i]:L.x_off[i] + L.ndx] = self.DX_prev[i]
        if self.U_prev is not None:
            contact = self.p["contact_schedule"]
            for i in range(self.nodes):
                f_des = self._f_des()
                for j in range(self.n_feet):
                    if contact[j, i] == 0:
                        f_des[3 * j:3 * j + 3] = 0
                u_prev = self.U_prev[i]
                if self.dynamics == "whole_body_aba":
                    u = np.concatenate([u_prev[:self.nj], f_des])
                elif self.dynamics == "centroidal_vel":  # ocp_centroidal_vel.py:152-158
                    u = np.concatenate([u_prev[:self.layout.nv_opt], f_des])
                else:
                    u = np.concatenate([u_prev[:self.na_opt], f_des])
                    if self.dynamics == "whole_body_rnea" and i < self.tau_nodes:
                        u = np.concatenate([u, u_prev[self.tau_idx:]])
                o = L.x_off[i] + L.ndx
                x[o:o + L.nu[i]] = u
        if self.solver == "fatrop" and self.lam_g is not None:  # ocp_whole_body_rnea.py:234-235 (every OCP)
            self._backend.set_lam(self.lam_g)

    # ------------------------------------------------------------------ solver
    def init_solver(self):
        """ocp.py:265-313: constant Hessian diagonal from the current parameters."""
        self._backend.set_params(self.param_vector())
        self._backend.init_solver()

    def compile_solver(self, warm_start):
        """ocp.py:324-353 / ocp_whole_body_rnea.py:237-258.  Fatrop: ``self.solver_function``
        takes the reference's parameter list -- x_init, dt_min, dt_max, contact_schedule,
        swing_schedule, n_contacts, swing_period, swing_height, swing_vel_limits, Q_diag,
        R_diag, base_vel_des, [ext_force_des], [arm_vel_des], [x_warm_start],
        [tau_prev, W_diag (whole_body_rnea)] -- and returns the solution x (CompiledSolver).
        OSQP: the reference generates C for sqp_data / f_data / g_data; the library's
        evaluation is native already (and exported in CasADi's external ABI by
        casadi_ext), so there is nothing to generate."""
        if self.solver != "fatrop":
            return
        names = ["x_init", "dt_min", "dt_max", "contact_schedule", "swing_schedule", "n_contacts", "swing_period",
                 "swing_height", "swing_vel_limits", "Q_diag", "R_diag", "base_vel_des"]
        if self.ext_force_frame:
            names.append("ext_force_des")
        if self.arm_ee_frame:
            names.append("arm_vel_des")
        if warm_start:
            names.append("x")
        if self.dynamics == "whole_body_rnea":
            names += ["tau_prev", "W_diag"]
        self.solver_function = CompiledSolver(self, names)

    def solve(self, retract_all=True, sqp_iters=1):
        """ocp.py:375-422 (OSQP branch) on the GPU: `sqp_iters` SQP iterations (the
        reference runs one, `for _ in range(1)`, ocp.py:382-383).  With solver
        "fatrop", one interior-point solve (ocp.py:360-373) from the warm start; a
        solve that does not converge returns its last iterate, as the reference's
        ``opti.debug`` fallback does, and ``lam_g`` holds the multipliers."""
        self._backend.set_sqp_iters(sqp_iters)
        self._backend.set_params(self.param_vector())
        self._backend.set_x(self._x_initial)
        start = time.time()
        st = self._backend.solve()
        self.solve_time = time.time() - start
        self.stats = {k: v[0] for k, v in st.items()}
        if self.solver == "fatrop":  # ocp.py:360-373: stats, retract, lam_g
            self.stats.update({"ip_" + k: v[0] for k, v in self._backend.ip_stats().items()})
            self.lam_g = self._backend.get_lam()[0]
        x = self._backend.get_x()[0]
        self._x_sol = x.copy()
        self.retract_stacked_sol(x, retract_all)
        return x

    def retract_stacked_sol(self, sol_x, retract_all=True):
        """ocp_whole_body_rnea.py:293-324 (ocp_whole_body_acc.py:195-234,
        ocp_whole_body_aba.py:177-214: a from aba_dynamics at the node)."""
        L = self.layout
        x_init = self.p["x_init"]
        integ = self.dyn.state_integrate()
        DX, U = L.split(np.asarray(sol_x, float))
        self.DX_prev = [np.array(d) for d in DX]
        self.U_prev = [np.array(u) for u in U]
        for i in range(self.nodes):
            if i == 0 or retract_all:
                xs = integ(x_init, DX[i])
                self.q_sol.append(xs[:self.nq])
                self.v_sol.append(xs[self.nq:])
                u = U[i]
                if self.dynamics == "whole_body_aba":
                    tau_j, forces = u[:self.nj], u[self.f_idx:]
                    self.tau_sol.append(tau_j)
                    self.forces_sol.append(forces)
                    ext = self.ext_force_frame
                    self.a_sol.append(self.dyn.aba_dynamics(ext)(xs[:self.nq], xs[self.nq:], tau_j, forces))
                elif self.dynamics in ("whole_body_acc", "centroidal_acc") and not self.include_base:
                    # a = [base_acc_dynamics(q, v, a_j, f), a_j] (ocp_whole_body_acc.py:124-135)
                    a_j, forces = u[:self.na_opt], u[self.f_idx:]
                    a_b = self.dyn.base_acc_dynamics(self.ext_force_frame)(xs[:self.nq], xs[self.nq:], a_j, forces)
                    self.a_sol.append(np.concatenate([a_b, a_j]))
                    self.forces_sol.append(forces)
                else:
                    self.a_sol.append(u[:self.na_opt])
                    self.forces_sol.append(u[self.f_idx:self.tau_idx] if self.tau_idx else u[self.f_idx:])
                    if self.dynamics == "whole_body_rnea":
                        self.tau_sol.append(u[self.tau_idx:])
        if retract_all:
            xs = integ(x_init, DX[-1])
            self.q_sol.append(xs[:self.nq])
            self.v_sol.append(xs[self.nq:])

    def get_tau_sol(self, i):
        return self.U_prev[i][self.tau_idx:]


class OCPWholeBodyRNEA(OCP):
    def __init__(self, robot, solver, nodes, tau_nodes, include_acc=True):
        super().__init__(robot, solver, nodes, "whole_body_rnea", tau_nodes=tau_nodes, include_acc=include_acc)


class OCPWholeBodyAcc(OCP):
    def __init__(self, robot, solver, nodes, include_base=False):
        super().__init__(robot, solver, nodes, "whole_body_acc", include_base=include_base)


class OCPWholeBodyABA(OCP):
    def __init__(self, robot, solver, nodes):
        super().__init__(robot, solver, nodes, "whole_body_aba")


class OCPCentroidalVel(OCP):
    """ocp_centroidal_vel.py: x = [h, q], dx = [dh, dq], u = [v | forces] or, with
    include_base=False (the class default), u = [v_j | forces] and the base velocity
    v_b = A_b^-1 (m h - A_j v_j) inside the rows (ocp_centroidal_vel.py:119-129)."""

    def __init__(self, robot, solver, nodes, include_base=False):
        super().__init__(robot, solver, nodes, "centroidal_vel", include_base=include_base)
        self.nv_opt = self.layout.nv_opt

    def retract_stacked_sol(self, sol_x, retract_all=True):
        """ocp_centroidal_vel.py:195-260: q, h from the state; v from the inputs; a by a
        forward difference of the input velocities, its base part replaced by
        base_acc_dynamics (pinocchio dccrba).  The reference's slice of the node after
        the last input is empty there (an error); the last node reuses the previous
        node's difference."""
        L = self.layout
        x_init = self.p["x_init"]
        integ = self.dyn.state_integrate()
        DX, U = L.split(np.asarray(sol_x, float))
        self.DX_prev = [np.array(d) for d in DX]
        self.U_prev = [np.array(u) for u in U]
        dts = self.dts
        base_acc = self.dyn.base_acc_dynamics(self.ext_force_frame)
        base_vel = self.dyn.base_vel_dynamics()
        nvo = self.nv_opt
        for i in range(self.nodes):
            if not (i == 0 or retract_all):
                continue
            xs = integ(x_init, DX[i])
            h, q = xs[:6], xs[6:]
            u = U[i]
            forces = u[self.f_idx:]

            def vel(uu):  # v from the inputs; without the base, v_b at this node's h, q (:228-246)
                if self.include_base:
                    return np.asarray(uu[:nvo], float)
                return np.concatenate([np.asarray(base_vel(h, q, uu[:nvo]), float).ravel(), uu[:nvo]])
            v = vel(u)
            k = i if i + 1 < self.nodes else i - 1
            a = (vel(U[k + 1]) - vel(U[k])) / dts[k]
            a_b = base_acc(q, v, a[6:], forces)
            self.q_sol.append(q)
            self.v_sol.append(v)
            self.a_sol.append(np.concatenate([a_b, a[6:]]))
            self.forces_sol.append(forces)
        if retract_all:
            self.q_sol.append(integ(x_init, DX[-1])[6:])


class OCPCentroidalAcc(OCP):
    """ocp_centroidal_acc.py: the whole-body state and inputs of OCPWholeBodyAcc with the base
    equations in centroidal form: the gap A a + dA v - dh (include_base) or the base
    acceleration A_b^-1 (dh - dA v - A_j a_j) (pinocchio computeCentroidalMap / dccrba)."""

    def __init__(self, robot, solver, nodes, include_base=False):
        super().__init__(robot, solver, nodes, "centroidal_acc", include_base=include_base)


def make_ocp(dynamics, default_args, **kwargs):
    """ocp_factory.py:8-27."""
    ocp_classes = {
        "centroidal_vel": OCPCentroidalVel,
        "centroidal_acc": OCPCentroidalAcc,
        "whole_body_acc": OCPWholeBodyAcc,
        "whole_body_aba": OCPWholeBodyABA,
        "whole_body_rnea": OCPWholeBodyRNEA,
    }
    if dynamics not in ocp_classes:
        raise ValueError(f"Unknown dynamics type: {dynamics}")
    args = default_args.copy()
    args.update(kwargs)
    ocp = ocp_classes[dynamics](**args)
    ocp.set_weights()
    return ocp
