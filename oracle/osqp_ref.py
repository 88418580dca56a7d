"""ORACLE (test infrastructure only) -- OSQP 0.6 ADMM restated in numpy/scipy.

The reference drives the third-party OSQP solver (``ocp.py:265-313, 391-401``;
``README.md:18`` pins no version).  OSQP is not vendored in ``/root/reference`` and
is not installed, so this file restates the published OSQP 0.6.x algorithm
(``src/osqp.c``, ``src/scaling.c``, ``src/auxil.c``, ``src/lin_sys`` with QDLDL) as
the reference calls it:

* settings from ``ocp.py:267-273``: max_iter=100, alpha=1.4, rho=0.02,
  warm_start=True, adaptive_rho=False; library defaults sigma=1e-6,
  eps_abs=eps_rel=1e-3, eps_prim_inf=eps_dual_inf=1e-4, scaling=10,
  check_termination=25, scaled_termination=False, polish=False;
* ``update(q, Ax, l, u)`` re-runs Ruiz equilibration on the new data and
  refactors (``osqp_update_A``); l/u are clipped to +-OSQP_INFTY (1e30);
* rho_vec: rows with u-l < 1e-4 get 1e3*rho, rows with both bounds infinite
  get RHO_MIN=1e-6, others rho;
* warm start keeps the SCALED iterates x, z, y across updates (zeros before the
  first solve);
* termination every 25 iterations on unscaled inf-norm residuals, primal/dual
  infeasibility certificates, and the "approximate" (x10 tolerance) check at
  max_iter; an infeasible status returns NaN and cold-starts the iterates.

PARITY UNPINNED (no OSQP binary or test vectors exist in the reference).  The
KKT system is solved exactly as OSQP's direct path does (full quasi-definite
KKT, z~ = z_prev + rho^-1 (nu - y)); the factorisation is SuperLU here instead of
QDLDL+AMD, which changes only round-off.

``kkt="reduced_block"`` (a diagnostic mode, not OSQP's algebra) solves the same ADMM step
the way the GPU does (csrc/k_factor.hip, csrc/k_admm.hip): the
reduced SPD system (P + sigma I + A^T R A) x~ = sigma x - q + A^T (rho z - y), z~ = A x~,
block-tridiagonal over the node blocks w_i = [dx_i, u_i], factored into explicit
symmetrised block inverses in the GPU's elimination order (per node: C^-1 of the u block,
G = C^-1 B^T, A' = A - B G, S_xx = (A' + E_i)^-1, S_ux = -G S_xx, S_uu = C^-1 + G S_xx G^T;
E_{i+1} = -K_{i+1,i} S_i K_{i+1,i}^T) and applied by a forward / backward block sweep.
Exact arithmetic gives the same iterates; in floating point the explicit inverses of the
ill-conditioned reduced blocks (sigma = 1e-6 against rho_eq = 20) lose digits the
quasi-definite LU does not, so this mode separates that formulation error from kernel
error in the GPU parity tests (tests/test_reduced_oracle.py).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

OSQP_INFTY = 1e30
MIN_SCALING = 1e-4
MAX_SCALING = 1e4
RHO_MIN = 1e-6
RHO_TOL = 1e-4
RHO_EQ_OVER_RHO_INEQ = 1e3
OSQP_DIVISION_TOL = 1e-30

SOLVED = 1
SOLVED_INACCURATE = 2
MAX_ITER_REACHED = -2
PRIMAL_INFEASIBLE = -3
PRIMAL_INFEASIBLE_INACCURATE = 3
DUAL_INFEASIBLE = -4
DUAL_INFEASIBLE_INACCURATE = 4
NON_CVX = -7
UNSOLVED = -10

DEFAULTS = dict(rho=0.1, sigma=1e-6, alpha=1.6, max_iter=4000, eps_abs=1e-3, eps_rel=1e-3,
                eps_prim_inf=1e-4, eps_dual_inf=1e-4, scaling=10, check_termination=25,
                warm_start=True, adaptive_rho=True)
REFERENCE_SETTINGS = dict(DEFAULTS, max_iter=100, alpha=1.4, rho=2e-2, warm_start=True, adaptive_rho=False)


def _limit(v):
    v = np.where(v < MIN_SCALING, 1.0, v)
    return np.where(v > MAX_SCALING, MAX_SCALING, v)


def _inf_norm(v):
    return float(np.max(np.abs(v))) if v.size else 0.0


def _sym(S):
    return 0.5 * (S + S.T)


class BlockReduced:
    """The GPU's linear algebra for one ADMM update (see the module docstring):
    explicit symmetrised inverses S_i of the block-tridiagonal reduced matrix and the
    forward / backward sweeps.  ``blocks``: (offset, width, ndx) of every node block."""

    def __init__(self, K: sp.csr_matrix, blocks, S_override=None):
        self.blocks = blocks
        K = K.tocsr()
        self.S, self.C = [], []
        prev = None
        for i, (o, w, X) in enumerate(blocks):
            Kii = K[o:o + w, o:o + w].toarray()
            if i > 0:
                po, pw, _ = blocks[i - 1]
                Ci = K[o:o + w, po:po + pw].toarray()
                if i > 1:  # block tridiagonal: nothing beyond the neighbour
                    qo, qw, _ = blocks[i - 2]
                    assert K[o:o + w, qo:qo + qw].nnz == 0
                Ei = -Ci @ prev @ Ci.T
            else:
                Ci, Ei = None, np.zeros((w, w))
            self.C.append(Ci)
            Xe = w if np.any(Ei[X:, :]) or np.any(Ei[:, X:]) else X  # E_i on the dx part only (else one stage)
            if Xe == w:
                S = _sym(np.linalg.inv(Kii + Ei))
            else:
                Am, Bm, Cm = Kii[:X, :X], Kii[:X, X:], Kii[X:, X:]
                Cinv = _sym(np.linalg.inv(Cm)) if w > X else np.zeros((0, 0))
                G = Cinv @ Bm.T
                Ap = Am - Bm @ G
                Sxx = _sym(np.linalg.inv(Ap + Ei[:X, :X]))
                Sux = -G @ Sxx
                Suu = _sym(Cinv + G @ Sxx @ G.T)
                S = np.block([[Sxx, Sux.T], [Sux, Suu]])
            if S_override is not None:  # diagnostics: another factor's blocks (e.g. the GPU's)
                S = S_override[i]
            self.S.append(S)
            prev = S

    def solve(self, r):
        bl, S, C = self.blocks, self.S, self.C
        bt, wv = [], []
        for i, (o, w, _) in enumerate(bl):
            b = r[o:o + w] - (C[i] @ wv[-1] if i > 0 else 0.0)
            bt.append(b)
            wv.append(S[i] @ b)
        x = np.zeros_like(r)
        xn = None
        for i in range(len(bl) - 1, -1, -1):
            o, w, _ = bl[i]
            xi = wv[i] if xn is None else S[i] @ (bt[i] - C[i + 1].T @ xn)
            x[o:o + w] = xi
            xn = xi
        return x


class OSQPRef:
    def __init__(self, P_diag, A_pattern: sp.csc_matrix, settings=None, kkt="quasi_definite", blocks=None):
        if kkt not in ("quasi_definite", "reduced_block"):
            raise ValueError(f"kkt mode {kkt}")
        if kkt == "reduced_block" and blocks is None:
            raise ValueError("reduced_block needs the node blocks")
        self.kkt = kkt
        self.blocks = blocks
        self.S_override = None
        self.s = dict(REFERENCE_SETTINGS if settings is None else settings)
        self.n = P_diag.size
        self.m = A_pattern.shape[0]
        self.P_raw = np.asarray(P_diag, dtype=float).copy()
        self.A_pat = A_pattern.tocsc()
        self.x = np.zeros(self.n)
        self.z = np.zeros(self.m)
        self.y = np.zeros(self.m)

    # ---------------------------------------------------------------- scaling
    def _scale(self, P, q, A):
        n, m, s = self.n, self.m, self.s
        D = np.ones(n)
        E = np.ones(m)
        c = 1.0
        A = A.copy()
        P = P.copy()
        q = q.copy()
        absA = abs(A)
        for _ in range(s["scaling"]):
            absA = abs(A)
            Dt = np.maximum(np.abs(P), np.asarray(absA.max(axis=0).todense()).ravel())
            Et = np.asarray(absA.max(axis=1).todense()).ravel()
            Dt = 1.0 / np.sqrt(_limit(Dt))
            Et = 1.0 / np.sqrt(_limit(Et))
            P = Dt * P * Dt
            A = sp.diags(Et) @ A @ sp.diags(Dt)
            q = Dt * q
            D = D * Dt
            E = E * Et
            c_temp = np.mean(np.abs(P))
            inf_q = _limit(np.array([_inf_norm(q)]))[0]
            c_temp = max(c_temp, inf_q)
            c_temp = _limit(np.array([c_temp]))[0]
            c_temp = 1.0 / c_temp
            P = P * c_temp
            q = q * c_temp
            c *= c_temp
        return P, q, A.tocsc(), D, E, c

    # ---------------------------------------------------------------- solve
    def update_and_solve(self, q, Ax, l, u):
        """osqp.update(q=q, Ax=Ax, l=l, u=u); osqp.solve() (ocp.py:391-401)."""
        s = self.s
        n, m = self.n, self.m
        A_raw = sp.csc_matrix((np.asarray(Ax, dtype=float), self.A_pat.indices, self.A_pat.indptr),
                              shape=self.A_pat.shape)
        l = np.maximum(np.asarray(l, dtype=float), -OSQP_INFTY)
        u = np.minimum(np.asarray(u, dtype=float), OSQP_INFTY)
        P, qs, A, D, E, c = self._scale(self.P_raw, np.asarray(q, dtype=float), A_raw)
        Dinv, Einv, cinv = 1.0 / D, 1.0 / E, 1.0 / c
        ls, us = E * l, E * u
        self.scaling = (D, E, c)
        rho = np.full(m, s["rho"])
        loose = (ls < -OSQP_INFTY * MIN_SCALING) & (us > OSQP_INFTY * MIN_SCALING)
        eq = (~loose) & (us - ls < RHO_TOL)
        rho[loose] = RHO_MIN
        rho[eq] = RHO_EQ_OVER_RHO_INEQ * s["rho"]
        rho_inv = 1.0 / rho
        sigma, alpha = s["sigma"], s["alpha"]
        if self.kkt == "quasi_definite":
            KKT = sp.bmat([[sp.diags(P + sigma), A.T], [A, sp.diags(-rho_inv)]], format="csc")
            lu = spla.splu(KKT, permc_spec="COLAMD")
        else:
            red = BlockReduced(sp.diags(P + sigma) + A.T @ sp.diags(rho) @ A, self.blocks, self.S_override)
        x, z, y = self.x.copy(), self.z.copy(), self.y.copy()
        if not s["warm_start"]:
            x[:], z[:], y[:] = 0, 0, 0
        status = UNSOLVED
        it_done = 0
        info = {}
        delta_x = np.zeros(n)
        delta_y = np.zeros(m)
        can_check = False
        for it in range(1, s["max_iter"] + 1):
            x_prev, z_prev = x, z
            if self.kkt == "quasi_definite":
                rhs = np.concatenate([sigma * x_prev - qs, z_prev - rho_inv * y])
                sol = lu.solve(rhs)
                xt = sol[:n]
                zt = (z_prev - rho_inv * y) + rho_inv * sol[n:]
            else:  # (P + sigma I + A^T R A) x~ = sigma x - q + A^T (rho z - y), z~ = A x~
                xt = red.solve(sigma * x_prev - qs + A.T @ (rho * z_prev - y))
                zt = A @ xt
            x = alpha * xt + (1 - alpha) * x_prev
            delta_x = x - x_prev
            z = np.clip(alpha * zt + (1 - alpha) * z_prev + rho_inv * y, ls, us)
            delta_y = rho * (alpha * zt + (1 - alpha) * z_prev - z)
            y = y + delta_y
            it_done = it
            can_check = s["check_termination"] and it % s["check_termination"] == 0
            if can_check:
                info = self._info(P, qs, A, x, z, y, Dinv, Einv, cinv)
                status = self._check(info, P, qs, A, ls, us, delta_x, delta_y, D, Dinv, Einv, c, cinv, False)
                if status != UNSOLVED:
                    break
        if not can_check:
            info = self._info(P, qs, A, x, z, y, Dinv, Einv, cinv)
            status = self._check(info, P, qs, A, ls, us, delta_x, delta_y, D, Dinv, Einv, c, cinv, False)
        if status == UNSOLVED:
            st2 = self._check(info, P, qs, A, ls, us, delta_x, delta_y, D, Dinv, Einv, c, cinv, True)
            status = st2 if st2 != UNSOLVED else MAX_ITER_REACHED
        info["iter"] = it_done
        info["status"] = status
        if status in (PRIMAL_INFEASIBLE, PRIMAL_INFEASIBLE_INACCURATE, DUAL_INFEASIBLE,
                      DUAL_INFEASIBLE_INACCURATE, NON_CVX):
            sol_x = np.full(n, np.nan)
            self.x[:], self.z[:], self.y[:] = 0, 0, 0
        else:
            sol_x = D * x
            self.x, self.z, self.y = x, z, y
        return sol_x, info

    def _info(self, P, q, A, x, z, y, Dinv, Einv, cinv):
        Ax = A @ x
        Px = P * x
        Aty = A.T @ y
        pri = _inf_norm(Einv * (Ax - z))
        dua = cinv * _inf_norm(Dinv * (q + Px + Aty))
        return dict(pri_res=pri, dua_res=dua, Ax=Ax, Px=Px, Aty=Aty, z=z, q=q)

    def _check(self, info, P, q, A, ls, us, delta_x, delta_y, D, Dinv, Einv, c, cinv, approximate):
        s = self.s
        eps_abs, eps_rel = s["eps_abs"], s["eps_rel"]
        eps_pinf, eps_dinf = s["eps_prim_inf"], s["eps_dual_inf"]
        if approximate:
            eps_abs, eps_rel, eps_pinf, eps_dinf = eps_abs * 10, eps_rel * 10, eps_pinf * 10, eps_dinf * 10
        if info["pri_res"] > OSQP_INFTY or info["dua_res"] > OSQP_INFTY:
            return NON_CVX
        eps_prim = eps_abs + eps_rel * max(_inf_norm(Einv * info["z"]), _inf_norm(Einv * info["Ax"]))
        prim_ok = info["pri_res"] < eps_prim
        prim_inf = False if prim_ok else self._primal_infeasible(A, ls, us, delta_y.copy(), Dinv, Einv, eps_pinf)
        eps_dual = eps_abs + eps_rel * cinv * max(_inf_norm(Dinv * q), _inf_norm(Dinv * info["Aty"]),
                                                  _inf_norm(Dinv * info["Px"]))
        dual_ok = info["dua_res"] < eps_dual
        dual_inf = False if dual_ok else self._dual_infeasible(P, q, A, ls, us, delta_x, D, Dinv, Einv, c, eps_dinf)
        if prim_ok and dual_ok:
            return SOLVED_INACCURATE if approximate else SOLVED
        if prim_inf:
            return PRIMAL_INFEASIBLE_INACCURATE if approximate else PRIMAL_INFEASIBLE
        if dual_inf:
            return DUAL_INFEASIBLE_INACCURATE if approximate else DUAL_INFEASIBLE
        return UNSOLVED

    @staticmethod
    def _primal_infeasible(A, ls, us, dy, Dinv, Einv, eps):
        big = OSQP_INFTY * MIN_SCALING
        uinf = us > big
        linf = ls < -big
        dy = np.where(uinf & linf, 0.0, np.where(uinf, np.minimum(dy, 0.0), np.where(linf, np.maximum(dy, 0.0), dy)))
        E = 1.0 / Einv
        norm_dy = _inf_norm(E * dy)
        if norm_dy > OSQP_DIVISION_TOL:
            ineq = float(np.sum(us * np.maximum(dy, 0) + ls * np.minimum(dy, 0)))
            if ineq < eps * norm_dy:
                Atdy = Dinv * (A.T @ dy)
                return _inf_norm(Atdy) < eps * norm_dy
        return False

    @staticmethod
    def _dual_infeasible(P, q, A, ls, us, dx, D, Dinv, Einv, c, eps):
        norm_dx = _inf_norm(D * dx)
        if norm_dx > OSQP_DIVISION_TOL:
            if float(np.dot(q, dx)) < c * eps * norm_dx:
                Pdx = Dinv * (P * dx)
                if _inf_norm(Pdx) < c * eps * norm_dx:
                    Adx = Einv * (A @ dx)
                    big = OSQP_INFTY * MIN_SCALING
                    bad = ((us < big) & (Adx > eps * norm_dx)) | ((ls > -big) & (Adx < -eps * norm_dx))
                    return not bool(np.any(bad))
        return False
