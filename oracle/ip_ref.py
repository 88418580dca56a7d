"""ORACLE (test infrastructure only) -- the interior-point solve of the reference's
Fatrop branch, restated in numpy.

The reference's default solver is Fatrop through CasADi Opti (``run_mpc.py:34-37``;
``ocp.py:248-263`` sets max_iter 10, tol 1e-3, mu_init 1e-4, warm_start_init_point,
bound_push 1e-7, warm_start_mult_bound_push 1e-7; ``ocp.py:360-373`` solves, falls
back to ``opti.debug`` when the solver does not converge, and stores ``lam_g``).
Fatrop (and BLASFEO) are absent from this container and from /root/reference, so its
published algorithm -- an IPOPT-style primal-dual barrier method with a filter line
search (Vanroye et al., "FATROP: A Fast Constrained Optimal Control Problem Solver
for Robot Trajectory Optimization and Control", IROS 2023; Waechter & Biegler,
Math. Prog. 106, 2006) -- is restated here, with these documented choices:

* problem: min f(x) s.t. g_E(x) = lbg_E (rows with lbg == ubg) and
  lbg_I <= s = g_I(x) <= ubg_I (slacks on the other rows, bounds on s only);
* Hessian (``hessian="exact"``, the default): the exact Lagrangian Hessian CasADi gives
  the Opti/Fatrop solve (``expand=True``): the objective's constant diagonal
  (``ocp.py:293-296``) + sum_r lam_r d^2 g_r / dx^2 (``OracleOCP.lag_hess``, block
  diagonal over the w_i since the rows are linear in dx_{i+1}) + delta_w I, with IPOPT's
  inertia correction (Waechter & Biegler 2006, Algorithm IC; Fatrop corrects the same way
  when its Riccati recursion meets a block that is not positive definite): the reduced
  matrix must be positive definite, else a shift delta I is added -- first 1e-4, or a
  third of the last shift of this solve, then x100 while no shift has succeeded in this
  solve, x8 after -- at most ``inertia_cap`` times.  ``hessian="gauss_newton"``: the
  objective's diagonal only (the OSQP branch's Hessian);
* Newton system: the slacks, bound multipliers and constraint multipliers are
  eliminated, leaving the reduced SPD system
      (H + J^T W J) dx = -(grad + J^T lam) - J^T W r^
  with W_E = 1/delta_c and W_I = Sigma / (1 + delta_c Sigma) (a fixed dual
  regularisation delta_c = 1e-4 in place of Fatrop's generalised Riccati on the
  exact KKT; the fixed point of the iteration is unchanged, since dlam -> 0 there.
  delta_c trades the constraint progress of one step, J dx + r = delta_c dlam,
  against the conditioning of the reduced system: at 1e-4 the GPU's block-inverse
  factor reproduces a sparse LU to ~1e-12, at 1e-6 it loses ~5 digits);
  This is the same block-tridiagonal operator the OSQP branch factors, so the GPU
  path reuses its factor and sweep kernels; ``n_refine`` iterative-refinement solves
  on the KKT x-row residual follow the first solve;
* initial point (warm_start_init_point): x from the warm start; slacks pushed into
  the interior with bound_push / bound_frac.  Cold (no lam_g yet, the reference's first
  solve): lam = 0 and the slack-bound multipliers centred, z = mu_init / slack.  Warm
  (``lam0`` given: the previous solve's lam_g, which the reference stores at ``ocp.py:373``
  and passes back with ``opti.set_initial(opti.lam_g, lam_g)``,
  ``ocp_whole_body_rnea.py:234-235``, ``ocp_whole_body_acc.py:164-165``): lam = lam0 and,
  as IPOPT's warm_start_init_point does for the slack bounds, the multipliers split by the
  sign of lam (stationarity in s: z_u - z_l = lam), z_l = max(-lam, 0), z_u = max(lam, 0),
  each pushed up to warm_start_mult_bound_push (1e-7, ``ocp.py:260``);
* barrier parameter: IPOPT's monotone rule mu <- max(tol / 10, min(kappa_mu mu,
  mu^theta_mu)) when E_mu <= kappa_eps mu (with tol 1e-3 and mu_init 1e-4 mu stays
  at 1e-4);
* line search: fraction-to-boundary tau = max(0.99, 1 - mu) on slacks and bound
  multipliers, backtracking by halves from alpha_max (at most ``ls_max`` trials),
  IPOPT's filter with the switching condition, Armijo on the barrier objective
  and the sufficient-decrease alternatives; a failed line search ends the solve
  with status -2 (the feasibility restoration phase is not restated);
* termination: IPOPT's scaled NLP error E_0 <= tol (s_max = 100), checked at the
  start of every iteration including after the last step; status 1 converged,
  -1 maximum iterations (the reference then uses ``opti.debug``'s iterate), -2
  line-search failure, -3 non-finite step.

PARITY UNPINNED against Fatrop itself (not available); the GPU path is checked
against this restatement (tests/test_ip.py, tests/golden/ip_*.npz).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

# ocp.py:254-262 (reference settings) + IPOPT / Fatrop defaults for the rest
IP_SETTINGS = dict(max_iter=10, tol=1e-3, mu_init=1e-4, bound_push=1e-7, bound_frac=1e-2,
                   warm_start_mult_bound_push=1e-7, delta_w=1e-8, delta_c=1e-4, ls_max=12, n_refine=8,
                   hessian="exact", inertia_cap=8, kkt_refine="regularized")
KAPPA_EPS, KAPPA_MU, THETA_MU = 10.0, 0.2, 1.5
TAU_MIN, S_MAX, KAPPA_SIGMA = 0.99, 100.0, 1e10
GAMMA_THETA, GAMMA_PHI, DELTA, S_THETA, S_PHI, ETA_PHI = 1e-5, 1e-8, 1.0, 1.1, 2.3, 1e-8
W_MIN = 1e-20

ST_CONVERGED, ST_MAX_ITER, ST_LS_FAIL, ST_NONFINITE = 1, -1, -2, -3


def row_classes(lbg, ubg):
    eq = lbg == ubg
    hl = ~eq & np.isfinite(lbg)
    hu = ~eq & np.isfinite(ubg)
    return eq, hl, hu


def push_slacks(g, lbg, ubg, eq, hl, hu, push, frac):
    """IPOPT's bound push of the initial slacks (Waechter & Biegler 2006, sec. 3.6)."""
    lb = np.where(hl, lbg, 0.0)
    ub = np.where(hu, ubg, 0.0)
    pl = push * np.maximum(1.0, np.abs(lb))
    pu = push * np.maximum(1.0, np.abs(ub))
    two = hl & hu
    width = np.where(two, ub - lb, np.inf)
    pl = np.where(two, np.minimum(pl, frac * width), pl)
    pu = np.where(two, np.minimum(pu, frac * width), pu)
    s = np.array(g, dtype=float, copy=True)
    s = np.where(hl, np.maximum(s, lb + pl), s)
    s = np.where(hu, np.minimum(s, ub - pu), s)
    return np.where(eq, 0.0, s)


def is_pd(K):
    """Positive definiteness of the reduced Newton matrix (dense Cholesky)."""
    try:
        np.linalg.cholesky(K.toarray())
    except np.linalg.LinAlgError:
        return False
    return True


def frac_to_boundary(v, dv, tau, mask):
    """max alpha in (0, 1] with v + alpha dv >= (1 - tau) v on the masked entries."""
    neg = mask & (dv < 0)
    if not np.any(neg):
        return 1.0
    return float(min(1.0, np.min(-tau * v[neg] / dv[neg])))


class IPRef:
    def __init__(self, ocp, settings=None):
        self.o = ocp
        self.s = dict(IP_SETTINGS)
        self.s.update(settings or {})
        self.trace = []  # per iteration: the Newton system and direction (debugging aid)

    # ---- merit pieces
    @staticmethod
    def _c(g, s, lbg, eq):
        return np.where(eq, g - np.where(eq, lbg, 0.0), g - s)

    def _phi(self, f, sl, su, hl, hu, mu):
        return f - mu * (np.sum(np.log(sl[hl])) + np.sum(np.log(su[hu])))

    def solve(self, x0, p, lam0=None, verbose=False):
        """Returns x, lam, dict(status, iter, err, mu, f, alphas, trials).  lam0: the
        multipliers of a previous solve (warm start, see the module docstring)."""
        o, st = self.o, self.s
        mu = st["mu_init"]
        tol = st["tol"]
        dw, dc = st["delta_w"], st["delta_c"]
        H = o.compute_hess_diag(p) + dw
        exact = st["hessian"] == "exact"
        dw_last = 0.0  # the last nonzero inertia shift of this solve
        x = np.array(x0, dtype=float, copy=True)
        g, lbg, ubg = o.eval_g(x, p)
        eq, hl, hu = row_classes(lbg, ubg)
        iq = ~eq
        lb = np.where(hl, lbg, 0.0)
        ub = np.where(hu, ubg, 0.0)
        s = push_slacks(g, lbg, ubg, eq, hl, hu, st["bound_push"], st["bound_frac"])
        m = g.size
        sl = np.where(hl, s - lb, 1.0)
        su = np.where(hu, ub - s, 1.0)
        if lam0 is None:
            lam = np.zeros(m)
            zl = np.where(hl, mu / sl, 0.0)
            zu = np.where(hu, mu / su, 0.0)
        else:
            lam = np.array(lam0, dtype=float, copy=True)
            wp = st["warm_start_mult_bound_push"]
            zl = np.where(hl, np.maximum(np.maximum(-lam, 0.0), wp), 0.0)
            zu = np.where(hu, np.maximum(np.maximum(lam, 0.0), wp), 0.0)
        nb = int(hl.sum() + hu.sum())
        theta0 = float(np.sum(np.abs(self._c(g, s, lbg, eq))))
        theta_max = 1e4 * max(1.0, theta0)
        theta_min = 1e-4 * max(1.0, theta0)
        filt = []
        status, it = ST_MAX_ITER, 0
        alphas, trials_all = [], []
        err = np.inf
        f = np.nan
        for k in range(st["max_iter"] + 1):
            it = k
            f, grad = o.f_and_grad(x, p)
            g, _, _ = o.eval_g(x, p)
            J = o.eval_J(x, p).tocsr()
            c = self._c(g, s, lbg, eq)
            rx = grad + J.T @ lam
            rs = np.where(iq, -lam - zl + zu, 0.0)
            sd = max(S_MAX, (np.sum(np.abs(lam)) + np.sum(zl) + np.sum(zu)) / max(m + nb, 1)) / S_MAX
            sc = max(S_MAX, (np.sum(zl) + np.sum(zu)) / max(nb, 1)) / S_MAX
            cl, cu = np.where(hl, sl * zl, 0.0), np.where(hu, su * zu, 0.0)

            def nlp_err(mu_):
                comp = max(np.max(np.abs(np.where(hl, cl - mu_, 0.0)), initial=0.0),
                           np.max(np.abs(np.where(hu, cu - mu_, 0.0)), initial=0.0))
                return max(np.max(np.abs(rx)) / sd, np.max(np.abs(rs)) / sd, np.max(np.abs(c)), comp / sc)

            err = nlp_err(0.0)
            if not np.isfinite(err):
                status = ST_NONFINITE
                break
            if err <= tol:
                status = ST_CONVERGED
                break
            if k == st["max_iter"]:
                status = ST_MAX_ITER
                break
            # monotone barrier update (IPOPT Algorithm A, step A-3)
            for _ in range(4):
                if nlp_err(mu) > KAPPA_EPS * mu:
                    break
                mu_new = max(tol / 10.0, min(KAPPA_MU * mu, mu ** THETA_MU))
                if mu_new == mu:
                    break
                mu = mu_new
                filt = []
            # ---- reduced Newton system
            sig = np.where(hl, zl / sl, 0.0) + np.where(hu, zu / su, 0.0)
            W = np.where(eq, 1.0 / dc, sig / (1.0 + dc * sig))
            W = np.maximum(W, W_MIN)
            bs = np.where(iq, lam + np.where(hl, mu / sl, 0.0) - np.where(hu, mu / su, 0.0), 0.0)
            sig_safe = np.where(iq, sig, 1.0)
            rhat = np.where(eq, c, c - bs / sig_safe)
            Kb = sp.diags(H) + J.T @ sp.diags(W) @ J
            Hl = o.lag_hess(x, p, lam) if exact else sp.csr_matrix((x.size, x.size))
            Kb = (Kb + Hl).tocsc()
            dw_before, dwi, tries = dw_last, 0.0, 0
            while exact:  # inertia correction (module docstring)
                if is_pd(Kb + dwi * sp.eye(x.size)):
                    if dwi > 0.0:
                        dw_last = dwi
                    break
                if tries >= st["inertia_cap"]:
                    break
                dwi = ((1e-4 if dw_last == 0.0 else max(1e-20, dw_last / 3.0)) if dwi == 0.0
                       else dwi * (100.0 if dw_last == 0.0 else 8.0))
                tries += 1
            K = (Kb + dwi * sp.eye(x.size)).tocsc()
            rhs = -rx - J.T @ (W * rhat)
            lu = spla.splu(K)
            if st["kkt_refine"] == "exact":
                # delta_c regularises the factor only: iterative refinement on the UNREGULARISED
                # KKT  [H_K  J^T; J  -D] [dx; dl] = [-rx; -rhat]  (D = 0 on equality rows, 1/Sigma on
                # the others), each correction solved with the regularised factor
                #   K ex = r1 + J^T W r2,  el = W (J ex - r2)
                # The iteration contracts (eigenvalues of delta_c (D + delta_c + J H_K^-1 J^T)^-1 in
                # [0, 1)), so the refined step tends to the delta_c = 0 Newton step that Fatrop's
                # Riccati recursion computes on the exact KKT.  The first solve is the first
                # correction from dx = dl = 0.
                Dd = np.where(eq, 0.0, 1.0 / sig_safe)
                dx, dl = np.zeros(x.size), np.zeros(m)
                for _ in range(st["n_refine"] + 1):
                    r1 = -(grad + J.T @ (lam + dl)) - (H + dwi) * dx - Hl @ dx
                    r2 = -rhat - J @ dx + Dd * dl
                    ex = lu.solve(r1 + J.T @ (W * r2))
                    dx = dx + ex
                    dl = dl + W * (J @ ex - r2)
            else:  # "regularized" (r02-r05): the step of the delta_c-regularised KKT
                dx = lu.solve(rhs)
                for _ in range(st["n_refine"]):  # iterative refinement on the reduced x-row residual
                    res = -(grad + J.T @ (lam + W * (J @ dx + rhat))) - (H + dwi) * dx - Hl @ dx
                    dx = dx + lu.solve(res)
                dl = W * (J @ dx + rhat)
            ds = np.where(iq, (bs + dl) / sig_safe, 0.0)
            dzl = np.where(hl, mu / sl - zl - zl / sl * ds, 0.0)
            dzu = np.where(hu, mu / su - zu + zu / su * ds, 0.0)
            if not (np.all(np.isfinite(dx)) and np.all(np.isfinite(dl))):
                status = ST_NONFINITE
                break
            tau = max(TAU_MIN, 1.0 - mu)
            amax = min(frac_to_boundary(sl, ds, tau, hl), frac_to_boundary(su, -ds, tau, hu))
            az = min(frac_to_boundary(zl, dzl, tau, hl), frac_to_boundary(zu, dzu, tau, hu))
            self.trace.append(dict(x=x.copy(), s=s.copy(), lam=lam.copy(), zl=zl.copy(), zu=zu.copy(), mu=mu, W=W,
                                   rhat=rhat, rx=rx, rhs=rhs, dx=dx, dl=dl, ds=ds, jdx=J @ dx, amax=amax, az=az,
                                   dw_last=dw_before, dwi=dwi, tries=tries))
            theta = float(np.sum(np.abs(c)))
            phi = self._phi(f, sl, su, hl, hu, mu)
            dphi = float(grad @ dx + np.sum(np.where(hl, -mu / sl, 0.0) * ds + np.where(hu, mu / su, 0.0) * ds))
            accepted, ftype = False, False
            a, t = amax, 0
            for t in range(st["ls_max"]):
                a = amax * 0.5 ** t
                xt = x + a * dx
                stt = s + a * ds
                ft, _ = o.f_and_grad(xt, p)
                gt, _, _ = o.eval_g(xt, p)
                slt = np.where(hl, stt - lb, 1.0)
                sut = np.where(hu, ub - stt, 1.0)
                th_t = float(np.sum(np.abs(self._c(gt, stt, lbg, eq))))
                ph_t = self._phi(ft, slt, sut, hl, hu, mu)
                if verbose:
                    print(f"  it {k} trial {t} a {a:.3e} theta {theta:.4e} -> {th_t:.4e}  phi {phi:.6e} -> {ph_t:.6e}"
                          f"  dphi {dphi:.3e} amax {amax:.3e} az {az:.3e} |dx| {np.max(np.abs(dx)):.3e}")
                if not (np.isfinite(th_t) and np.isfinite(ph_t)) or th_t > theta_max:
                    continue
                if any(th_t >= tf and ph_t >= pf for tf, pf in filt):
                    continue
                switching = dphi < 0 and a * (-dphi) ** S_PHI > DELTA * theta ** S_THETA
                if theta <= theta_min and switching:
                    if ph_t <= phi + ETA_PHI * a * dphi:
                        accepted, ftype = True, True
                        break
                elif th_t <= (1 - GAMMA_THETA) * theta or ph_t <= phi - GAMMA_PHI * theta:
                    accepted = True
                    break
            trials_all.append(t + 1)
            if not accepted:
                status = ST_LS_FAIL
                alphas.append(0.0)
                break
            alphas.append(a)
            if not ftype:
                filt.append(((1 - GAMMA_THETA) * theta, phi - GAMMA_PHI * theta))
            x = x + a * dx
            s = s + a * ds
            lam = lam + a * dl
            zl = zl + az * dzl
            zu = zu + az * dzu
            sl = np.where(hl, s - lb, 1.0)
            su = np.where(hu, ub - s, 1.0)
            # bound-multiplier safeguard (IPOPT eq. 16)
            zl = np.where(hl, np.clip(zl, mu / (KAPPA_SIGMA * sl), KAPPA_SIGMA * mu / sl), 0.0)
            zu = np.where(hu, np.clip(zu, mu / (KAPPA_SIGMA * su), KAPPA_SIGMA * mu / su), 0.0)
        return x, lam, dict(status=status, iter=it, err=float(err), mu=mu, f=float(f), alphas=np.array(alphas),
                            trials=np.array(trials_all, dtype=int), s=s, zl=zl, zu=zu)
