"""Numerics prototype (development tool, CPU, numpy): the reduced-chain form of the ADMM
linear solve against the block sweep the GPU runs today and against a sparse LU.

K = diag(P + sigma) + A^T diag(rho) A is block tridiagonal in w_i = (dx_i, u_i), and the
sub-diagonal block K_{i+1,i} is nonzero only in the dx_{i+1} rows: C_i (ndx x nw_i).

block sweep (k_admm):   w_i = S_i (rhs_i - [C_{i-1} w_{i-1}; 0]),  x_i = S_i (bt_i - C_i^T x_{i+1,dx})
reduced chain:          g_i = S_i rhs_i, c_i = C_i g_i, h_i = g_i[dx]           (node-parallel)
                        d_{i+1} = c_i - F_i d_i,  w_i[dx] = h_i - G_i d_i          (chain, F_i = C_i S_i[:, dx],
                        e_i = w_i[dx] - F_i^T e_{i+1}                              G_i = S_i[dx, dx])
                        x_i = S_i (rhs_i - [d_i; 0] - C_i^T e_{i+1})               (node-parallel)

Usage: python tools/proto_chain.py [fixture] [problem]
"""
import os
import sys

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "pino-locoman_amd"))

from oracle import osqp_ref  # noqa: E402
from oracle.ocp import OracleOCP  # noqa: E402
from pinoloco import robots  # noqa: E402


def capture_qp(fix, b):
    d = np.load(os.path.join(HERE, "..", "tests", "golden", fix + ".npz"))
    name = fix.split("_")
    rob, rest = name[1], "_".join(name[2:])
    dyn = {"rnea": "whole_body_rnea", "aba": "whole_body_aba", "acc": "whole_body_acc", "cv": "centroidal_vel"}[
        rest.split("_")[0]]
    N = int([t for t in name if t.startswith("n") and t[1:].isdigit()][0][1:])
    R = robots.ROBOTS[rob]()
    R.set_gait_sequence(str(d["gait"]) if d["gait"].shape == () else "trot", 0.8)
    o = OracleOCP(R, dyn, N)
    x, p = d["X"][b], d["P"][b]
    o.init_solver(x, p)
    f, grad = o.f_and_grad(x, p)
    g, lbg, ubg = o.eval_g(x, p)
    Ax = o.jacobian_values(x, p)
    s = o.osqp
    A_raw = sp.csc_matrix((Ax, s.A_pat.indices, s.A_pat.indptr), shape=s.A_pat.shape)
    l = np.maximum(lbg - g, -osqp_ref.OSQP_INFTY)
    u = np.minimum(ubg - g, osqp_ref.OSQP_INFTY)
    P, qs, A, D, E, c = s._scale(s.P_raw, grad, A_raw)
    ls, us = E * l, E * u
    rho = np.full(s.m, s.s["rho"])
    loose = (ls < -osqp_ref.OSQP_INFTY * osqp_ref.MIN_SCALING) & (us > osqp_ref.OSQP_INFTY * osqp_ref.MIN_SCALING)
    eq = (~loose) & (us - ls < osqp_ref.RHO_TOL)
    rho[loose] = osqp_ref.RHO_MIN
    rho[eq] = osqp_ref.RHO_EQ_OVER_RHO_INEQ * s.s["rho"]
    return o, P, qs, A, ls, us, rho, s.s["sigma"], s.s["alpha"]


def blocks(o, n):
    offs = list(o.x_off) + [n]
    return [(offs[i], offs[i + 1]) for i in range(len(offs) - 1)]


def block_factor(K, bl, ndx):
    """S_i = (K_ii - C_{i-1} S_{i-1}[dx... ] ...)^-1 by block elimination, symmetrised (as k_factor)."""
    S = []
    for i, (a, b) in enumerate(bl):
        Kii = K[a:b, a:b].toarray()
        if i > 0:
            pa, pb = bl[i - 1]
            Ci = K[a:a + ndx, pa:pb].toarray()  # C_{i-1}
            Kii[:ndx, :ndx] -= Ci @ S[-1] @ Ci.T
        Si = np.linalg.inv(Kii)
        S.append(0.5 * (Si + Si.T))
    return S


def gj_inv(M, equil=False):
    """Gauss-Jordan inverse without pivoting (the sweep operator the GPU factor runs), optionally
    on the symmetrically equilibrated matrix D M D, D = diag(M)^-1/2."""
    M = np.array(M, dtype=float)
    n = M.shape[0]
    d = np.ones(n)
    if equil:
        d = 1.0 / np.sqrt(np.abs(np.diag(M)))
        M = d[:, None] * M * d[None, :]
    for k in range(n):
        p = M[k, k]
        rowk = M[k, :].copy()
        colk = M[:, k].copy()
        M -= np.outer(colk, rowk) / p
        M[k, :] = rowk / p
        M[:, k] = -colk / p
        M[k, k] = 1.0 / p
    M = -M  # sweep gives -M^-1 off the swept block convention; fix sign below
    M = -M
    return d[:, None] * M * d[None, :]


def block_factor_two_stage(K, bl, ndx):
    """The GPU factor's formulas (k_factor.hip): C^-1 of the u block, A' = A - B C^-1 B^T,
    S_xx = (A' + E)^-1, S_ux = -G S_xx (G = C^-1 B^T), S_uu = C^-1 + G S_xx G^T, symmetrised."""
    S = []
    for i, (a, b) in enumerate(bl):
        Kii = K[a:b, a:b].toarray()
        Eb = np.zeros((ndx, ndx))
        if i > 0:
            pa, pb = bl[i - 1]
            Ci = K[a:a + ndx, pa:pb].toarray()
            Eb = -Ci @ S[-1] @ Ci.T
        X = ndx
        if b - a == X:
            Si = INV(Kii + Eb)
        else:
            A_, B_, C_ = Kii[:X, :X], Kii[:X, X:], Kii[X:, X:]
            inv = INV
            Ci_ = inv(C_)
            G = Ci_ @ B_.T
            Ap = A_ - B_ @ G
            Sxx = inv(Ap + Eb)
            Sux = -G @ Sxx
            Suu = Ci_ + G @ Sxx @ G.T
            Si = np.block([[Sxx, Sux.T], [Sux, Suu]])
        S.append(0.5 * (Si + Si.T))
    return S


def solve_sweep(K, S, bl, ndx, rhs):
    N1 = len(bl)
    w = [None] * N1
    for i, (a, b) in enumerate(bl):
        v = rhs[a:b].copy()
        if i > 0:
            pa, pb = bl[i - 1]
            v[:ndx] -= K[a:a + ndx, pa:pb] @ w[i - 1]
        w[i] = S[i] @ v
    x = np.zeros_like(rhs)
    xn = None
    for i in range(N1 - 1, -1, -1):
        a, b = bl[i]
        v = rhs[a:b].copy()
        if i > 0:
            pa, pb = bl[i - 1]
            v[:ndx] -= K[a:a + ndx, pa:pb] @ w[i - 1]
        if i < N1 - 1:
            na, nb = bl[i + 1]
            v -= K[na:na + ndx, a:b].T @ xn
        xi = S[i] @ v
        x[a:b] = xi
        xn = xi[:ndx]
    return x


def chain_setup(K, S, bl, ndx):
    C, F, G = [], [], []
    for i, (a, b) in enumerate(bl):
        G.append(S[i][:ndx, :ndx].copy())
        if i + 1 < len(bl):
            na, nb = bl[i + 1]
            Ci = K[na:na + ndx, a:b].toarray()
            C.append(Ci)
            F.append(Ci @ S[i][:, :ndx])
    return C, F, G


def solve_chain(S, C, F, G, bl, ndx, rhs):
    N1 = len(bl)
    g = [S[i] @ rhs[a:b] for i, (a, b) in enumerate(bl)]
    c = [C[i] @ g[i] for i in range(N1 - 1)]
    d = [np.zeros(ndx)]
    wdx = []
    for i in range(N1):
        wdx.append(g[i][:ndx] - G[i] @ d[i])
        if i + 1 < N1:
            d.append(c[i] - F[i] @ d[i])
    e = [None] * (N1 + 1)
    e[N1 - 1] = wdx[N1 - 1]
    for i in range(N1 - 2, -1, -1):
        e[i] = wdx[i] - F[i].T @ e[i + 1]
    x = np.zeros_like(rhs)
    for i, (a, b) in enumerate(bl):
        u = rhs[a:b].copy()
        u[:ndx] -= d[i]
        if i + 1 < N1:
            u -= C[i].T @ e[i + 1]
        x[a:b] = S[i] @ u
    return x


def admm(solve, P, qs, A, ls, us, rho, sigma, alpha, iters):
    n, m = A.shape[1], A.shape[0]
    x, z, y = np.zeros(n), np.zeros(m), np.zeros(m)
    hist = []
    for _ in range(iters):
        rhs = sigma * x - qs + A.T @ (rho * z - y)
        xt = solve(rhs)
        zt = A @ xt
        xn = alpha * xt + (1 - alpha) * x
        zr = alpha * zt + (1 - alpha) * z
        zn = np.clip(zr + y / rho, ls, us)
        y = y + rho * (zr - zn)
        x, z = xn, zn
        hist.append(x.copy())
    return hist


MODE = os.environ.get("PROTO_INV", "lu")
INV = {"lu": np.linalg.inv, "gj": gj_inv, "gje": lambda M: gj_inv(M, True)}[MODE]


def main():
    fix = sys.argv[1] if len(sys.argv) > 1 else "sqp_go2_rnea_n20"
    b = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    o, P, qs, A, ls, us, rho, sigma, alpha = capture_qp(fix, b)
    n = A.shape[1]
    K = (sp.diags(P + sigma) + A.T @ sp.diags(rho) @ A).tocsr()
    bl = blocks(o, n)
    ndx = o.ndx
    # structure checks the chain relies on
    for i in range(len(bl)):
        for j in range(len(bl)):
            if abs(i - j) > 1:
                a, b_ = bl[i]
                c_, d_ = bl[j]
                assert abs(K[a:b_, c_:d_]).sum() == 0
        if i > 0:
            a, b_ = bl[i]
            pa, pb = bl[i - 1]
            assert abs(K[a + ndx:b_, pa:pb]).sum() == 0
    S = block_factor(K, bl, ndx)
    if os.environ.get("PROTO_TWO_STAGE"):
        S = block_factor_two_stage(K, bl, ndx)
    C, F, G = chain_setup(K, S, bl, ndx)
    lu = spla.splu(sp.bmat([[sp.diags(P + sigma), A.T], [A, sp.diags(-1.0 / rho)]], format="csc"))
    m = A.shape[0]

    def solve_lu(rhs_x):
        # the quasi-definite KKT with rhs [sigma x - q; z - y/rho] equals K x = rhs_x here
        sol = lu.solve(np.concatenate([rhs_x, np.zeros(m)]))
        return sol[:n]

    Kc = K.tocsc()
    lu2 = spla.splu(Kc)
    rhs = np.random.default_rng(0).standard_normal(n)
    xr = lu2.solve(rhs)
    for nm, fn in [("sweep", lambda r: solve_sweep(K, S, bl, ndx, r)), ("chain", lambda r: solve_chain(S, C, F, G, bl, ndx, r))]:
        xs = fn(rhs)
        print(f"{nm}: one solve rel err vs LU {np.abs(xs - xr).max() / np.abs(xr).max():.3e}")
    its = 100
    ref = admm(lambda r: lu2.solve(r), P, qs, A, ls, us, rho, sigma, alpha, its)
    for nm, fn in [("sweep", lambda r: solve_sweep(K, S, bl, ndx, r)), ("chain", lambda r: solve_chain(S, C, F, G, bl, ndx, r))]:
        h = admm(fn, P, qs, A, ls, us, rho, sigma, alpha, its)
        errs = [np.abs(h[k] - ref[k]).max() / np.abs(ref[k]).max() for k in (0, 24, 49, 99)]
        print(f"{nm}: ADMM x rel err vs LU at it 1/25/50/100: " + " ".join(f"{e:.2e}" for e in errs))
    print("norms: S max", max(np.abs(s).max() for s in S), "F max", max(np.abs(f).max() for f in F))


if __name__ == "__main__":
    main()
