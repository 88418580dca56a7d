"""Where do the step's digits go?  The GPU block factor S_i against a numpy block factor of
the GPU's own scaled QP (run on the GPU box).

For each problem of a fixture: the scaled data the GPU built (As, Ps, rho) define
K = diag(Ps) + sigma I + As^T diag(rho) As; numpy factors it node by node (LU inverses of
K_ii - C S C^T, symmetrised) and solves K x = r for a random r with the GPU's S (block
sweeps) and with a sparse LU.  Prints per problem: max relative error of each S_i, and the
relative error of one linear solve with the GPU factor.
Usage: python tools/gpu_factor_err.py fixture robot dynamics N
"""
import json
import os
import sys

import numpy as np
import scipy.sparse as sp
import scipy.sparse.linalg as spla

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "pino-locoman_amd")]

from conftest import golden  # noqa: E402
from test_gpu import _batched  # noqa: E402


def decode_S(Sflat, s_off, nw, ntile, K):
    """Lane-tile layout (state.h) -> dense symmetric nw x nw."""
    T = ntile
    M = np.zeros((4 * T, 4 * T))
    for I in range(T):
        for J in range(I + 1):
            t = I * (I + 1) // 2 + J
            ln, sl = t // K, t % K
            for r in range(4):
                for h in range(2):
                    j = 2 * r + h
                    base = s_off + ((sl * 8 + j) * 64 + ln) * 2
                    M[4 * I + r, 4 * J + 2 * h] = Sflat[base]
                    M[4 * I + r, 4 * J + 2 * h + 1] = Sflat[base + 1]
    L = np.tril(M, -1)
    D = np.diag(np.diag(M))
    full = M.copy()
    # off-diagonal tiles: upper = lower^T; diagonal tiles stored full
    for I in range(T):
        for J in range(I):
            full[4 * J:4 * J + 4, 4 * I:4 * I + 4] = M[4 * I:4 * I + 4, 4 * J:4 * J + 4].T
    del L, D
    return full[:nw, :nw]


def main():
    fix, rname, dyn, N = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    G = golden(f"sqp_{fix}.npz")
    R, bo = _batched(rname, dyn, N, G)
    bo.solve()
    B, n, m, nnz = bo.batch, bo.n, bo.m, bo.nnz
    As = bo.debug("As", B * nnz).reshape(B, nnz)
    Ps = bo.debug("Ps", B * n).reshape(B, n)
    rho = bo.debug("rho", B * m).reshape(B, m)
    S_stride = bo.sizes()["S_stride"]
    Sall = bo.debug("S", B * S_stride).reshape(B, S_stride)
    rows, cols = bo.pattern()
    nodes = bo.node_table()
    sigma = bo.settings["sigma"]
    X = R and bo.layout.ndx
    out = []
    for b in range(B):
        A = sp.csr_matrix((As[b], (rows, cols)), shape=(m, n))
        K = (sp.diags(Ps[b] + sigma) + A.T @ sp.diags(rho[b]) @ A).tocsr()
        S_np, errs, S_gpu, S_ts, errs_ts, errs_gt = [], [], [], [], [], []
        for i, nd in enumerate(nodes):
            nw, x_off, ntile, nunit, s_off = nd[0], nd[2], nd[8], nd[9], nd[10]
            Kii = K[x_off:x_off + nw, x_off:x_off + nw].toarray()
            if i > 0:
                p = nodes[i - 1]
                C = K[x_off:x_off + X, p[2]:p[2] + p[0]].toarray()
                Kii[:X, :X] -= C @ S_np[-1] @ C.T
            Si = np.linalg.inv(Kii)
            Si = 0.5 * (Si + Si.T)
            S_np.append(Si)
            # the GPU factor's two-stage formulas in numpy (k_factor.hip header), same K
            K2 = K[x_off:x_off + nw, x_off:x_off + nw].toarray()
            if i > 0:
                p = nodes[i - 1]
                C = K[x_off:x_off + X, p[2]:p[2] + p[0]].toarray()
                K2[:X, :X] -= C @ S_ts[-1] @ C.T
            if nw == X:
                St = np.linalg.inv(K2)
            else:
                A_, B_, C_ = K2[:X, :X], K2[:X, X:], K2[X:, X:]
                Ci = np.linalg.inv(C_)
                Gm = Ci @ B_.T
                Sxx = np.linalg.inv(A_ - B_ @ Gm)
                Sux = -Gm @ Sxx
                St = np.block([[Sxx, Sux.T], [Sux, Ci + Gm @ Sxx @ Gm.T]])
            St = 0.5 * (St + St.T)
            S_ts.append(St)
            errs_ts.append(float(np.abs(St - Si).max() / np.abs(Si).max()))
            Sg = decode_S(Sall[b], s_off, nw, ntile, nunit)
            S_gpu.append(Sg)
            errs.append(float(np.abs(Sg - Si).max() / np.abs(Si).max()))
            errs_gt.append(float(np.abs(Sg - St).max() / np.abs(St).max()))
        # one solve with the GPU factor (block sweeps) vs sparse LU
        rhs = np.random.default_rng(b).standard_normal(n)
        xr = spla.spsolve(K.tocsc(), rhs)
        w = []
        for i, nd in enumerate(nodes):
            nw, x_off = nd[0], nd[2]
            v = rhs[x_off:x_off + nw].copy()
            if i > 0:
                p = nodes[i - 1]
                v[:X] -= K[x_off:x_off + X, p[2]:p[2] + p[0]] @ w[-1]
            w.append(S_gpu[i] @ v)
        xg = np.zeros(n)
        xn = None
        for i in range(len(nodes) - 1, -1, -1):
            nw, x_off = nodes[i][0], nodes[i][2]
            v = rhs[x_off:x_off + nw].copy()
            if i > 0:
                p = nodes[i - 1]
                v[:X] -= K[x_off:x_off + X, p[2]:p[2] + p[0]] @ w[i - 1]
            if i + 1 < len(nodes):
                q = nodes[i + 1]
                v -= K[q[2]:q[2] + X, x_off:x_off + nw].T @ xn
            xi = S_gpu[i] @ v
            xg[x_off:x_off + nw] = xi
            xn = xi[:X]
        solve_err = float(np.abs(xg - xr).max() / np.abs(xr).max())
        worst = int(np.argmax(errs))
        out.append({"problem": b, "S_err_max": max(errs), "worst_node": worst, "solve_err": solve_err,
                    "two_stage_vs_direct": max(errs_ts), "gpu_vs_two_stage": max(errs_gt),
                    "S_err_by_node": errs})
        print(f"{fix} b={b}: S err max {max(errs):.2e} (node {worst}), one solve with the GPU factor {solve_err:.2e}; "
              f"numpy two-stage vs direct {max(errs_ts):.2e}, GPU vs numpy two-stage {max(errs_gt):.2e}")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"factor_err_{fix}.json"), "w") as f:
        json.dump(out, f)
    bo.close()


if __name__ == "__main__":
    main()
