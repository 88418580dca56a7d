"""Accuracy of each stage of the GPU block factor (k_fnode: C^-1, G = C^-1 B^T, A' = A - B G;
k_fchain: S_i) against an extended-precision (x87 long double) Gauss-Jordan of the GPU's own
scaled data, next to the float64 numpy values of the same stages (run on the GPU box).
Usage: python tools/gpu_factor_stages.py fixture robot dynamics N [problem ...]
"""
import json
import os
import sys

import numpy as np
import scipy.sparse as sp

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "pino-locoman_amd"), os.path.join(ROOT, "tools")]

from conftest import golden  # noqa: E402
from gpu_factor_err import decode_S  # noqa: E402
from test_gpu import _batched  # noqa: E402

LD = np.longdouble


def gj_inv(M, dt=LD):
    M = np.array(M, dtype=dt)
    for k in range(M.shape[0]):
        p = M[k, k]
        r, c = M[k, :].copy(), M[:, k].copy()
        M -= np.outer(c, r) / p
        M[k, :], M[:, k] = r / p, c / p
        M[k, k] = -1 / p
    return -M


def rel(a, ref):
    ref = np.asarray(ref, dtype=np.float64)
    return float(np.abs(np.asarray(a, dtype=np.float64) - ref).max() / max(np.abs(ref).max(), 1e-300))


def main():
    fix, rname, dyn, N = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    probs = [int(a) for a in sys.argv[5:]]
    G = golden(f"sqp_{fix}.npz")
    _, bo = _batched(rname, dyn, N, G)
    bo.solve()
    B, n, m, nnz = bo.batch, bo.n, bo.m, bo.nnz
    As = bo.debug("As", B * nnz).reshape(B, nnz)
    Ps = bo.debug("Ps", B * n).reshape(B, n)
    rho = bo.debug("rho", B * m).reshape(B, m)
    S_stride = bo.sizes()["S_stride"]
    Sall = bo.debug("S", B * S_stride).reshape(B, S_stride)
    nodes = bo.node_table()
    X = bo.layout.ndx
    fs_off, fs = [], 0
    for nd in nodes:
        U = int(nd[1])
        fs_off.append(fs)
        fs = (fs + X * X + U * X + U * U + 31) & ~31
    fs_stride = max(fs, 32)
    FS = bo.debug("FS", B * fs_stride).reshape(B, fs_stride)
    rows, cols = bo.pattern()
    sig = bo.settings["sigma"]
    out = []
    for b in probs or range(B):
        A = sp.csr_matrix((As[b], (rows, cols)), shape=(m, n))
        K = (sp.diags(Ps[b] + sig) + A.T @ sp.diags(rho[b]) @ A).tocsr()
        S_prev_ld = None
        for i, nd in enumerate(nodes):
            nw, U, xo, ro, nr = int(nd[0]), int(nd[1]), int(nd[2]), int(nd[3]), int(nd[4])
            Ai = A[ro:ro + nr, xo:xo + nw].toarray()
            Kt = np.diag(Ps[b][xo:xo + nw] + sig) + Ai.T @ np.diag(rho[b][ro:ro + nr]) @ Ai
            Kt_ld = np.diag(np.array(Ps[b][xo:xo + nw], LD) + LD(sig)) + \
                np.array(Ai.T, LD) @ np.diag(np.array(rho[b][ro:ro + nr], LD)) @ np.array(Ai, LD)
            rec = dict(problem=b, node=i)
            o = fs_off[i]
            if U > 0:
                Ag = FS[b][o:o + X * X].reshape(X, X)
                Gg = FS[b][o + X * X:o + X * X + U * X].reshape(U, X)
                Cg = FS[b][o + X * X + U * X:o + X * X + U * X + U * U].reshape(U, U)
                C_ld, B_ld, A_ld = Kt_ld[X:, X:], Kt_ld[:X, X:], Kt_ld[:X, :X]
                Ci_ld = gj_inv(C_ld)
                G_ld = Ci_ld @ B_ld.T
                Ap_ld = A_ld - B_ld @ G_ld
                Ci_np = np.linalg.inv(Kt[X:, X:])
                G_np = Ci_np @ Kt[:X, X:].T
                Ap_np = Kt[:X, :X] - Kt[:X, X:] @ G_np
                Cg_low = np.tril(Cg) + np.tril(Cg, -1).T  # the lower triangle the chain reads
                rec.update(Cinv_gpu=rel(Cg_low, Ci_ld), Cinv_np=rel(Ci_np, Ci_ld), Cinv_gpu_asym=rel(Cg, Cg.T),
                           G_gpu=rel(Gg, G_ld), G_np=rel(G_np, G_ld), Ap_gpu=rel(Ag, Ap_ld), Ap_np=rel(Ap_np, Ap_ld))
            # S_i from the long-double chain on the same data
            Kii_ld = np.array(K[xo:xo + nw, xo:xo + nw].toarray(), LD)
            if i > 0:
                p = nodes[i - 1]
                C = np.array(K[xo:xo + nw, p[2]:p[2] + p[0]].toarray(), LD)
                Kii_ld = Kii_ld - C @ S_prev_ld @ C.T
            S_ld = gj_inv(Kii_ld)
            S_ld = (S_ld + S_ld.T) / 2
            S_prev_ld = S_ld
            Sg = decode_S(Sall[b], nd[10], nw, nd[8], nd[9])
            rec["S_gpu"] = rel(Sg, S_ld)
            out.append(rec)
            print(json.dumps({k: (f"{v:.1e}" if isinstance(v, float) else v) for k, v in rec.items()}), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"factor_stages_{fix}.json"), "w") as f:
        json.dump(out, f, indent=1)
    bo.close()


if __name__ == "__main__":
    main()
