"""Formulation error vs kernel error on the SQP step (run on the GPU box).

For each problem of a fixture and each ADMM kernel: the GPU step against
  * the oracle on the quasi-definite KKT (the golden dx),
  * the oracle on the GPU's own algebra (oracle/osqp_ref.py kkt="reduced_block": the reduced
    SPD system, explicit symmetrised block inverses in the GPU's elimination order),
  * the same ADMM iterations in numpy on the GPU's own scaled QP data and factor blocks S_i
    (decoded from the device), which isolates the ADMM kernel from the factor.
Usage: python tools/gpu_reduced_diag.py fixture robot dynamics N [kernel ...]
"""
import json
import os
import sys

import numpy as np
import scipy.sparse as sp

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "pino-locoman_amd"), os.path.join(ROOT, "tools")]

from conftest import golden, make_robot  # noqa: E402
from gpu_factor_err import decode_S  # noqa: E402
from oracle.ocp import OracleOCP  # noqa: E402
from oracle.osqp_ref import REFERENCE_SETTINGS, BlockReduced  # noqa: E402
from test_gpu import _batched, _kw, _settings  # noqa: E402


def rel(a, b):
    return float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-300))


def main():
    fix, rname, dyn, N = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    kernels = sys.argv[5:] or ["sweep"]
    G = golden(f"sqp_{fix}.npz")
    settings, gait = _settings(G)
    s = dict(REFERENCE_SETTINGS)
    s.update(settings)
    R = make_robot(rname, gait)
    B = G["P"].shape[0]
    red = []
    for b in range(B):
        o = OracleOCP(R, dyn, N, osqp_settings=s, kkt="reduced_block", **_kw(G))
        o.init_solver(G["X"][b], G["P"][b])
        _, dxr, st = o.sqp_step(G["X"][b], G["P"][b])
        red.append((dxr, st))
    out = []
    for kern in kernels:
        _, bo = _batched(rname, dyn, N, G)
        bo.set_admm_kernel(kern)
        st = bo.solve()
        dx = bo.get_step()
        n, m, nnz = bo.n, bo.m, bo.nnz
        As = bo.debug("As", B * nnz).reshape(B, nnz)
        Ps = bo.debug("Ps", B * n).reshape(B, n)
        rho = bo.debug("rho", B * m).reshape(B, m)
        S_stride = bo.sizes()["S_stride"]
        Sall = bo.debug("S", B * S_stride).reshape(B, S_stride)
        rows, cols = bo.pattern()
        nodes = bo.node_table()
        sig = bo.settings["sigma"]
        X = bo.layout.ndx
        for b in range(B):
            if np.all(np.isnan(G["dx"][b])):
                continue
            A = sp.csr_matrix((As[b], (rows, cols)), shape=(m, n))
            K = sp.diags(Ps[b] + sig) + A.T @ sp.diags(rho[b]) @ A
            blocks = [(int(nd[2]), int(nd[0]), X) for nd in nodes]
            br = BlockReduced(K, blocks)  # numpy factor of the GPU's scaled data
            Sg = [decode_S(Sall[b], nd[10], nd[0], nd[8], nd[9]) for nd in nodes]
            s_err = max(rel(a, c) for a, c in zip(Sg, br.S))
            o = OracleOCP(R, dyn, N, osqp_settings=s, kkt="reduced_block", **_kw(G))
            o.init_solver(G["X"][b], G["P"][b])
            o.osqp.S_override = Sg  # the oracle's ADMM with the GPU's factor blocks
            _, dx_gS, st_gS = o.sqp_step(G["X"][b], G["P"][b])
            rec = dict(fixture=fix, kernel=kern, problem=b, status=int(st["status"][b]),
                       iters=int(st["admm_iters"][b]), gpu_vs_kkt=rel(dx[b], G["dx"][b]),
                       gpu_vs_reduced=rel(dx[b], red[b][0]), reduced_vs_kkt=rel(red[b][0], G["dx"][b]),
                       reduced_outcome=[int(red[b][1]["status"]), int(red[b][1]["iter"])],
                       S_gpu_vs_numpy_on_gpu_data=s_err, gpu_vs_numpy_admm_on_gpu_factor=rel(dx[b], dx_gS),
                       numpy_admm_on_gpu_factor_vs_kkt=rel(dx_gS, G["dx"][b]))
            out.append(rec)
            print(json.dumps(rec), flush=True)
        bo.close()
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"reduced_diag_{fix}.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
