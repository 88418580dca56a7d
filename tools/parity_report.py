"""GPU vs golden errors of every SQP fixture (run on the GPU box).

Writes gpurun_out/parity_errors.json: per fixture and problem the relative
(inf-norm) errors of g, grad, J (where stored), the QP step dx and the new iterate,
and whether the solver outcome (status, iterations, branch, trials, alpha) is exact --
the step errors once per ADMM kernel (sweep, sweep2, chain) that supports the fixture.
Usage: python tools/parity_report.py   (PARITY_KERNELS=sweep,chain limits the kernels,
PARITY_TAG=x writes gpurun_out/parity_errors_x.json)
"""
import json
import os
import sys

import numpy as np
import scipy.sparse as sp

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "pino-locoman_amd")]

from conftest import golden  # noqa: E402
from test_gpu import ACCF, CONFIGS, EDGE, FD, _batched  # noqa: E402


def rel(a, b):
    a, b = np.asarray(a), np.asarray(b)
    if np.all(np.isnan(b)):
        return 0.0 if np.all(np.isnan(a)) else float("inf")
    return float(np.abs(a - b).max() / max(1e-300, np.abs(b).max()))


def main():
    out = {}
    for name, rname, dyn, N in CONFIGS + EDGE + ACCF + FD:
        G = golden(f"sqp_{name}.npz")
        out[name] = {"kernels": {}}
        for kernel in os.environ.get("PARITY_KERNELS", "sweep,sweep2,chain").split(","):
            R, bo = _batched(rname, dyn, N, G)
            try:
                bo.set_admm_kernel(kernel)
            except RuntimeError:
                bo.close()
                continue
            grad, J, g, lbg, ubg = bo.eval_sqp_data()
            rows, cols = bo.pattern()
            st = bo.solve()
            dx, xn = bo.get_step(), bo.get_x()
            recs = []
            for b in range(G["P"].shape[0]):
                r = {"g": rel(g[b], G["g"][b]), "grad": rel(grad[b], G["grad"][b]), "dx": rel(dx[b], G["dx"][b]),
                     "x_new": rel(xn[b], G["x_new"][b]),
                     "outcome_exact": bool(st["status"][b] == G["status"][b] and st["admm_iters"][b] == G["iters"][b]
                                           and st["ls_branch"][b] == G["branch"][b]
                                           and st["ls_trials"][b] == G["trials"][b]
                                           and st["ls_alpha"][b] == G["alpha"][b])}
                if f"J_data_{b}" in G:
                    Jg = sp.csr_matrix((G[f"J_data_{b}"], G[f"J_indices_{b}"], G[f"J_indptr_{b}"]), shape=(bo.m, bo.n))
                    r["J"] = rel(J[b], np.asarray(Jg[rows, cols]).ravel())
                recs.append(r)
            bo.close()
            out[name]["kernels"][kernel] = {
                "problems": recs, "outcome_exact": all(r["outcome_exact"] for r in recs),
                "max": {k: max(r[k] for r in recs if k in r) for k in ("g", "grad", "dx", "x_new")}}
            print(name, kernel, out[name]["kernels"][kernel]["max"], out[name]["kernels"][kernel]["outcome_exact"],
                  flush=True)
        out[name]["max_over_kernels"] = {k: max(v["max"][k] for v in out[name]["kernels"].values())
                                         for k in ("dx", "x_new")}
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    tag = os.environ.get("PARITY_TAG")
    with open(os.path.join(ROOT, "gpurun_out", f"parity_errors{'_' + tag if tag else ''}.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
