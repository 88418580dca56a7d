"""GPU Lagrangian Hessian (k_lag_hess, hyper-dual) against the oracle's complex-step /
finite-difference Hessian (OracleOCP.lag_hess) at each IP fixture's returned iterate
(run on the GPU box).  Usage: python tools/gpu_hess_check.py [fixture ...]"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "pino-locoman_amd")]

from conftest import golden, make_robot  # noqa: E402
from test_ip import IP_FIXTURES  # noqa: E402


def main():
    from oracle.ocp import OracleOCP
    from pinoloco.ocp import BatchedOCP
    want = set(sys.argv[1:])
    out = {}
    for name, rname, dyn, N in IP_FIXTURES:
        if want and name not in want:
            continue
        G = golden(f"{name}.npz")
        gait = str(G["gait"])
        ib = bool(int(G["include_base"])) if "include_base" in G else True
        R = make_robot(rname, gait)
        bo = BatchedOCP(R, dyn, N, batch=1, device=0, gait_type=gait, include_base=ib)
        bo.set_solver("fatrop")
        bo.set_ip_settings()
        bo.set_params(G["P"][:1])
        bo.init_solver()
        t = time.time()
        bo.ip_direction(G["x_out"][0], G["s"][0], G["lam"][0], G["zl"][0], G["zu"][0], G["mu"][0])
        tg = time.time() - t
        Hg = bo.lag_hess()[0]
        bo.close()
        o = OracleOCP(R, dyn, N, include_base=ib)
        t = time.time()
        Ho = o.lag_hess(G["x_out"][0], G["P"][0], G["lam"][0])
        to = time.time() - t
        d = abs(Hg - Ho).max()
        sc = abs(Ho).max()
        out[name] = dict(rel=float(d / sc), max_abs=float(sc), nnz_gpu=int((Hg != 0).sum()), nnz_oracle=int(Ho.nnz),
                         t_gpu=tg, t_oracle=to)
        print(name, out[name], flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", "hess_check.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
