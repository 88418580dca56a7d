"""Formulation error on every SQP fixture (CPU): the reduced-form oracle's step (the GPU's
algebra in numpy, oracle/osqp_ref.py kkt="reduced_block") against the KKT oracle's golden step.
Writes profiles/r05/reduced_vs_kkt.json.  Usage: python tools/reduced_vs_kkt.py [workers]"""
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "pino-locoman_amd")]


def one(args):
    from conftest import golden, make_robot
    from oracle.ocp import OracleOCP
    from oracle.osqp_ref import REFERENCE_SETTINGS
    name, rname, dyn, N, b = args
    G = golden(f"sqp_{name}.npz")
    s = dict(REFERENCE_SETTINGS)
    s.update(eps_abs=float(G["osqp_eps"][0]), eps_rel=float(G["osqp_eps"][1]), max_iter=int(G["osqp_max_iter"]))
    kw = {k: bool(int(G[k])) for k in ("include_base", "include_acc") if k in G}
    o = OracleOCP(make_robot(rname, str(G["gait"])), dyn, N, osqp_settings=s, kkt="reduced_block", **kw)
    o.init_solver(G["X"][b], G["P"][b])
    _, dx, st = o.sqp_step(G["X"][b], G["P"][b])
    if np.all(np.isnan(G["dx"][b])):
        err = 0.0 if np.all(np.isnan(dx)) else float("inf")
    else:
        err = float(np.abs(dx - G["dx"][b]).max() / np.abs(G["dx"][b]).max())
    same = (st["status"], st["iter"], st["branch"], st["trials"]) == \
        (int(G["status"][b]), int(G["iters"][b]), int(G["branch"][b]), int(G["trials"][b]))
    return name, b, err, bool(same)


def main():
    from test_gpu import ACCF, CONFIGS, EDGE, FD
    from conftest import golden
    jobs = [(n, r, d, N, b) for n, r, d, N in CONFIGS + EDGE + ACCF + FD
            for b in range(golden(f"sqp_{n}.npz")["P"].shape[0])]
    with ProcessPoolExecutor(int(sys.argv[1]) if len(sys.argv) > 1 else 8) as ex:
        res = list(ex.map(one, jobs))
    out = {}
    for name, b, err, same in res:
        out.setdefault(name, {"problems": []})["problems"].append({"problem": b, "dx_rel": err, "outcome_exact": same})
    for name, v in out.items():
        v["max_dx_rel"] = max(p["dx_rel"] for p in v["problems"])
        v["outcome_exact"] = all(p["outcome_exact"] for p in v["problems"])
        print(f"{name:24s} {v['max_dx_rel']:.1e} {v['outcome_exact']}")
    os.makedirs(os.path.join(ROOT, "profiles", "r05"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "r05", "reduced_vs_kkt.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
