"""Teacher-forced interior-point directions of one fixture problem with the oracle run live
(run on the GPU box): per iteration the GPU's Newton direction from the oracle's iterate,
its inertia shift against the oracle's, and the errors.
Usage: python tools/gpu_ip_tf.py fixture problem"""
import json
import os
import sys

import numpy as np

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests"), os.path.join(ROOT, "pino-locoman_amd")]

from conftest import golden, make_robot  # noqa: E402
from test_ip import IP_FIXTURES  # noqa: E402


def rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(1e-300, np.abs(np.asarray(b)).max()))


def main():
    from oracle.ip_ref import IPRef
    from oracle.ocp import OracleOCP
    from pinoloco.ocp import BatchedOCP
    name, b = sys.argv[1], int(sys.argv[2])
    _, rname, dyn, N = [f for f in IP_FIXTURES if f[0] == name][0]
    G = golden(f"{name}.npz")
    gait = str(G["gait"])
    ib = bool(int(G["include_base"])) if "include_base" in G else True
    R = make_robot(rname, gait)
    ip = IPRef(OracleOCP(R, dyn, N, include_base=ib))
    ip.s["n_refine"] = int(os.environ.get("NREF", "2"))
    x, lam, st = ip.solve(G["X"][b], G["P"][b], verbose=True)
    bo = BatchedOCP(R, dyn, N, batch=1, device=0, gait_type=gait, include_base=ib)
    bo.set_solver("fatrop")
    bo.set_ip_settings(n_refine=int(os.environ.get("NREF", "2")))
    bo.set_params(G["P"][b:b + 1])
    bo.init_solver()
    out = []
    for k, t in enumerate(ip.trace):
        bo.debug_set("ip_dwi", [0.0, float(t["dw_last"])])
        dx, dl, ds, am, az = bo.ip_direction(t["x"], t["s"], t["lam"], t["zl"], t["zu"], t["mu"])
        dwi = bo.debug("ip_dwi", 2)[0]
        e = dict(k=k, dx=rel(dx[0], t["dx"]), dl=rel(dl[0], t["dl"]), ds=rel(ds[0], t["ds"]),
                 amax=abs(am[0] - t["amax"]) / max(t["amax"], 1e-300), az=abs(az[0] - t["az"]) / max(t["az"], 1e-300),
                 dwi=float(dwi), dwi_oracle=float(t["dwi"]), tries=int(t["tries"]))
        out.append(e)
        print(json.dumps(e), flush=True)
    print("oracle status", st["status"], st["iter"], "fixture", G["status"][b], G["iter"][b],
          "x vs fixture", rel(x, G["x_out"][b]), flush=True)
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    with open(os.path.join(ROOT, "gpurun_out", f"ip_tf_{name}_{b}.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
