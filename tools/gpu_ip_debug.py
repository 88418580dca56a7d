"""GPU side of the interior-point debugging aid: runs fixture problem(s) with
max_iter = 0, 1, 2 and dumps the iterate, multipliers and iteration-0 Newton system.
Usage (on the box): python tools/gpu_ip_debug.py FIXTURE ROBOT DYN N"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "pino-locoman_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
from conftest import golden, make_robot  # noqa: E402
from pinoloco.ocp import BatchedOCP  # noqa: E402

name, rname, dyn, N = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
G = golden(f"{name}.npz")
gait = str(G["gait"])
R = make_robot(rname, gait)
B = G["P"].shape[0]
out = {}
for mi in (0, 1, 2):
    bo = BatchedOCP(R, dyn, N, batch=B, device=0, gait_type=gait)
    bo.set_solver("fatrop")
    bo.set_ip_settings(max_iter=mi, delta_c=float(os.environ.get("IP_DC", "1e-6")), delta_w=float(os.environ.get("IP_DW", "1e-8")), n_refine=int(os.environ.get("IP_NR", "2")))
    bo.set_params(G["P"])
    bo.set_x(G["X"])
    bo.init_solver()
    bo.solve()
    st = bo.ip_stats()
    out[f"x{mi}"] = bo.get_x()
    out[f"lam{mi}"] = bo.get_lam()
    for k in ("err", "status", "iter", "alphas", "mu"):
        out[f"{k}{mi}"] = st[k]
    if mi == 1:
        for nm, ln in (("ip_dx", bo.n), ("ip_jdx", bo.m), ("rho", bo.m), ("qs", bo.n), ("xa", bo.n), ("za", bo.m), ("ip_rh", bo.m), ("ip_dl", bo.m),
                       ("ip_ds", bo.m), ("rhs", bo.n), ("Ps", bo.n)):
            out[nm] = bo.debug(nm, B * ln).reshape(B, ln)
    bo.close()
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(ROOT, "gpurun_out", f"ipdbg_{name}{os.environ.get('IP_TAG', '')}.npz"), **out)
print("ok", {k: out[k] for k in ("err0", "err1", "err2", "alphas1")})
