"""Dump GPU outputs of the centroidal_vel IP fixture (bitwise A/B of two library builds).

Run on the GPU box:  [PINOLOCO_LIB=...] python tools/gpu_bits.py out.npz
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "pino-locoman_amd"))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))
from conftest import golden, make_robot  # noqa: E402
from pinoloco.ocp import BatchedOCP  # noqa: E402

G = golden("ip_go2_cv_n20.npz")
R = make_robot("go2", str(G["gait"]))
B = G["P"].shape[0]
out = {}
bo = BatchedOCP(R, "centroidal_vel", 20, batch=B, device=0, gait_type=str(G["gait"]))
bo.set_params(G["P"])
bo.set_x(G["X"])
bo.init_solver()
grad, J, g, lbg, ubg = bo.eval_sqp_data()
out.update(grad=grad, J=J, g=g)
st = bo.solve()
out["dx_osqp"] = bo.get_step()
bo.set_solver("fatrop")
bo.set_ip_settings()
bo.set_params(G["P"])
bo.set_x(G["X"])
bo.init_solver()
bo.solve()
out["x_ip"] = bo.get_x()
out["alphas"] = np.asarray(bo.ip_stats()["alphas"])
np.savez(sys.argv[1], **out)
print("ok")
