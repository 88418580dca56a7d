"""Interior-point line-search trials per solve at the headline batch, per MPC step (GPU)."""
import os, sys, numpy as np
ROOT = os.environ.get("GRAFT_REPO_ROOT", os.getcwd())
sys.path[:0] = [ROOT, os.path.join(ROOT, "pino-locoman_amd")]
from pinoloco import robots
from pinoloco.ocp import BatchedOCP
from pinoloco.synthetic import build_batch
R = robots.ROBOTS["b2g"](); R.set_gait_sequence("trot", 0.8)
B = 1024
lay, P, X, XS, T0 = build_batch(R, "whole_body_rnea", 50, B, 0)
bo = BatchedOCP(R, "whole_body_rnea", 50, batch=B, device=0, gait_type="trot", gait_period=0.8)
bo.set_solver("fatrop"); bo.set_ip_settings(); bo.set_params(P); bo.set_x(X); bo.init_solver(); bo.mpc_setup(XS, T0)
for k in range(3):
    bo.mpc_step(k)
    st = bo.ip_stats()
    print(k, {kk: (float(np.mean(v)), float(np.max(v))) for kk, v in st.items() if kk in ("iter", "ls_trials")}, flush=True)
