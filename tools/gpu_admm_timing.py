"""Phase timing of the ADMM sweep kernel (s_memtime, thread 0 of each workgroup).

Run on the GPU box:  python tools/gpu_admm_timing.py [B]
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pino-locoman_amd"))
from pinoloco import robots  # noqa: E402
from pinoloco.ocp import BatchedOCP  # noqa: E402
from pinoloco.synthetic import build_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
N = 50
R = robots.ROBOTS["b2g"]()
R.set_gait_sequence("trot", 0.8)
lay, P, X, XS, T0 = build_batch(R, "whole_body_rnea", N, B, 0)
bo = BatchedOCP(R, "whole_body_rnea", N, batch=B, device=0, debug_paths=("admm_timing",))
bo.set_params(P)
bo.set_x(X)
bo.init_solver()
t = time.time()
st = bo.solve(timed=True)
print("solve s", time.time() - t, "phase_ms", st["phase_ms"], "iters", np.bincount(st["admm_iters"]).nonzero())
ALL = bo.debug("admm_t", B * 40)[:B * 32]
T = ALL[:B * 16].reshape(B, 16)
it = st["admm_iters"].astype(float)
steps = it * (2 * N)  # one factor block per step
names = ["start(issue+stage)", "flush stores", "gathers+v", "prefetch issue", "matvec", "rows gather",
         "z update", "cols gather", "x update", "T0 + end"]
per = T[:, :10] / steps[:, None]
wait = T[:, 10] / steps
print(f"{'vmcnt wait':18s} mean cycles/step {wait.mean():9.1f}")
for k, nm in ((11, "  prefetch LR"), (12, "  prefetch LC"), (13, "  issue stores")):
    print(f"{nm:18s} mean cycles/step {(T[:, k] / steps).mean():9.1f}")
sub = T[:, 11:14].sum(1) / steps
for k, nm in enumerate(names):
    print(f"{nm:18s} mean cycles/step {per[:, k].mean():9.1f}  p10 {np.percentile(per[:, k], 10):9.1f}  "
          f"p90 {np.percentile(per[:, k], 90):9.1f}")
print("total cycles/step", per.sum(1).mean() + wait.mean() + sub.mean())
F = ALL[B * 16:].reshape(B, 16)[:, :8] / (N + 1)
fn = ["sweep+symm+wait", "S_ux", "S_uu", "Y", "E", "(sweep only)", "last store", "(waves1-3 work)"]
for k, nm in enumerate(fn):
    print(f"factor chain {nm:10s} mean cycles/node {F[:, k].mean():10.1f}")
print("factor chain total cycles/node", F[:, [0, 1, 2, 3, 4, 6]].sum(1).mean())
