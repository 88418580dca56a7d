"""Phase timing of the reduced-chain ADMM kernel (k_admm_rc, s_memtime on wave 0).

Run on the GPU box:  python tools/gpu_rc_timing.py robot dynamics N B [debug_path ...]
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pino-locoman_amd"))
from pinoloco import robots  # noqa: E402
from pinoloco.ocp import BatchedOCP  # noqa: E402
from pinoloco.synthetic import build_batch  # noqa: E402

rob, dyn, N, B = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
R = robots.ROBOTS[rob]()
R.set_gait_sequence("trot", 0.8)
lay, P, X, XS, T0 = build_batch(R, dyn, N, B, 0)
bo = BatchedOCP(R, dyn, N, batch=B, device=0, debug_paths=("admm_timing",) + tuple(sys.argv[5:]))
bo.set_admm_kernel("chain")
bo.set_params(P)
bo.set_x(X)
bo.init_solver()
st = bo.solve(timed=True)
T = bo.debug("admm_t", B * 40)[:B * 16].reshape(B, 16)
it = T[:, 6]
names = ["P (first)", "C1 chain", "P2", "C2 chain", "P3 + P", "barrier / hand-off waits"]
per = T[:, :6] / it[:, None]
print(f"{rob} {dyn} N={N} B={B} workgroups/problem {bo.admm_groups()}: phase_ms {st['phase_ms']}")
for k, nm in enumerate(names):
    print(f"{nm:14s} mean cycles/iteration {per[:, k].mean():10.1f}  p90 {np.percentile(per[:, k], 90):10.1f}")
print(f"total cycles/iteration {per.sum(1).mean():.1f}; C1 cycles/step {per[:, 1].mean() / N:.1f}, "
      f"C2 cycles/step {per[:, 3].mean() / (N - 1):.1f}")
sub = T[:, 8:15] / it[:, None]
if sub.sum() > 0:  # PL_RC_SUBTIMING build: node sub-phases of wave 0 (node 0), cycles per iteration
    for nm, k in zip(["loads", "coupling + u", "matvec x~", "rows / columns", "x update", "matvec g", "coupling out"], range(7)):
        print(f"  node 0 {nm:16s} {sub[:, k].mean():10.1f}")
full = bo.debug("admm_t", B * 40)
if B == 1 and sub.sum() > 0 and full[16:20].sum() > 0:  # PL_RC_SUBTIMING build: chain_fwd step sub-phases (wave 0), cycles per step
    nsteps = it[0] * (N + 1)
    for nm, k in zip(["lds + fma", "reduce + stores", "refill issue", "barrier"], range(4)):
        print(f"  C1 step {nm:16s} {full[16 + k] / nsteps:10.1f}")
