"""Phase timing of the factor (k_fchain and k_fnode, s_memtime on thread 0, the last launch of a
solve).  Run on the GPU box:  python tools/gpu_fchain_timing.py robot dynamics N B [fatrop]
(fatrop: the interior point's exact-Hessian factor, the last real factorisation of a solve)
Slots (k_factor.hip T(k)): 7 staging, 0 X x X sweep, 1 S_ux, 2 S_uu, 3 Y / Z, 4 E, 6 final store."""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pino-locoman_amd"))
from pinoloco import robots  # noqa: E402
from pinoloco.ocp import BatchedOCP  # noqa: E402
from pinoloco.synthetic import build_batch  # noqa: E402

rob, dyn, N, B = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
ip = len(sys.argv) > 5 and sys.argv[5] == "fatrop"
R = robots.ROBOTS[rob]()
R.set_gait_sequence("trot", 0.8)
lay, P, X, XS, T0 = build_batch(R, dyn, N, B, 0)
bo = BatchedOCP(R, dyn, N, batch=B, device=0, debug_paths=("admm_timing",))
if ip:
    bo.set_solver("fatrop")
    bo.set_ip_settings()
bo.set_params(P)
bo.set_x(X)
bo.init_solver()
bo.debug_set("admm_t", np.zeros(B * 40))
st = bo.solve()
ALL = bo.debug("admm_t", B * 40)
T = ALL[16 * B:32 * B].reshape(B, 16)[:, :8] / (N + 1)
nfac = 1 if ip else 2  # factorisations per SQP solve (setup + the rho update; k_fnode launches per group / 2)
F = ALL[32 * B:].reshape(B, 8)[:, :6] / (N + 1) / (10 if ip else nfac)  # IP: 10 Newton systems
names = {7: "staging", 0: "X sweep", 1: "S_ux", 2: "S_uu", 3: "Y / Z", 4: "E", 6: "store"}
print(f"{rob} {dyn} N={N} B={B} {'fatrop' if ip else 'osqp'} kernel={bo.admm_kernel()}: k_fchain cycles per node (thread 0)")
for k, nm in names.items():
    print(f"  {nm:10s} {T[:, k].mean():10.1f}")
print(f"  total      {T.sum(1).mean():10.1f}")
fn = {0: "staging", 1: "assembly", 2: "diag / H", 3: "u sweep", 4: "C / G store", 5: "A' MFMA"}
print("k_fnode cycles per node (thread 0, one factorisation)")
for k, nm in fn.items():
    print(f"  {nm:12s} {F[:, k].mean():10.1f}")
print(f"  total        {F.sum(1).mean():10.1f}")
