"""Headline MPC step with the batch split over S handles (one HIP stream each), stepped
back to back so their kernels overlap: solves/s for S = 1, 2, 4 (run on the GPU box).
Usage: python tools/gpu_streams.py [S ...]   (PL_ADMM_KERNEL applies to every handle)"""
import json
import os
import sys
import time

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pino-locoman_amd")]

from pinoloco import robots  # noqa: E402
from pinoloco.ocp import BatchedOCP  # noqa: E402
from pinoloco.synthetic import build_batch  # noqa: E402


def run(S, B=1024, steps=10, warmup=3, robot="b2g", dyn="whole_body_rnea", N=50):
    R = robots.ROBOTS[robot]()
    R.set_gait_sequence("trot", 0.8)
    hs = []
    for s in range(S):
        lay, P, X, XS, T0 = build_batch(R, dyn, N, B // S, s * (B // S))
        bo = BatchedOCP(R, dyn, N, batch=B // S, device=0, gait_type="trot", gait_period=0.8)
        bo.set_params(P)
        bo.set_x(X)
        bo.init_solver()
        bo.mpc_setup(XS, T0)
        hs.append(bo)
    for k in range(warmup):
        for bo in hs:
            bo.mpc_step(k)
    for bo in hs:
        bo.sync()
    t0 = time.perf_counter()
    for k in range(warmup, warmup + steps):
        for bo in hs:
            bo.mpc_step(k)
    for bo in hs:
        bo.sync()
    dt = time.perf_counter() - t0
    kern = hs[0].admm_kernel()
    for bo in hs:
        bo.close()
    return dict(S=S, solves_per_s=B * steps / dt, ms_per_step=dt / steps * 1e3, kernel=kern)


if __name__ == "__main__":
    for S in [int(a) for a in sys.argv[1:]] or [1, 2, 4]:
        print(json.dumps(run(S)), flush=True)
