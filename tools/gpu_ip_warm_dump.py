"""Inputs of the benchmark's warm-started interior-point solves (GPU), for the oracle fixtures
that pin the failed-line-search exit (status -2): bench.py --solver fatrop's MPC loop runs
B = 1024 problems; after steps 0 and 1 this dumps, for the first NP problems, step 2's
parameters (x_init = the device state, gait at t0 + 2 dt_min), its warm start (the
OracleOCP.warm_start of step 1's solution, ocp_whole_body_rnea.py:207-235) and lam_g (step 1's
multipliers, carried as the device loop carries them), then checks that one solve of exactly
these inputs reproduces the device loop's step 2 (status, iterations, x, lam).
Usage: python tools/gpu_ip_warm_dump.py dynamics [NP]"""
import os
import sys

import numpy as np

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "pino-locoman_amd")]

from oracle.ocp import OracleOCP  # noqa: E402
from pinoloco import robots  # noqa: E402
from pinoloco.gait import horizon_dts  # noqa: E402
from pinoloco.ocp import BatchedOCP  # noqa: E402
from pinoloco.synthetic import DT_MAX, DT_MIN, build_batch  # noqa: E402


def main():
    dyn = sys.argv[1]
    NP = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    B, N, K = 1024, 50, 2
    R = robots.ROBOTS["b2g"]()
    R.set_gait_sequence("trot", 0.8)
    lay, P, X, XS, T0 = build_batch(R, dyn, N, B, 0)
    bo = BatchedOCP(R, dyn, N, batch=B, device=0, gait_type="trot", gait_period=0.8)
    bo.set_solver("fatrop")
    bo.set_ip_settings()
    bo.set_params(P)
    bo.set_x(X)
    bo.init_solver()
    bo.mpc_setup(XS, T0)
    for k in range(K):
        bo.mpc_step(k)
    xs, X1, lam1 = bo.mpc_state()[:NP], bo.get_x()[:NP], bo.get_lam()[:NP]
    st1 = {k: v[:NP].copy() for k, v in bo.ip_stats().items()}
    bo.mpc_step(K)
    st = bo.ip_stats()
    dev = {"status": st["status"][:NP].copy(), "iter": st["iter"][:NP].copy(), "alphas": st["alphas"][:NP].copy(),
           "x": bo.get_x()[:NP], "lam": bo.get_lam()[:NP]}
    P2dev = bo.get_params()[:NP]
    X1full, lam1full = bo.get_x(), bo.get_lam()
    bo.close()
    o = OracleOCP(R, dyn, N)
    P2, X2 = np.zeros((NP, lay.np)), np.zeros((NP, lay.n))
    for b in range(NP):
        contact, swing = R.gait_sequence.get_gait_schedule(T0[b] + K * DT_MIN, horizon_dts(DT_MIN, DT_MAX, N), N)
        vals = {"x_init": xs[b], "contact_schedule": contact, "swing_schedule": swing}
        P2[b] = P[b]
        for key in vals:
            o_, s_ = lay.poff[key]
            P2[b][o_:o_ + s_] = lay.pack(vals)[o_:o_ + s_]
        X2[b] = o.warm_start(X1[b], P2[b])
    print("params of step 2: host reconstruction vs device", float(np.abs(P2 - P2dev).max()))
    b2 = BatchedOCP(R, dyn, N, batch=NP, device=0, gait_type="trot", gait_period=0.8)
    b2.set_solver("fatrop")
    b2.set_ip_settings()
    b2.set_params(P2)
    b2.set_x(X2)
    b2.init_solver()
    b2.set_lam(lam1)
    b2.solve()
    s2 = b2.ip_stats()
    xr, lr = b2.get_x(), b2.get_lam()
    same = (s2["status"] == dev["status"]) & (s2["iter"] == dev["iter"])
    exs = [float(np.abs(xr[b] - dev["x"][b]).max() / np.abs(dev["x"][b]).max()) for b in range(NP)]
    ex = max(exs)
    for b in np.argsort(exs)[::-1][:6]:
        print(f"  problem {b}: x {exs[b]:.1e}, loop status {dev['status'][b]} iter {dev['iter'][b]}, "
              f"one solve {s2['status'][b]} iter {s2['iter'][b]}; step-1 status {st1['status'][b]} iter {st1['iter'][b]}")
    el = max(float(np.abs(lr[b] - dev["lam"][b]).max() / max(1.0, np.abs(dev["lam"][b]).max())) for b in range(NP))
    print(f"{dyn}: step {K} statuses {dict(zip(*np.unique(dev['status'], return_counts=True)))}; "
          f"one solve of the dumped inputs reproduces the loop: outcome {int(same.sum())}/{NP}, x {ex:.1e}, lam {el:.1e}")
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    np.savez_compressed(os.path.join(ROOT, "gpurun_out", f"ip_warm_{dyn}.npz"), P=P2, X=X2, LAM0=lam1, XS=xs,
                        T0=T0[:NP], step=K, dev_status=dev["status"], dev_iter=dev["iter"], dev_alphas=dev["alphas"],
                        dev_x=dev["x"], dev_lam=dev["lam"])
    b2.close()


if __name__ == "__main__":
    main()
