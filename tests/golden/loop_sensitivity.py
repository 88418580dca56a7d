"""Sensitivity of the whole_body_aba closed loop to round-off (test infrastructure; the numpy
oracle, no GPU).  Writes tests/golden/loop_b2_aba_n40_sensitivity.json.

For every problem of tests/golden/loop_b2_aba_n40.npz the oracle loop runs again with the initial
state x_init scaled by (1 +- 1e-15) -- a perturbation at the level of one rounding -- and the
relative state difference to the fixture's unperturbed trajectory is recorded per MPC step (the
larger of the two signs), for both linear-algebra forms: the reduced SPD system with block
inverses (kkt="reduced_block", the GPU's algebra) and the quasi-definite KKT.  Measured: the
reduced form turns the 1e-15 into ~5e-10 at step 0 of problem 0 and ~6e-7 by step 21, the KKT
form keeps it near 1e-11.  tests/test_gpu.py takes the whole_body_aba closed-loop bars from these
envelopes: no implementation whose round-off differs from the oracle's can do better.

Usage: python tests/golden/loop_sensitivity.py
"""
import json
import os
import sys
from concurrent.futures import ProcessPoolExecutor

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import make_golden as mg  # noqa: E402

EPS = 1e-15
FIX = os.path.join(HERE, "loop_b2_aba_n40.npz")


def run(args):
    j, kkt, eps = args
    G = np.load(FIX)
    ref = G["loop_states_reduced" if kkt == "reduced_block" else "loop_states"][j]
    R = mg.robots.ROBOTS["b2"]()
    R.set_gait_sequence("trot", 0.8)
    dyn, N = "whole_body_aba", 40
    lay = mg.Layout(R, dyn, N)
    o = mg.OracleOCP(R, dyn, N, kkt=kkt)
    P0, X0, XS0, t0 = mg.make_problem(R, lay, dyn, N, ("syn", int(G["gidx"][j])))
    xs, x = XS0 * (1.0 + eps), X0.copy()
    errs = []
    for k in range(ref.shape[0]):
        p = P0.copy()
        contact, swing = R.gait_sequence.get_gait_schedule(t0 + k * mg.DT_MIN, mg.horizon_dts(mg.DT_MIN, mg.DT_MAX, N), N)
        vals = {"x_init": xs, "contact_schedule": contact, "swing_schedule": swing}
        for key in vals:
            o_, s_ = lay.poff[key]
            p[o_:o_ + s_] = lay.pack(vals)[o_:o_ + s_]
        if k == 0:
            o.init_solver(x, p)
        else:
            x = o.warm_start(x, p)
        x, _, st = o.sqp_step(x, p)
        DX, U = o.split(x)
        xs = o.integrate_state(xs, DX[1])
        errs.append(float(np.linalg.norm(xs - ref[k]) / max(np.linalg.norm(ref[k]), 1e-300)))
    return errs


if __name__ == "__main__":
    n = len(np.load(FIX)["gidx"])
    jobs = [(j, kkt, s * EPS) for kkt in ("reduced_block", "quasi_definite") for j in range(n) for s in (1, -1)]
    with ProcessPoolExecutor(int(os.environ.get("GOLDEN_WORKERS", "8"))) as ex:
        res = dict(zip(jobs, ex.map(run, jobs)))
    out = {"eps": EPS, "what": "max over x_init * (1 +- eps) of the relative state difference to the unperturbed "
                              "oracle trajectory, per problem and MPC step"}
    for kkt in ("reduced_block", "quasi_definite"):
        out[kkt] = [np.maximum(res[(j, kkt, EPS)], res[(j, kkt, -EPS)]).tolist() for j in range(n)]
        print(kkt, [f"{max(v):.2e}" for v in out[kkt]])
    with open(os.path.join(HERE, "loop_b2_aba_n40_sensitivity.json"), "w") as f:
        json.dump(out, f)
