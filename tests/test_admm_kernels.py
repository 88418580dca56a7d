"""The three GPU mappings of the ADMM linear solve (pl_ocp_set_admm_kernel) on the MI355X.

"sweep" (k_admm: one wave per problem, node-by-node block sweeps), "sweep2" (k_admm2: two
waves per problem) and "chain" (k_admm_rc: the reduced-chain form, one workgroup per
problem) run the same OSQP 0.6 iteration (osqp.solve(), optimization/ocp.py:401) on the
same block factor; they differ only in summation order.  Bars:

* every golden fixture with every kernel forced, and the device MPC loops with the sweep
  and chain kernels: test_gpu.py (test_sqp_step_matches_golden,
  test_device_mpc_loop_matches_oracle_loop, test_device_mpc_loop_inside_benchmark_batch);
* the kernels against each other on the BASELINE fixtures: outcome exact, dx <= 1e-9;
* chain-kernel batch invariance and repeatability: bit-exact (a problem gives the same bits
  in any batch that runs this kernel; across kernels the order of the sums differs);
* the interior-point branch with the chain kernel.
"""
import numpy as np
import pytest

from conftest import golden, make_robot
from test_gpu import CONFIGS, _batched, _rel

pytestmark = pytest.mark.gpu


def _solve(name, rname, dyn, N, kernel, B=None):
    G = golden(f"sqp_{name}.npz")
    R, bo = _batched(rname, dyn, N, G, B=B)
    bo.set_admm_kernel(kernel)
    assert bo.admm_kernel() == kernel
    st = bo.solve()
    out = (st, bo.get_step(), bo.get_x())
    bo.close()
    return G, R, out


def test_general_coupling_refuses_chain_kernel():
    """The chain kernel's blocks F_i = C_i S_i[:, dx] assume one coupling row per dx_{i+1}
    column: selecting it for include_acc=False fails loudly; AUTO picks a sweep kernel."""
    from pinoloco import _lib
    G = golden("sqp_go2_rnea_fd_n20.npz")
    R, bo = _batched("go2", "whole_body_rnea", 20, G)
    assert bo.admm_kernel() in ("sweep", "sweep2")
    with pytest.raises(_lib.PinolocoError):
        bo.set_admm_kernel("chain")
    bo.close()


@pytest.mark.parametrize("name,rname,dyn,N", CONFIGS)
def test_kernels_agree(name, rname, dyn, N):
    res = {k: _solve(name, rname, dyn, N, k)[2] for k in ("sweep", "sweep2", "chain")}
    st0, dx0, _ = res["sweep"]
    for k in ("sweep2", "chain"):
        st, dx, _ = res[k]
        for key in ("status", "admm_iters", "ls_branch", "ls_trials"):
            assert np.array_equal(st[key], st0[key]), (k, key)
        for b in range(dx.shape[0]):
            assert _rel(dx[b], dx0[b]) < 1e-9, (k, b)


def test_chain_batch_invariance_and_repeatability():
    from pinoloco.ocp import BatchedOCP
    from pinoloco.synthetic import build_batch
    R = make_robot("b2g")
    lay, P, X, XS, T0 = build_batch(R, "whole_body_rnea", 50, 6, 0)

    def run(Pb, Xb):
        bo = BatchedOCP(R, "whole_body_rnea", 50, batch=Pb.shape[0], device=0)
        bo.set_admm_kernel("chain")
        bo.set_params(Pb)
        bo.set_x(Xb)
        bo.init_solver()
        st = bo.solve()
        out = (bo.get_x(), st["admm_iters"])
        bo.close()
        return out

    x1, it1 = run(P, X)
    x2, it2 = run(P, X)
    assert np.array_equal(x1, x2) and np.array_equal(it1, it2)
    x3, it3 = run(P[3:4], X[3:4])
    assert np.array_equal(x3[0], x1[3]) and it3[0] == it1[3]


@pytest.mark.parametrize("kernel", ["sweep", "chain"])
def test_bit_identical_across_batch_sizes_per_kernel(kernel):
    """A problem gives the same bits alone and inside a batch of 1024 when the same ADMM
    kernel runs both (the AUTO choice depends on the batch size; across kernels the sums
    run in other orders and agree to round-off, test_kernels_agree)."""
    from pinoloco.ocp import BatchedOCP
    from pinoloco.synthetic import build_batch
    R = make_robot("go2")
    B = 1024
    lay, P, X, XS, T0 = build_batch(R, "centroidal_vel", 20, B, 0)
    out = []
    for rows in (slice(0, B), slice(700, 701)):
        bo = BatchedOCP(R, "centroidal_vel", 20, batch=rows.stop - rows.start, device=0)
        bo.set_admm_kernel(kernel)
        bo.set_params(P[rows])
        bo.set_x(X[rows])
        bo.init_solver()
        st = bo.solve()
        out.append((bo.get_x(), st["admm_iters"]))
        bo.close()
    assert np.array_equal(out[1][0][0], out[0][0][700]) and out[1][1][0] == out[0][1][700]


def test_auto_kernel_choice():
    from pinoloco.ocp import BatchedOCP
    R = make_robot("b2")
    for B, want in ((1, "chain"), (256, "chain"), (512, "sweep2"), (1024, "sweep")):
        bo = BatchedOCP(R, "whole_body_aba", 10, batch=B, device=0)
        assert bo.admm_kernel() == want, (B, bo.admm_kernel())
        bo.close()


def test_chain_interior_point_agrees_with_sweep():
    """The interior-point branch (k_ip.hip) solves its Newton systems with one ADMM sweep
    per refinement: the chain kernel gives the same outcome and iterates to round-off."""
    from pinoloco.ocp import BatchedOCP
    G = golden("ip_go2_rnea_n20.npz")
    gait = str(G["gait"])
    R = make_robot("go2", gait)
    out = {}
    for k in ("sweep", "chain"):
        bo = BatchedOCP(R, "whole_body_rnea", 20, batch=G["P"].shape[0], device=0, gait_type=gait)
        bo.set_solver("fatrop")
        bo.set_ip_settings()
        bo.set_admm_kernel(k)
        bo.set_params(G["P"])
        bo.set_x(G["X"])
        bo.init_solver()
        bo.solve()
        out[k] = (bo.get_x(), bo.ip_stats())
        bo.close()
    xs, ss = out["sweep"]
    xc, sc = out["chain"]
    assert np.array_equal(ss["iter"], sc["iter"]) and np.array_equal(ss["status"], sc["status"])
    for b in range(xs.shape[0]):
        assert _rel(xc[b], xs[b]) < 1e-6, b


@pytest.mark.parametrize("rname,dyn,N,B,groups", [("go2", "whole_body_rnea", 20, 1, 3),
                                                  ("b2g", "whole_body_rnea", 50, 6, 7)])
def test_chain_groups_bit_identical(rname, dyn, N, B, groups):
    """k_admm_rc spreads its node phases over ceil((N + 1) / 8) workgroups per problem (r06,
    in-launch hand-offs); the node arithmetic is the same, so the iterates are bit-identical to
    the one-workgroup kernel (PL_PATH_RC_ONE_GROUP) over whole solves and MPC steps."""
    from pinoloco.ocp import BatchedOCP
    from pinoloco.synthetic import build_batch
    R = make_robot(rname)
    lay, P, X, XS, T0 = build_batch(R, dyn, N, B, 0)
    out = []
    for paths, want in (((), groups), (("rc_one_group",), 1)):
        bo = BatchedOCP(R, dyn, N, batch=B, device=0, debug_paths=paths)
        bo.set_admm_kernel("chain")
        assert bo.admm_groups() == want
        bo.set_params(P)
        bo.set_x(X)
        bo.init_solver()
        st = bo.solve()
        out.append((bo.get_x(), st["admm_iters"], st["status"]))
        bo.close()
    assert np.array_equal(out[0][0], out[1][0])
    assert np.array_equal(out[0][1], out[1][1]) and np.array_equal(out[0][2], out[1][2])
    assert np.all(np.isfinite(out[0][0]))
