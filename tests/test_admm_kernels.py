"""The three GPU mappings of the ADMM linear solve (pl_ocp_set_admm_kernel) on the MI355X.

"sweep" (k_admm: one wave per problem, node-by-node block sweeps), "sweep2" (k_admm2: two
waves per problem) and "chain" (k_admm_rc: the reduced-chain form, one workgroup per
problem) run the same OSQP 0.6 iteration (osqp.solve(), optimization/ocp.py:401) on the
same block factor; they differ only in summation order.  Bars:

* every golden fixture with the chain kernel: the bars of test_gpu.py (solver outcome
  exact, dx / new iterate <= step_tol -- 1e-9 but for two named edge fixtures --,
  violation metric <= 1e-10 at the returned point);
* the kernels against each other on the BASELINE fixtures: outcome exact, dx <= 1e-9;
* chain-kernel batch invariance and repeatability: bit-exact (a problem gives the same bits
  in any batch that runs this kernel; across kernels the order of the sums differs);
* the device MPC loop and the interior-point branch with the chain kernel.
"""
import numpy as np
import pytest

from conftest import golden, make_robot
from test_gpu import ACCF, CONFIGS, EDGE, FD, _batched, _kw, _rel, step_tol

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


@pytest.mark.parametrize("name,rname,dyn,N", CONFIGS + EDGE + ACCF)
def test_chain_sqp_step_matches_golden(name, rname, dyn, N):
    from oracle.ocp import OracleOCP
    G, R, (st, dx, xn) = _solve(name, rname, dyn, N, "chain")
    o = OracleOCP(R, dyn, N, include_base=bool(int(G["include_base"])) if "include_base" in G else True)
    for b in range(G["P"].shape[0]):
        assert st["status"][b] == G["status"][b], b
        assert st["admm_iters"][b] == G["iters"][b], b
        assert st["ls_accepted"][b] == G["accepted"][b], b
        assert st["ls_branch"][b] == G["branch"][b], b
        assert st["ls_trials"][b] == G["trials"][b], b
        assert st["ls_alpha"][b] == G["alpha"][b], b
        if np.all(np.isnan(G["dx"][b])):
            assert np.all(np.isnan(dx[b])) and np.array_equal(xn[b], G["X"][b])
        else:
            assert _rel(dx[b], G["dx"][b]) < step_tol(name), b
        assert _rel(xn[b], G["x_new"][b]) < step_tol(name), b
        g, l, u = o.eval_g(xn[b], G["P"][b])
        assert st["viol_max"][b] == pytest.approx(o.violation_max(g, l, u), rel=1e-10, abs=1e-14), b


@pytest.mark.parametrize("name,rname,dyn,N", FD)
@pytest.mark.parametrize("kernel", ["sweep", "sweep2"])
def test_general_coupling_sweeps_match_golden(name, rname, dyn, N, kernel):
    """whole_body_rnea include_acc=False: the RNEA rows of node i read dv_{i+1}, so the
    factor takes the general coupling program (E_{i+1} = Wc^T Z Wc) and the sweeps the
    coupling lists with several entries per dx_{i+1} column; the test_gpu.py bars."""
    from oracle.ocp import OracleOCP
    G, R, (st, dx, xn) = _solve(name, rname, dyn, N, kernel)
    o = OracleOCP(R, dyn, N, **_kw(G))
    for b in range(G["P"].shape[0]):
        for key, gk in (("status", "status"), ("admm_iters", "iters"), ("ls_branch", "branch"),
                        ("ls_trials", "trials"), ("ls_alpha", "alpha")):
            assert st[key][b] == G[gk][b], (key, b)
        assert _rel(dx[b], G["dx"][b]) < step_tol(name), b
        assert _rel(xn[b], G["x_new"][b]) < step_tol(name), b
        g, l, u = o.eval_g(xn[b], G["P"][b])
        assert st["viol_max"][b] == pytest.approx(o.violation_max(g, l, u), rel=1e-10, abs=1e-14), b


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


@pytest.mark.parametrize("name,rname,dyn,N", [CONFIGS[0], CONFIGS[1], EDGE[0]])
def test_chain_device_mpc_loop(name, rname, dyn, N):
    G = golden(f"sqp_{name}.npz")
    R, bo = _batched(rname, dyn, N, G, B=1)
    bo.set_admm_kernel("chain")
    bo.mpc_setup(G["XS"][:1], G["T0"][:1])
    for k, want in enumerate(G["loop_states"]):
        bo.mpc_step(k)
        assert _rel(bo.mpc_state()[0], want) < 1e-7, k
        st = bo.mpc_stats()
        assert [st["status"][0], st["admm_iters"][0], st["ls_branch"][0], st["ls_trials"][0]] == \
            G["loop_stats"][k].tolist(), k
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
