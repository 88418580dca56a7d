"""The round-4 rewrites of the Jacobian, the Lagrangian Hessian and the factor chain against
the paths they replaced, on the same handle inputs (the replaced paths are selected by the
handle's pl_ocp_desc.debug_paths bits, BatchedOCP(debug_paths=...)).  Each rewrite is an exact identity in real arithmetic, so the two paths agree to
round-off:

* Jacobian (k_eval_jac_lin: the rnea / acc a and f columns from primal zero-gravity RNEA passes
  confined to one chain; the constant columns written by the first evaluation only) vs
  jac_dual_all + jac_const_every (the base-position columns skip the tree pass in both): <= 1e-13
  relative to max |J|, at two evaluation points of one handle (the second evaluation runs
  without the constant columns);
* Lagrangian Hessian (pairs confined to one chain, the linear-column blocks) vs
  hess_full_tree + hess_dual_all: <= 1e-12 relative to max |H|;
* the factor chain's E_{i+1} on the f64 MFMA (aba, centroidal) vs fchain_list (the list
  route): one SQP step, solver outcome exact and the QP step <= 2e-9 relative.
"""
import numpy as np
import pytest

from conftest import golden, make_robot

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return float(np.abs(np.asarray(a) - np.asarray(b)).max() / max(1e-300, np.abs(np.asarray(b)).max()))


def _handle(name, rname, dyn, N, **kw):
    from pinoloco.ocp import BatchedOCP
    G = golden(f"sqp_{name}.npz")
    gait = str(G["gait"]) if "gait" in G else "trot"
    ib = bool(int(G["include_base"])) if "include_base" in G else True
    ia = bool(int(G["include_acc"])) if "include_acc" in G else True
    R = make_robot(rname, gait)
    bo = BatchedOCP(R, dyn, N, batch=G["P"].shape[0], device=0, gait_type=gait, include_base=ib, include_acc=ia,
                    **kw)
    bo.set_params(G["P"])
    bo.set_x(G["X"])
    bo.init_solver()
    return G, bo


@pytest.mark.parametrize("name,rname,dyn,N", [("b2g_rnea_n50", "b2g", "whole_body_rnea", 50),
                                               ("b2g_acc_n50", "b2g", "whole_body_acc", 50),
                                               ("go2_rnea_fd_n20", "go2", "whole_body_rnea", 20)])
def test_jacobian_rewrites_match_dual_columns(name, rname, dyn, N):
    out = {}
    for tag, paths in (("new", ()), ("old", ("jac_dual_all", "jac_const_every"))):
        G, bo = _handle(name, rname, dyn, N, debug_paths=paths)
        J1 = bo.eval_sqp_data()[1].copy()
        x2 = G["X"] + 1e-3 * np.random.default_rng(5).standard_normal(G["X"].shape)
        bo.set_x(x2)
        J2 = bo.eval_sqp_data()[1].copy()
        bo.close()
        out[tag] = (J1, J2)
    for k in range(2):
        assert _rel(out["new"][k], out["old"][k]) <= 1e-13


@pytest.mark.parametrize("name,rname,dyn,N", [("ip_b2g_rnea_n50", "b2g", "whole_body_rnea", 50),
                                               ("ip_b2g_acc_n50", "b2g", "whole_body_acc", 50),
                                               ("ip_go2_rnea_n20", "go2", "whole_body_rnea", 20)])
def test_hessian_rewrites_match_full_pairs(name, rname, dyn, N):
    from pinoloco.ocp import BatchedOCP
    G = golden(f"{name}.npz")
    gait = str(G["gait"])
    H = {}
    # new: the r06 forward-over-reverse columns (k_lag_hess_col); pairs: the r05 hyper-dual pair
    # sweeps (PL_PATH_HESS_PAIRS); old: every pair in hyper-dual node rows over the whole tree (r04)
    for tag, paths in (("new", ()), ("pairs", ("hess_pairs",)), ("old", ("hess_full_tree", "hess_dual_all"))):
        ib = bool(int(G["include_base"])) if "include_base" in G else True
        R = make_robot(rname, gait)
        bo = BatchedOCP(R, dyn, N, batch=1, device=0, gait_type=gait, include_base=ib, debug_paths=paths)
        assert bo.sizes()["debug_paths"] == sum(__import__("pinoloco")._lib.PATHS[p] for p in paths)
        bo.set_solver("fatrop")
        bo.set_ip_settings()
        bo.set_params(G["P"][:1])
        bo.init_solver()
        bo.ip_direction(G["x_out"][0], G["s"][0], G["lam"][0], G["zl"][0], G["zu"][0], G["mu"][0])
        H[tag] = bo.lag_hess()[0]
        bo.close()
    d = abs(H["new"] - H["old"]).max()
    assert d <= 1e-12 * abs(H["old"]).max()
    assert abs(H["new"] - H["pairs"]).max() <= 1e-13 * abs(H["pairs"]).max()


@pytest.mark.parametrize("name,rname,dyn,N", [("b2_aba_n40", "b2", "whole_body_aba", 40),
                                               ("go2_cv_n20", "go2", "centroidal_vel", 20)])
def test_factor_mfma_coupling_matches_list_route(name, rname, dyn, N):
    res = {}
    for tag, paths in (("new", ()), ("old", ("fchain_list",))):
        G, bo = _handle(name, rname, dyn, N, debug_paths=paths)
        st = bo.solve()
        res[tag] = (bo.get_x().copy(), bo.get_step().copy(), st)
        bo.close()
    xn, dn, sn = res["new"]
    xo, do, so = res["old"]
    for key in ("status", "admm_iters", "ls_accepted", "ls_branch", "ls_trials", "ls_alpha"):
        assert np.array_equal(sn[key], so[key]), key
    # two fp64 routes through the reduced system: each within 1e-9 of the oracle's step on these
    # fixtures (test_gpu.py header), so within 2e-9 of each other
    assert _rel(dn, do) <= 2e-9 and _rel(xn, xo) <= 2e-9
