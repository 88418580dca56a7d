"""Oracle self-consistency: the reference's own known-answer identities
and regression against the committed golden vectors (tests/golden/, parity unpinned).
"""
import numpy as np
import pytest
import scipy.sparse as sp

from conftest import golden, make_robot
from oracle import rbd
from oracle.ocp import OracleOCP

ROBOTS = ("go2", "b2", "b2g")


def _random_state(R, rng):
    q = R.q0.copy()
    q[:3] += rng.normal(0, 0.1, 3)
    qu = rng.normal(size=4)
    q[3:7] = qu / np.linalg.norm(qu)
    q[7:] += rng.normal(0, 0.2, R.nj)
    return q, rng.normal(0, 0.5, R.nv), rng.normal(0, 1.0, R.nv)


@pytest.mark.parametrize("name", ROBOTS)
def test_eom_identity(name):
    """run_mpc.py:201-236: RNEA(q,v,a,f_ext) = M a + nle - sum_k J_lin,k^T f_k (LOCAL_WORLD_ALIGNED)."""
    R = make_robot(name)
    M = rbd.ModelArrays(R.model)
    rng = np.random.default_rng(1)
    frames = list(R.foot_frames) + ([R.ext_force_frame] if R.ext_force_frame is not None else [])
    q, v, a = _random_state(R, rng)
    f = rng.normal(0, 40, 3 * len(frames))
    tau = rbd.rnea_dynamics(M, frames, q, v, a, f)
    Mq = rbd.crba(M, q)
    nle = rbd.rnea(M, q, v, np.zeros(R.nv))
    Jt = sum(rbd.frame_jacobian_lwa(M, q, fid)[:3].T @ f[3 * k:3 * k + 3] for k, fid in enumerate(frames))
    assert np.abs(tau - (Mq @ a + nle - Jt)).max() < 1e-10 * max(1.0, np.abs(tau).max())
    assert np.allclose(Mq, Mq.T, atol=1e-12)
    assert np.all(np.linalg.eigvalsh(Mq) > 0)
    assert Mq[0, 0] == pytest.approx(R.mass, rel=1e-12)  # A_b[0,0] == total mass


@pytest.mark.parametrize("name", ROBOTS)
def test_aba_inverts_rnea(name):
    R = make_robot(name)
    M = rbd.ModelArrays(R.model)
    rng = np.random.default_rng(2)
    frames = list(R.foot_frames)
    q, v, a = _random_state(R, rng)
    a[:6] = 0.0
    f = rng.normal(0, 40, 12)
    tau = rbd.rnea_dynamics(M, frames, q, v, a, f)
    # with the base wrench actually applied (tau[:6] != 0) ABA(q,v,tau,f) == a
    _, oM = rbd.forward_kinematics(M, q)
    acc = rbd.aba(M, q, v, tau, rbd.contact_fext(M, oM, frames, f))
    assert np.abs(acc - a).max() < 1e-9


@pytest.mark.parametrize("name", ROBOTS)
def test_difference_integrate_roundtrip(name):
    R = make_robot(name)
    M = rbd.ModelArrays(R.model)
    rng = np.random.default_rng(3)
    for _ in range(5):
        q, _, _ = _random_state(R, rng)
        dq = rng.normal(0, 0.4, R.nv)
        q1 = rbd.integrate(M, q, dq)
        assert np.linalg.norm(q1[3:7]) == pytest.approx(1.0, abs=1e-12)
        assert np.abs(rbd.difference(M, q, q1) - dq).max() < 1e-10


def test_integrate_small_angle_taylor():
    """exp6 uses its Taylor branch below eps^(1/4); both sides of it agree."""
    R = make_robot("go2")
    M = rbd.ModelArrays(R.model)
    q = R.q0.copy()
    for s in (1e-5, 1.2e-4, 1.3e-4, 1e-3):
        dq = np.zeros(R.nv)
        dq[3:6] = s * np.array([0.3, -0.5, 0.8])
        dq[:3] = 0.1
        assert np.abs(rbd.difference(M, q, rbd.integrate(M, q, dq)) - dq).max() < 1e-12


@pytest.mark.parametrize("name", ROBOTS)
def test_rbd_golden(name):
    """Regression of the restatement against tests/golden/rbd_<robot>.npz."""
    G = golden(f"rbd_{name}.npz")
    R = make_robot(name)
    M = rbd.ModelArrays(R.model)
    frames = list(G["frames"])
    for k in range(len(G["q"])):
        q, v, a, f = G["q"][k], G["v"][k], G["a"][k], G["f"][k]
        np.testing.assert_allclose(rbd.rnea_dynamics(M, frames, q, v, a, f), G["tau"][k], rtol=1e-12, atol=1e-10)
        np.testing.assert_allclose(rbd.crba(M, q), G["M"][k], rtol=1e-12, atol=1e-12)
        np.testing.assert_allclose(rbd.integrate(M, q, G["dq"][k]), G["q_int"][k], rtol=1e-13, atol=1e-14)


@pytest.mark.parametrize("name,rname,dyn,N,n,m", [
    ("go2_rnea_n20", "go2", "whole_body_rnea", 20, 1392, 2032),
    ("b2_aba_n40", "b2", "whole_body_aba", 40, 2436, 3680),
    ("b2g_acc_n50", "b2g", "whole_body_acc", 50, 4398, 6397),
    ("b2g_rnea_n50", "b2g", "whole_body_rnea", 50, 4452, 6505),
])
def test_ocp_sizes_and_golden_eval(name, rname, dyn, N, n, m):
    """SURVEY 8 size table, and g / grad / J_g against the golden vectors."""
    G = golden(f"sqp_{name}.npz")
    R = make_robot(rname)
    o = OracleOCP(R, dyn, N)
    x, p = G["X"][0], G["P"][0]
    g, lbg, ubg = o.eval_g(x, p)
    assert (o.n, len(g)) == (n, m)
    np.testing.assert_allclose(g, G["g"][0], rtol=1e-12, atol=1e-10)
    assert np.array_equal(lbg, G["lbg"][0]) and np.array_equal(ubg, G["ubg"][0])
    f, grad = o.f_and_grad(x, p)
    np.testing.assert_allclose(grad, G["grad"][0], rtol=1e-13, atol=1e-12)
    assert f == pytest.approx(float(G["f"][0]), rel=1e-13)
    if rname == "go2":
        J = o.eval_J(x, p).tocsr()
        Jg = sp.csr_matrix((G["J_data_0"], G["J_indices_0"], G["J_indptr_0"]), shape=J.shape)
        assert abs(J - Jg).max() < 1e-10


def test_complex_step_matches_finite_difference():
    R = make_robot("go2")
    o = OracleOCP(R, "whole_body_rnea", 6)
    G = golden("sqp_go2_rnea_n20.npz")
    from pinoloco.synthetic import build_batch
    lay, P, X, _, _ = build_batch(R, "whole_body_rnea", 6, 1, 0)
    x, p = X[0] + np.random.default_rng(0).normal(0, 0.01, o.n), P[0]
    J = o.eval_J(x, p).toarray()
    rng = np.random.default_rng(1)
    d = rng.normal(size=o.n)
    h = 1e-6
    fd = (o.eval_g(x + h * d, p)[0] - o.eval_g(x - h * d, p)[0]) / (2 * h)
    assert np.abs(J @ d - fd).max() < 1e-5 * max(1.0, np.abs(fd).max())
    assert G["P"].shape[1] == 318  # np of config 2


@pytest.mark.slow
def test_sqp_step_golden_go2():
    """One SQP iteration (ocp.py:375-414) reproduces the committed QP step and line search."""
    G = golden("sqp_go2_rnea_n20.npz")
    R = make_robot("go2")
    o = OracleOCP(R, "whole_body_rnea", 20)
    x, p = G["X"][0], G["P"][0]
    o.init_solver(x, p)
    x_new, dx, st = o.sqp_step(x, p)
    assert st["status"] == G["status"][0] and st["iter"] == G["iters"][0]
    assert st["branch"] == G["branch"][0] and st["alpha"] == G["alpha"][0]
    assert np.abs(dx - G["dx"][0]).max() <= 1e-9 * np.abs(G["dx"][0]).max()


def test_osqp_restatement_kkt():
    """OSQP restatement: with a tiny problem run to convergence the returned point
    satisfies the KKT conditions within eps."""
    from oracle.osqp_ref import OSQPRef, REFERENCE_SETTINGS
    rng = np.random.default_rng(5)
    n, m = 12, 18
    A = sp.random(m, n, density=0.4, random_state=1, format="csc") + sp.eye(m, n, format="csc")
    Pd = rng.uniform(0.5, 2.0, n)
    q = rng.normal(size=n)
    l = -rng.uniform(0.1, 1.0, m)
    u = rng.uniform(0.1, 1.0, m)
    l[:3] = u[:3] = 0.2  # equality rows use rho * 1e3
    s = dict(REFERENCE_SETTINGS)
    s.update(max_iter=4000, eps_abs=1e-7, eps_rel=1e-7)
    solver = OSQPRef(Pd, A, s)
    x, info = solver.update_and_solve(q, A.data.copy(), l, u)
    assert info["status"] == 1
    Ax = A @ x
    assert np.all(Ax >= l - 1e-5) and np.all(Ax <= u + 1e-5)
    D, E, c = solver.scaling
    y = E * solver.y / c  # unscaled duals (OSQP unscale_solution)
    assert np.abs(Pd * x + q + A.T @ y).max() < 1e-4
    # complementarity: y < 0 only at the lower bound, y > 0 only at the upper bound
    assert np.all((y > 1e-6) <= (np.abs(Ax - u) < 1e-4)) and np.all((y < -1e-6) <= (np.abs(Ax - l) < 1e-4))


@pytest.mark.parametrize("name,rname,dyn,N", [("go2_rnea_n20_walk", "go2", "whole_body_rnea", 20),
                                             ("go2_cv_n20", "go2", "centroidal_vel", 20)])
def test_rho_classification_independent_of_scaling_step(name, rname, dyn, N):
    """The reference calls osqp_prob.update(q=, Ax=, l=, u=) (ocp.py:395); OSQP 0.6's
    wrapper applies update_bounds before update_A, so it classifies the rows (equality
    when the scaled width u-l < RHO_TOL) with the previous step's E, while the device and
    the oracle use the current E.  For this problem family both give the same classes:
    equality rows have width 0, and every finite two-sided row is so wide that the
    scaled width clears RHO_TOL by orders of magnitude under either E."""
    from oracle.osqp_ref import RHO_TOL
    G = golden(f"sqp_{name}.npz")
    gait = str(G["gait"]) if "gait" in G else "trot"
    R = make_robot(rname, gait)
    o = OracleOCP(R, dyn, N)
    p = G["P"][0]
    o.init_solver(G["X"][0], p)
    Es = []
    for x in (G["X"][0], G["x_new"][0]):  # this step's and the next step's linearisation
        Ax = o.jacobian_values(x, p)
        A = sp.csc_matrix((Ax, o.pattern.indices, o.pattern.indptr), shape=o.pattern.shape)
        Es.append(o.osqp._scale(o.hess_diag, o.f_and_grad(x, p)[1], A)[4])
    _, lbg, ubg = o.eval_g(G["x_new"][0], p)
    w = ubg - lbg
    two = np.isfinite(w) & (w > 0)
    assert np.array_equal(w * Es[0] < RHO_TOL, w * Es[1] < RHO_TOL)
    margin = min((w[two] * E[two]).min() for E in Es) / RHO_TOL
    print(f"{name}: narrowest scaled two-sided row = {margin:.3g} x RHO_TOL")
    assert margin > 10.0


def test_centroidal_vel_without_base_momentum_identity():
    """centroidal_vel with include_base=False (ocp_centroidal_vel.py:119-129): the rows use
    v = [base_vel_dynamics(h, q, v_j), v_j], which reproduces the momentum A(q) v = m h, so
    the include_base form's gap rows vanish there; no gap rows, u = [v_j | f]; the fixture
    evaluates (g, grad, f) the same way."""
    R = make_robot("go2")
    o = OracleOCP(R, "centroidal_vel", 20, include_base=False)
    ob = OracleOCP(R, "centroidal_vel", 20, include_base=True)
    assert o.nu[0] == R.nj + R.nf and ob.nu[0] == R.nv + R.nf
    G = golden("sqp_go2_cv_nb_n20.npz")
    x, p = G["X"][1], G["P"][1]
    g, lbg, ubg = o.eval_g(x, p)
    np.testing.assert_allclose(g, G["g"][1], rtol=1e-12, atol=1e-10)
    P = o.unpack(p)
    DX, U = o.split(x)
    rng = np.random.default_rng(3)
    for i in (0, 7):
        dx = DX[i] + rng.normal(0, 0.05, o.ndx)
        h, q = o.state(dx, P)
        v_j = U[i][:R.nj] + rng.normal(0, 0.3, R.nj)
        v = np.concatenate([rbd.base_vel_cv(o.M, h, q, v_j, o.mass), v_j])
        hg = rbd.centroidal_momentum(o.M, q, v)
        np.testing.assert_allclose(hg, o.mass * h, rtol=1e-12, atol=1e-12)
        rows_nb = sum(r[0].shape[-1] for r in o.node_rows(i, dx, U[i], DX[i + 1], P))
        ub = np.concatenate([v, U[i][R.nj:]])
        rows_b = ob.node_rows(i, dx, ub, DX[i + 1], P)
        assert rows_nb == sum(r[0].shape[-1] for r in rows_b) - 6
        # the include_base form's gap row block (after the 6 + nv dynamics rows) is 0 at this v
        gap = rows_b[2][0]
        assert gap.shape[-1] == 6
        assert np.abs(gap).max() < 1e-10 * max(1.0, o.mass * np.abs(h).max())
