"""CasADi external-function ABI (include/pinoloco_casadi.h) without a GPU: exported
symbols, n_in/n_out/work, compressed-column sparsity of every input/output, and
retract_solution (host computation) against the oracle's state integrate."""
import os
import re

import numpy as np
import pytest

from conftest import make_robot

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    txt = open(os.path.join(ROOT, "include", "pinoloco_casadi.h")).read()
    names = re.findall(r"^PL_CASADI_DECLARE\((\w+)\)", txt, re.M)
    suffixes = re.findall(r"NAME##_(\w+)\(", txt)
    return names, suffixes


def test_casadi_symbols_exported():
    from pinoloco import _lib, casadi_ext
    names, suffixes = _declared()
    assert tuple(names) == casadi_ext.FUNCTIONS
    L = _lib.lib()
    for n in names:
        getattr(L, n)
        for s in suffixes:
            getattr(L, f"{n}_{s}")


def test_unbound_is_an_error():
    from pinoloco import _lib, casadi_ext
    casadi_ext.unbind()
    with pytest.raises(_lib.PinolocoError):
        casadi_ext.ExternalFunction("sqp_data")


@pytest.mark.parametrize("rname,dyn,N", [("go2", "whole_body_rnea", 10), ("b2g", "whole_body_rnea", 8)])
def test_shapes_and_sparsity(rname, dyn, N):
    from pinoloco import casadi_ext
    from pinoloco.ocp import BatchedOCP
    R = make_robot(rname)
    bo = BatchedOCP(R, dyn, N, batch=1, device=-1)
    casadi_ext.bind(bo, 3)
    f = casadi_ext.ExternalFunction("sqp_data")
    assert (f.n_in, f.n_out, f.sz_arg, f.sz_res, f.sz_iw, f.sz_w) == (2, 5, 2, 5, 0, 0)
    assert f.sp_in[0][:2] == (bo.n, 1) and f.sp_in[1][:2] == (bo.np, 1)
    nrow, ncol, colind, row = f.sp_out[1]
    assert (nrow, ncol) == (bo.m, bo.n) and int(colind[-1]) <= bo.nnz
    assert np.all(np.diff(colind) >= 0)
    for j in range(ncol):  # rows strictly increasing inside each column
        assert np.all(np.diff(row[colind[j]:colind[j + 1]]) > 0)
    # the structural-dependency pattern (generic-point probe): inside the library's
    # kinematic-dependency pattern, strictly smaller for whole-body RNEA (the base position
    # columns RNEA never reads)
    rows, cols = bo.pattern()
    got = set(zip(row.tolist(), np.repeat(np.arange(ncol), np.diff(colind)).tolist()))
    lib = set(zip(rows.tolist(), cols.tolist()))
    assert got < lib
    assert int(colind[-1]) == len(got)
    assert [s[:2] for s in f.sp_out[2:]] == [(bo.m, 1)] * 3
    h = casadi_ext.ExternalFunction("hess_data")
    assert h.sp_out[0][:2] == (bo.n, bo.n) and int(h.sp_out[0][2][-1]) == bo.n
    fd = casadi_ext.ExternalFunction("f_data")
    assert fd.sp_out[0][:2] == (1, 1) and fd.sp_out[1][:2] == (bo.n, 1)
    casadi_ext.unbind()
    bo.close()


@pytest.mark.parametrize("name,rname,dyn,N", [("go2_rnea_n20", "go2", "whole_body_rnea", 20),
                                              ("go2_cv_n20", "go2", "centroidal_vel", 20),
                                              ("b2_aba_n40", "b2", "whole_body_aba", 40),
                                              ("b2g_acc_n50", "b2g", "whole_body_acc", 50),
                                              ("b2g_rnea_n50", "b2g", "whole_body_rnea", 50),
                                              ("go2_cv_nb_n20", "go2", "centroidal_vel", 20),
                                              ("go2_rnea_fd_n20", "go2", "whole_body_rnea", 20)])
def test_jg_pattern_covers_the_oracle_jacobian(name, rname, dyn, N):
    """The reference sets OSQP's A up from J_g.sparsity() and feeds J_g.nonzeros()
    (optimization/ocp.py:305-306, 391): every entry of the oracle's complex-step Jacobian at
    the fixture point above round-off (1e-13 of the largest) lies inside the exported J_g
    pattern, so the pattern loses nothing the solve needs."""
    import scipy.sparse as sps
    from conftest import golden
    from pinoloco import casadi_ext
    from pinoloco.ocp import BatchedOCP
    G = golden(f"sqp_{name}.npz")
    kw = {k: bool(int(G[k])) for k in ("include_base", "include_acc") if k in G}
    R = make_robot(rname)
    bo = BatchedOCP(R, dyn, N, batch=1, device=-1, **kw)
    casadi_ext.bind(bo, 3)
    nrow, ncol, colind, row = casadi_ext.ExternalFunction("sqp_data").sp_out[1]
    pat = sps.csc_matrix((np.ones(int(colind[-1])), row, colind), shape=(nrow, ncol))
    J = sps.csr_matrix((G["J_data_0"], G["J_indices_0"], G["J_indptr_0"]), shape=(nrow, ncol)).tocoo()
    # complex-step round-off where the derivative vanishes identically (|J| ~ 1e-17) is no entry
    nz = np.abs(J.data) > 1e-13 * np.abs(J.data).max()
    assert np.all(np.asarray(pat.tocsr()[J.row[nz], J.col[nz]]).ravel() == 1)
    casadi_ext.unbind()
    bo.close()


@pytest.mark.parametrize("include_acc", [True, False])
def test_retract_solution_matches_oracle(include_acc):
    """retract_solution (ocp_whole_body_rnea.py:326-366): node-major rows of q, v, a,
    forces, tau over the first 3 nodes, q/v by the Lie-group integrate; with
    include_acc=False a is u_sol[:0] (no columns)."""
    from oracle.ocp import OracleOCP
    from pinoloco import casadi_ext
    from pinoloco.ocp import BatchedOCP
    R = make_robot("b2g")
    N = 8
    bo = BatchedOCP(R, "whole_body_rnea", N, batch=1, device=-1, include_acc=include_acc)
    casadi_ext.bind(bo, 3)
    fr = casadi_ext.ExternalFunction("retract_solution")
    rng = np.random.default_rng(3)
    sol = rng.normal(size=bo.n) * 0.1
    x_init = np.concatenate([R.q0, rng.normal(size=R.nv) * 0.1])
    q, v, a, f, tau = fr(sol, x_init)
    o = OracleOCP(R, "whole_body_rnea", N, include_acc=include_acc)
    DX, U = o.split(sol)
    assert q.shape == (3, R.nq) and v.shape == (3, R.nv) and a.shape == (3, o.na)
    for i in range(3):
        xs = o.integrate_state(x_init, DX[i])
        assert np.abs(q[i] - xs[:R.nq]).max() < 1e-12
        assert np.abs(v[i] - xs[R.nq:]).max() < 1e-12
        assert np.array_equal(a[i], U[i][:o.na])
        assert np.array_equal(f[i], U[i][o.na:o.na + o.nf])
        assert np.array_equal(tau[i], U[i][o.na + o.nf:])
    with pytest.raises(Exception):
        casadi_ext.ExternalFunction("sqp_data")(sol, np.zeros(bo.np))  # no device on this handle
    casadi_ext.unbind()
    bo.close()


def test_destroy_unbinds():
    """Closing a bound OCP clears the process-global binding: a later call reports
    'no OCP bound' instead of touching freed memory (pl_ocp_destroy -> cas_forget)."""
    from pinoloco import _lib, casadi_ext
    from pinoloco.ocp import BatchedOCP
    R = make_robot("go2")
    bo = BatchedOCP(R, "whole_body_rnea", 6, batch=1, device=-1)
    casadi_ext.bind(bo, 2)
    fr = casadi_ext.ExternalFunction("retract_solution")
    n, nx = bo.n, R.nq + R.nv
    bo.close()
    with pytest.raises(_lib.PinolocoError, match="no OCP bound"):
        fr(np.zeros(n), np.zeros(nx))


@pytest.mark.parametrize("dyn", ["whole_body_aba", "whole_body_acc"])
def test_retract_solution_dynamics_outputs(dyn):
    """retract_solution fills a (ABA, ocp_whole_body_aba.py:239) and tau (RNEA joint rows,
    ocp_whole_body_acc.py:262) from the library's point functions, against the oracle."""
    from oracle import rbd
    from oracle.ocp import OracleOCP
    from pinoloco import casadi_ext
    from pinoloco.ocp import BatchedOCP
    R = make_robot("b2g")
    N = 6
    bo = BatchedOCP(R, dyn, N, batch=1, device=-1)
    casadi_ext.bind(bo, 3)
    rng = np.random.default_rng(5)
    o = OracleOCP(R, dyn, N)
    sol = rng.normal(size=bo.n) * 0.1
    x_init = np.concatenate([R.q0, rng.normal(size=R.nv) * 0.1])
    q, v, a, f, tau = casadi_ext.ExternalFunction("retract_solution")(sol, x_init)
    M = rbd.ModelArrays(R.model)
    frames = list(R.foot_frames) + [R.ext_force_frame]
    DX, U = o.split(sol)
    assert a.shape == (3, R.nv) and tau.shape == (3, R.nj)
    for i in range(3):
        xs = o.integrate_state(x_init, DX[i])
        qi, vi = xs[:R.nq], xs[R.nq:]
        if dyn == "whole_body_aba":
            want_a = rbd.aba_dynamics(M, frames, qi, vi, U[i][:R.nj], U[i][R.nj:])
            assert np.abs(a[i] - want_a).max() < 1e-10 * max(1, np.abs(want_a).max())
            assert np.array_equal(tau[i], U[i][:R.nj])
        else:
            assert np.array_equal(a[i], U[i][:R.nv])
            want_t = rbd.rnea_dynamics(M, frames, qi, vi, U[i][:R.nv], U[i][R.nv:])[6:]
            assert np.abs(tau[i] - want_t).max() < 1e-12 * max(1, np.abs(want_t).max())
    casadi_ext.unbind()
    bo.close()


@pytest.mark.gpu
def test_retract_solution_centroidal_vel_without_base():
    """retract_solution of centroidal_vel with include_base=False (ocp_centroidal_vel.py:
    284-318): v = [base_vel_dynamics(h, q, v_j), v_j], the next node's v_b at this node's
    h, q, a = [base_acc_dynamics(q, v, a_j, f), a_j] with the finite-difference a_j, and
    tau the RNEA joint rows; against the oracle."""
    from oracle import rbd
    from oracle.ocp import OracleOCP
    from pinoloco import casadi_ext
    from pinoloco.gait import horizon_dts
    from pinoloco.ocp import BatchedOCP
    from pinoloco.synthetic import DT_MAX, DT_MIN, build_batch
    R = make_robot("go2")
    N = 6
    _, P, _, _, _ = build_batch(R, "centroidal_vel", N, 1, 0, include_base=False)
    bo = BatchedOCP(R, "centroidal_vel", N, batch=1, device=0, include_base=False)
    bo.set_params(P)  # the step sizes of the finite-difference accelerations
    casadi_ext.bind(bo, 3)
    o = OracleOCP(R, "centroidal_vel", N, include_base=False)
    rng = np.random.default_rng(6)
    sol = rng.normal(size=bo.n) * 0.1
    x_init = np.concatenate([rng.normal(size=6) * 0.2, R.q0])
    q, v, a, f, tau = casadi_ext.ExternalFunction("retract_solution")(sol, x_init)
    M = rbd.ModelArrays(R.model)
    frames = list(R.foot_frames)
    dts = horizon_dts(DT_MIN, DT_MAX, N)
    DX, U = o.split(sol)
    nj = R.nj
    for i in range(3):
        xs = o.integrate_state(x_init, DX[i])
        h, qi = xs[:6], xs[6:]
        vi = np.concatenate([rbd.base_vel_cv(M, h, qi, U[i][:nj], R.mass), U[i][:nj]])
        vn = np.concatenate([rbd.base_vel_cv(M, h, qi, U[i + 1][:nj], R.mass), U[i + 1][:nj]])
        a_j = (vn - vi)[6:] / dts[i]
        want_a = np.concatenate([rbd.base_acc_cv(M, frames, qi, vi, a_j, U[i][nj:], R.mass), a_j])
        want_t = rbd.rnea_dynamics(M, frames, qi, vi, want_a, U[i][nj:])[6:]
        assert np.abs(q[i] - qi).max() < 1e-13
        assert np.abs(v[i] - vi).max() < 1e-11 * max(1, np.abs(vi).max())
        assert np.abs(a[i] - want_a).max() < 1e-9 * max(1, np.abs(want_a).max())
        assert np.array_equal(f[i], U[i][nj:])
        assert np.abs(tau[i] - want_t).max() < 1e-9 * max(1, np.abs(want_t).max())
    casadi_ext.unbind()
    bo.close()
