"""Dynamics plugin surface (pinoloco/dynamics.py over pl_dyn_eval) against the oracle's
golden vectors (tests/golden/rbd_<robot>.npz, parity unpinned) and the reference's
own identities:

* every factory of dynamics/*.py: rnea / aba / frame position / frame velocity
  (incl. base-relative) / whole-body-acc gaps and base acceleration / centroidal
  com_dynamics, base_vel, base_acc (pinocchio dccrba), gaps; the state maps;
* the debug identity of run_mpc.py:201-236 evaluated through the callables:
  tau_rnea = M a + nle - sum_k J_lin,k^T f_k;
* A_b[0, 0] = m and the OCS2 closed-form A_b^-1 at identity base orientation
  (dynamics_centroidal_vel.py:150-159).

The CPU tests use a host handle (device = -1, the library's host build of the same
code); the -m gpu tests run the same checks with one GPU thread per point.
Tolerance: 1e-12 relative to the largest magnitude of each output (1e-10 for the
difference-based crba / frame Jacobian / base accelerations).
"""
import numpy as np
import pytest

from conftest import golden, make_robot

ROBOTS = ("go2", "b2", "b2g")


def _close(got, want, tol=1e-12):
    got, want = np.asarray(got), np.asarray(want)
    assert got.shape == want.shape, (got.shape, want.shape)
    assert np.abs(got - want).max() <= tol * max(1.0, np.abs(want).max())


def check_surface(name, device):
    from pinoloco.dynamics import DynamicsCentroidalVel, DynamicsWholeBodyAcc, DynamicsWholeBodyTorque
    G = golden(f"rbd_{name}.npz")
    R = make_robot(name)
    ext = R.ext_force_frame
    wb = DynamicsWholeBodyTorque(R, device=device)
    acc = DynamicsWholeBodyAcc(R, device=device)
    cv = DynamicsCentroidalVel(R, device=device)
    q, v, a, f = G["q"], G["v"], G["a"], G["f"]  # batches of 3 points
    _close(wb.rnea_dynamics(ext)(q, v, a, f), G["tau"])
    _close(wb.aba_dynamics(ext)(q, v, G["tau"][:, 6:], f), G["aba"], 1e-10)
    _close(wb.crba()(q), G["M"], 1e-10)
    _close(wb.nonlinear_effects()(q, v), G["nle"])
    _close(wb.center_of_mass()(q), G["com"])
    _close(wb.centroidal_map()(q), G["cmap"])
    _close(wb.frame_jacobian(R.foot_frames[0])(q), G["foot_jac0"], 1e-10)
    for k, fid in enumerate(R.foot_frames):
        _close(wb.get_frame_position(fid)(q), G["foot_pos"][:, 3 * k:3 * k + 3])
        _close(wb.get_frame_velocity(fid)(q, v), G["foot_vel"][:, 6 * k:6 * k + 6])
    if R.arm_ee_frame is not None:
        _close(wb.get_frame_velocity(R.arm_ee_frame, relative_to_base=True)(q, v), G["arm_vel_rel"])
    _close(acc.dynamics_gaps(ext)(q, v, a, f), G["gaps_wb"])
    _close(acc.base_acc_dynamics(ext)(q, v, G["a_j"], f), G["base_acc_wb"], 1e-10)
    _close(cv.com_dynamics(ext)(q, f), G["com_dyn"])
    _close(cv.dynamics_gaps()(G["h"], q, v), G["gaps_cv"])
    _close(cv.base_vel_dynamics()(G["h"], q, G["v_j"]), G["base_vel_cv"], 1e-10)
    _close(cv.base_acc_dynamics(ext)(q, v, G["a_j"], f), G["base_acc_cv"], 1e-10)
    # DynamicsCentroidalAcc (dynamics_centroidal_acc.py): its base_acc equals the centroidal_vel
    # one; the gap A a + dA v - dh against the oracle (computeCentroidalMap + dccrba restated)
    from oracle import rbd as orbd
    from pinoloco.dynamics import DynamicsCentroidalAcc
    ca = DynamicsCentroidalAcc(R, device=device)
    Mo = orbd.ModelArrays(R.model)
    fr = list(G["frames"])
    want = np.stack([orbd.centroidal_map(Mo, q[b]) @ a[b] + orbd.dccrba_v(Mo, q[b], v[b])
                     - orbd.com_dynamics(Mo, fr, q[b], f[b], R.mass, scale=False) for b in range(len(q))])
    _close(ca.dynamics_gaps(ext)(q, v, a, f), want, 1e-10)
    _close(ca.base_acc_dynamics(ext)(q, v, G["a_j"], f), G["base_acc_cv"], 1e-10)
    # single points give 1-D results; state maps round-trip
    x = np.concatenate([q[0], v[0]])
    dx = np.concatenate([G["dq"][0], v[1]])
    _close(wb.state_integrate()(x, dx)[:R.nq], G["q_int"][0], 1e-13)
    _close(wb.state_difference()(x, wb.state_integrate()(x, dx)), dx, 1e-10)
    xc = np.concatenate([G["h"][0], q[0]])
    dxc = np.concatenate([G["h"][1], G["dq"][0]])
    xn = cv.state_integrate()(xc, dxc)
    _close(xn[6:], G["q_int"][0], 1e-13)
    _close(cv.state_difference()(xc, xn), dxc, 1e-10)
    # run_mpc.py:201-236: RNEA(q, v, a, f_ext) == M a + nle - sum J_lin^T f through the callables
    frames = list(G["frames"])
    for b in range(len(q)):
        Mq = wb.crba()(q[b])
        nle = wb.nonlinear_effects()(q[b], v[b])
        Jt = sum(wb.frame_jacobian(fid)(q[b])[:3].T @ f[b][3 * k:3 * k + 3] for k, fid in enumerate(frames))
        tau = wb.rnea_dynamics(ext)(q[b], v[b], a[b], f[b])
        _close(tau, Mq @ a[b] + nle - Jt, 1e-10)


@pytest.mark.parametrize("name", ROBOTS)
def test_dynamics_surface_host(name):
    check_surface(name, device=-1)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ROBOTS)
def test_dynamics_surface_gpu(name):
    check_surface(name, device=0)


@pytest.mark.gpu
def test_dynamics_batched_gpu_matches_host():
    """A batch of 4096 points on the GPU equals the host evaluation point by point."""
    from pinoloco.dynamics import DynamicsCentroidalVel, DynamicsWholeBodyTorque
    R = make_robot("b2g")
    rng = np.random.default_rng(3)
    B = 4096
    q = np.tile(R.q0, (B, 1))
    q[:, 7:] += rng.normal(0, 0.2, (B, R.nj))
    v, a = rng.normal(0, 0.5, (B, R.nv)), rng.normal(0, 1.0, (B, R.nv))
    f = rng.normal(0, 50, (B, R.nf))
    for cls, meth, args in ((DynamicsWholeBodyTorque, "rnea_dynamics", (q, v, a, f)),
                            (DynamicsWholeBodyTorque, "aba_dynamics", (q, v, a[:, 6:], f)),
                            (DynamicsCentroidalVel, "base_acc_dynamics", (q, v, a[:, 6:], f))):
        g = getattr(cls(R, device=0), meth)(R.ext_force_frame)(*args)
        h = getattr(cls(R, device=-1), meth)(R.ext_force_frame)(*args)
        assert g.shape[0] == B
        _close(g, h, 1e-13)


def test_centroidal_base_block_identities():
    """A_b[0, 0] = m and A_b^-1 = the OCS2 closed form (dynamics_centroidal_vel.py:150-159)
    when the base frame is world-aligned.  (With pinocchio's local base velocity,
    A_b[:3, :3] = m R_base, so both hold only at identity base orientation.)"""
    from oracle import rbd
    from pinoloco.dynamics import Dynamics
    for name in ROBOTS:
        R = make_robot(name)
        q = R.q0.copy()
        q[:3] += 0.3
        q[7:] += np.random.default_rng(1).normal(0, 0.2, R.nj)
        A = Dynamics(R).centroidal_map()(q)
        assert A[0, 0] == pytest.approx(R.mass, rel=1e-13)
        _close(np.linalg.inv(A[:, :6]), rbd.ab_inv_ocs2(A[:, :6]), 1e-12)
        _close(A, rbd.centroidal_map(rbd.ModelArrays(R.model), q))


def test_point_function_errors():
    from pinoloco import _lib
    from pinoloco.dynamics import Dynamics, DynamicsWholeBodyTorque
    R = make_robot("go2")
    with pytest.raises(ValueError):
        DynamicsWholeBodyTorque(R).rnea_dynamics()(R.q0, np.zeros(R.nv))
    with pytest.raises(_lib.PinolocoError):  # Go2 has no external-force frame
        Dynamics(R).rnea_dynamics(ext_force_frame=999)
    with pytest.raises(_lib.PinolocoError):  # no base_link frame on Go2 (root link "base")
        Dynamics(R).get_frame_velocity(R.foot_frames[0], relative_to_base=True)(R.q0, np.zeros(R.nv))
