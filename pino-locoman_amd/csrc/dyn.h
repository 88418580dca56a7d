// Point functions of the reference's Dynamics plugin surface (host+device, fp64).
//
// Each function evaluates one sample of a factory the reference builds with
// pinocchio.casadi (dynamics/*.py) and returns as a ca.Function:
//   rnea_dynamics(ext)(q, v, a, forces) -> tau        dynamics/dynamics.py:33-65
//   aba_dynamics(ext)(q, v, tau_j, forces) -> a        dynamics_whole_body_torque.py:73-103
//   get_frame_position(f)(q) -> pos                    dynamics/dynamics.py:67-75
//   get_frame_velocity(f, relative_to_base)(q, v)      dynamics/dynamics.py:77-118
//   dynamics_gaps(ext)(q, v, a, forces) -> gaps        dynamics_whole_body_acc.py:85-126
//   base_acc_dynamics(ext)(q, v, a_j, forces) -> a_b   dynamics_whole_body_acc.py:43-83
//   com_dynamics(ext)(q, forces) -> h_dot              dynamics_centroidal_vel.py:43-71
//   base_vel_dynamics()(h, q, v_j) -> v_b              dynamics_centroidal_vel.py:73-89
//   base_acc_dynamics(ext)(q, v, a_j, forces) -> a_b   dynamics_centroidal_vel.py:91-134
//   dynamics_gaps()(h, q, v) -> A(q) v - m h           dynamics_centroidal_vel.py:136-148
// plus the pinocchio terms the reference's debug identity uses (crba,
// nonLinearEffects, computeFrameJacobian LOCAL_WORLD_ALIGNED; run_mpc.py:201-236),
// computeCentroidalMap and centerOfMass.  Built on the same tree passes as the OCP
// rows (rbd.h); the kernels in k_dyn.hip run one sample per thread.
#pragma once
#include "../../include/pinoloco.h"
#include "rows.h"

namespace pl {

// Function codes: PL_FN_* of include/pinoloco.h (the ABI numbers them).
#define PL_FN_COUNT 20

// Output length of one sample.
PL_HD int dyn_out_len(const PlModel& M, int fn) {
  const int nq = M.nq, nv = M.nv;
  switch (fn) {
    case PL_FN_RNEA: case PL_FN_ABA: case PL_FN_NLE: return nv;
    case PL_FN_FRAME_POS: case PL_FN_COM: return 3;
    case PL_FN_CRBA: return nv * nv;
    case PL_FN_FRAME_JAC: case PL_FN_CMAP: return 6 * nv;
    case PL_FN_INTEGRATE_WB: return nq + nv;
    case PL_FN_DIFFERENCE_WB: return 2 * nv;
    case PL_FN_INTEGRATE_CV: return 6 + nq;
    case PL_FN_DIFFERENCE_CV: return 6 + nv;
    default: return 6;
  }
}

// Input lengths of one sample (up to four inputs); ext = external-force frame in use.
PL_HD void dyn_in_len(const PlModel& M, int fn, int nf, int* len) {
  const int nq = M.nq, nv = M.nv, nj = nq - 7;
  for (int k = 0; k < 4; ++k) len[k] = 0;
  switch (fn) {
    case PL_FN_RNEA: case PL_FN_GAPS_WB: case PL_FN_GAPS_CA: len[0] = nq; len[1] = nv; len[2] = nv; len[3] = nf; break;
    case PL_FN_ABA: case PL_FN_BASE_ACC_WB: case PL_FN_BASE_ACC_CV:
      len[0] = nq; len[1] = nv; len[2] = nj; len[3] = nf; break;
    case PL_FN_FRAME_POS: case PL_FN_CRBA: case PL_FN_FRAME_JAC: case PL_FN_CMAP: case PL_FN_COM: len[0] = nq; break;
    case PL_FN_FRAME_VEL: case PL_FN_NLE: len[0] = nq; len[1] = nv; break;
    case PL_FN_COM_DYN: len[0] = nq; len[1] = nf; break;
    case PL_FN_BASE_VEL_CV: len[0] = 6; len[1] = nq; len[2] = nj; break;
    case PL_FN_GAPS_CV: len[0] = 6; len[1] = nq; len[2] = nv; break;
    case PL_FN_INTEGRATE_WB: len[0] = nq + nv; len[1] = 2 * nv; break;
    case PL_FN_DIFFERENCE_WB: len[0] = nq + nv; len[1] = nq + nv; break;
    case PL_FN_INTEGRATE_CV: len[0] = 6 + nq; len[1] = 6 + nv; break;
    case PL_FN_DIFFERENCE_CV: len[0] = 6 + nq; len[1] = 6 + nq; break;
    default: break;
  }
}

// World placements (and local velocities when v != nullptr) of every joint frame.
struct FkAll {
  double oR[PL_MAXJ][9];
  double op[PL_MAXJ][3];
  double vl[PL_MAXJ][6];
};
PL_HD void fk_all(const PlModel& M, const double* q, const double* v, FkAll& K) {
  for (int j = 1; j < M.njoints; ++j) {
    const int par = M.parent[j];
    double lR[9], lp[3], vJ[6];
    if (M.jtype[j] == PL_JT_FREEFLYER) {
      quat_to_R(q + M.idx_q[j] + 3, lR);
      for (int k = 0; k < 3; ++k) lp[k] = q[M.idx_q[j] + k];
      for (int k = 0; k < 6; ++k) vJ[k] = v ? v[M.idx_v[j] + k] : 0.0;
    } else {
      double s, c;
      sincos_s(q[M.idx_q[j]], &s, &c);
      rev_rot(M, j, s, c, lR);
      for (int k = 0; k < 3; ++k) lp[k] = M.jp[j][k];
      const double qd = v ? v[M.idx_v[j]] : 0.0;
      for (int k = 0; k < 3; ++k) { vJ[k] = 0.0; vJ[3 + k] = M.axis[j][k] * qd; }
    }
    if (par == 0) {
      for (int k = 0; k < 9; ++k) K.oR[j][k] = lR[k];
      for (int k = 0; k < 3; ++k) K.op[j][k] = lp[k];
      for (int k = 0; k < 6; ++k) K.vl[j][k] = vJ[k];
    } else {
      matmul3(K.oR[par], lR, K.oR[j]);
      double t[3];
      matvec(K.oR[par], lp, t);
      for (int k = 0; k < 3; ++k) K.op[j][k] = K.op[par][k] + t[k];
      act_inv_motion(lR, lp, K.vl[par], K.vl[j]);
      for (int k = 0; k < 6; ++k) K.vl[j][k] += vJ[k];
    }
  }
}

// oMf (rotation, translation) of frame F.
PL_HD void frame_placement(const FkAll& K, const PlFrameRef& F, double* R, double* p) {
  matmul3(K.oR[F.joint], F.R, R);
  double t[3];
  matvec(K.oR[F.joint], F.p, t);
  for (int k = 0; k < 3; ++k) p[k] = K.op[F.joint][k] + t[k];
}

// getFrameVelocity(LOCAL_WORLD_ALIGNED): [R_j (v + w x p_f); R_j w]
PL_HD void frame_vel_lwa(const FkAll& K, const PlFrameRef& F, double* out) {
  const double* vj = K.vl[F.joint];
  double wxp[3];
  cross3(vj + 3, F.p, wxp);
  double lv[3] = {vj[0] + wxp[0], vj[1] + wxp[1], vj[2] + wxp[2]};
  matvec(K.oR[F.joint], lv, out);
  matvec(K.oR[F.joint], vj + 3, out + 3);
}

// Dynamics.get_frame_velocity(frame, relative_to_base) (dynamics/dynamics.py:77-118).
PL_HD void frame_velocity(const FkAll& K, const PlFrameRef& F, const PlFrameRef& base, bool rel, double* out) {
  double fv[6];
  frame_vel_lwa(K, F, fv);
  if (!rel) {
    for (int k = 0; k < 6; ++k) out[k] = fv[k];
    return;
  }
  double bv[6], Rb[9], pb[3], Rf[9], pf[3];
  frame_vel_lwa(K, base, bv);
  frame_placement(K, base, Rb, pb);
  frame_placement(K, F, Rf, pf);
  double rel_p[3] = {pf[0] - pb[0], pf[1] - pb[1], pf[2] - pb[2]};
  double corr[3];
  cross3(bv + 3, rel_p, corr);
  double rl[3], ra[3];
  for (int k = 0; k < 3; ++k) { rl[k] = fv[k] - bv[k] - corr[k]; ra[k] = fv[3 + k] - bv[3 + k]; }
  double rlb[3], rab[3];
  mattvec(Rb, rl, rlb);
  mattvec(Rb, ra, rab);
  out[0] = rlb[0]; out[1] = rlb[1]; out[2] = fv[2];
  out[3] = rab[0]; out[4] = rab[1]; out[5] = fv[5];
}

// Full-array accessors for the tree passes.
struct ArrIn {
  const double* a;
  PL_HD double operator[](int k) const { return a ? a[k] : 0.0; }
};

// rnea_dynamics(ext)(q, v, a, forces): the OCP's RNEA pass on full arrays.
PL_HD void rnea_full(const PlModel& M, const PlOcpConst& O, const double* q, const double* v, const double* a,
                     const double* f, double* tau) {
  double kst[PL_KIN_STORE];
  NodeKin<double> kin;
  kin.store = kst;
  kin.stride = 1;
  const RevQArr<double> qr{q};
  tree_pass<double>(M, O, q, qr, ArrIn{v}, ArrIn{a}, ArrIn{f}, true, false, kin);
  for (int k = 0; k < 6; ++k) tau[k] = kin.tau[k];
  for (int k = 6; k < M.nv; ++k) tau[k] = kin.tau_j(k - 6);
}

// Solve the 6x6 system A x = b in place (Gaussian elimination, partial pivoting).
PL_HD void solve6(double* A, double* b) {
  for (int c = 0; c < 6; ++c) {
    int piv = c;
    for (int r = c + 1; r < 6; ++r)
      if (fabs(A[6 * r + c]) > fabs(A[6 * piv + c])) piv = r;
    if (piv != c) {
      for (int k = 0; k < 6; ++k) { double t = A[6 * c + k]; A[6 * c + k] = A[6 * piv + k]; A[6 * piv + k] = t; }
      double t = b[c]; b[c] = b[piv]; b[piv] = t;
    }
    const double inv = 1.0 / A[6 * c + c];
    for (int r = c + 1; r < 6; ++r) {
      const double fr = A[6 * r + c] * inv;
      for (int k = c; k < 6; ++k) A[6 * r + k] -= fr * A[6 * c + k];
      b[r] -= fr * b[c];
    }
  }
  for (int r = 5; r >= 0; --r) {
    double t = b[r];
    for (int k = r + 1; k < 6; ++k) t -= A[6 * r + k] * b[k];
    b[r] = t / A[6 * r + r];
  }
}

// Centroidal momentum h_G = A_G(q) v, CoM moment and (optionally) com_dynamics.
PL_HD void centroidal_full(const PlModel& M, const PlOcpConst& O, const double* q, const double* v, const double* f,
                           double* hg, double* hdot) {
  const RevQArr<double> qr{q};
  centroidal_pass<double>(M, O, q, qr, ArrIn{v}, ArrIn{f}, v != nullptr, f != nullptr, hg, hdot);
}

// d/dt h_G = A_G(q) a + dA_G/dt(q, v) v (pinocchio dccrba applied to v, plus A a):
// Newton-Euler body forces without gravity, summed in world axes at the origin and
// moved to the CoM (the CoM drift term vanishes: c_dot x m c_dot = 0).
PL_HD void momentum_rate(const PlModel& M, const double* q, const double* v, const double* a, double* out) {
  FkAll K;
  fk_all(M, q, v, K);
  double acc[PL_MAXJ][6];
  double Hd[6] = {0, 0, 0, 0, 0, 0}, mc[3] = {0, 0, 0};
  for (int j = 1; j < M.njoints; ++j) {
    const int par = M.parent[j];
    double aj[6];
    if (M.jtype[j] == PL_JT_FREEFLYER) {
      for (int k = 0; k < 6; ++k) aj[k] = a[M.idx_v[j] + k];  // c_J = 0, v x v_J = 0 for the root
    } else {
      double s, c, lR[9];
      sincos_s(q[M.idx_q[j]], &s, &c);
      rev_rot(M, j, s, c, lR);
      act_inv_motion(lR, M.jp[j], acc[par], aj);
      const double qd = v[M.idx_v[j]], qdd = a[M.idx_v[j]];
      const double* ax = M.axis[j];
      const double wJ[3] = {ax[0] * qd, ax[1] * qd, ax[2] * qd};
      double t1[3], t2[3];
      cross3(K.vl[j], wJ, t1);      // v_lin x w_J
      cross3(K.vl[j] + 3, wJ, t2);  // w x w_J
      for (int k = 0; k < 3; ++k) { aj[k] += t1[k]; aj[3 + k] += ax[k] * qdd + t2[k]; }
    }
    for (int k = 0; k < 6; ++k) acc[j][k] = aj[k];
    double fj[6], h[6], vxh[6];
    inertia_mul(M.mass[j], M.lever[j], M.Ic[j], aj, fj);
    inertia_mul(M.mass[j], M.lever[j], M.Ic[j], K.vl[j], h);
    motion_cross_force(K.vl[j], h, vxh);
    for (int k = 0; k < 6; ++k) fj[k] += vxh[k];
    double fw[6];
    act_force(K.oR[j], K.op[j], fj, fw);
    for (int k = 0; k < 6; ++k) Hd[k] += fw[k];
    double lc[3];
    matvec(K.oR[j], M.lever[j], lc);
    for (int k = 0; k < 3; ++k) mc[k] += M.mass[j] * (K.op[j][k] + lc[k]);
  }
  double com[3] = {mc[0] / M.total_mass, mc[1] / M.total_mass, mc[2] / M.total_mass}, cx[3];
  cross3(com, Hd, cx);
  for (int k = 0; k < 3; ++k) { out[k] = Hd[k]; out[3 + k] = Hd[3 + k] - cx[k]; }
}

// Shared primal of the ABA Jacobian lanes of one node (rows.h PL_ABA_SH): q, v from
// x_init + dx; the mass matrix by RNEA columns (as crba below), its Cholesky factor, and
// a = M^-1 ([0; tau_j] - RNEA(q, v, 0, f)).  Split in two so a wave can spread the
// RNEA columns over its lanes: column c < nv is M e_c + t0, c = nv is t0 = RNEA(q, 0, 0),
// c = nv + 1 is RNEA(q, v, 0, f); aba_primal_finish combines them (raw: (nv + 2) x nv).
PL_HD void aba_primal_column(const PlModel& M, const PlOcpConst& O, const double* p, const double* dx, int c,
                             double* out) {
  const int nq = O.nq, nv = O.nv, nj = O.nj;
  const double* xi = p + O.P.x_init;
  const double* u = dx + O.ndx;
  double q[PL_MAXQ], v[PL_MAXV], z[PL_MAXV], e[PL_MAXV];
  VecIn<double> dq{dx, nullptr, 0.0, -1};
  integrate_ff<double>(xi, dq, q);
  for (int k = 7; k < nq; ++k) q[k] = xi[k] + dx[k - 1];
  for (int k = 0; k < nv; ++k) {
    v[k] = xi[nq + k] + dx[nv + k];
    z[k] = 0.0;
    e[k] = (k == c) ? 1.0 : 0.0;
  }
  if (c < nv) rnea_full(M, O, q, z, e, nullptr, out);
  else if (c == nv) rnea_full(M, O, q, z, z, nullptr, out);
  else rnea_full(M, O, q, v, z, u + nj, out);  // nle - J^T f
}

PL_HD void aba_primal_finish(const PlOcpConst& O, const double* dx, const double* raw, double* sh) {
  const int nv = O.nv;
  const double* u = dx + O.ndx;
  const double* t0 = raw + nv * nv;
  const double* bq = raw + (nv + 1) * nv;
  double* L = sh + PL_MAXV;
  for (int c = 0; c < nv; ++c)
    for (int r = c; r < nv; ++r) L[r * (r + 1) / 2 + c] = raw[c * nv + r] - t0[r];
  for (int c = 0; c < nv; ++c) {  // Cholesky in place
    double* Lc = L + c * (c + 1) / 2;
    double dd = Lc[c];
    for (int k = 0; k < c; ++k) dd -= Lc[k] * Lc[k];
    dd = sqrt(dd);
    Lc[c] = dd;
    for (int r = c + 1; r < nv; ++r) {
      double* Lr = L + r * (r + 1) / 2;
      double t = Lr[c];
      for (int k = 0; k < c; ++k) t -= Lr[k] * Lc[k];
      Lr[c] = t / dd;
    }
  }
  for (int k = 0; k < nv; ++k) sh[k] = (k < 6 ? 0.0 : u[k - 6]) - bq[k];
  chol_solve(L, nv, sh);
}

// Serial form (host callers: the CPU baseline and the host row tests).
PL_HD void aba_primal(const PlModel& M, const PlOcpConst& O, const double* p, const double* dx, double* sh) {
  double raw[(PL_MAXV + 2) * PL_MAXV];
  for (int c = 0; c < O.nv + 2; ++c) aba_primal_column(M, O, p, dx, c, raw + c * O.nv);
  aba_primal_finish(O, dx, raw, sh);
}

// One sample of function `fn`.  O carries the contact frames (feet [+ ext], nee)
// and the base frame; F is the frame argument of the frame functions.
PL_HD void dyn_eval(const PlModel& M, const PlOcpConst& O, const PlFrameRef& F, int fn, int flags,
                    const double* in0, const double* in1, const double* in2, const double* in3, double* out) {
  const int nv = M.nv, nq = M.nq;
  double z[PL_MAXV], e[PL_MAXV];
  for (int k = 0; k < PL_MAXV; ++k) z[k] = 0.0;
  switch (fn) {
    case PL_FN_RNEA:
      rnea_full(M, O, in0, in1, in2, in3, out);
      break;
    case PL_FN_ABA: {
      aba_forward<double>(M, O, in0, in1, ArrIn{in2}, ArrIn{in3}, out);
    } break;
    case PL_FN_FRAME_POS: {
      FkAll K;
      fk_all(M, in0, nullptr, K);
      double R[9];
      frame_placement(K, F, R, out);
    } break;
    case PL_FN_FRAME_VEL: {
      FkAll K;
      fk_all(M, in0, in1, K);
      frame_velocity(K, F, O.base, (flags & 2) != 0, out);
    } break;
    case PL_FN_GAPS_WB: {
      double tau[PL_MAXV];
      rnea_full(M, O, in0, in1, in2, in3, tau);
      for (int k = 0; k < 6; ++k) out[k] = tau[k];
    } break;
    case PL_FN_BASE_ACC_WB: {
      // M_bb a_b = -nle_b - M_bj a_j + sum J_c,lin,b^T f  <=>  rnea(q, v, [a_b, a_j], f)[:6] = 0
      double a[PL_MAXV], tau[PL_MAXV], t0[PL_MAXV], Mbb[36], b[6];
      for (int k = 0; k < 6; ++k) a[k] = 0.0;
      for (int k = 6; k < nv; ++k) a[k] = in2[k - 6];
      rnea_full(M, O, in0, in1, a, in3, tau);
      rnea_full(M, O, in0, z, z, nullptr, t0);
      for (int c = 0; c < 6; ++c) {
        for (int k = 0; k < nv; ++k) e[k] = (k == c) ? 1.0 : 0.0;
        double tc[PL_MAXV];
        rnea_full(M, O, in0, z, e, nullptr, tc);
        for (int r = 0; r < 6; ++r) Mbb[6 * r + c] = tc[r] - t0[r];
      }
      for (int k = 0; k < 6; ++k) b[k] = -tau[k];
      solve6(Mbb, b);
      for (int k = 0; k < 6; ++k) out[k] = b[k];
    } break;
    case PL_FN_COM_DYN: {
      double hg[6];
      centroidal_full(M, O, in0, nullptr, in1, hg, out);
    } break;
    case PL_FN_GAPS_CA: {  // A a + dA v - dh (dynamics_centroidal_acc.py:92-119)
      double rate[6], hg[6], hd[6];
      momentum_rate(M, in0, in1, in2, rate);
      centroidal_full(M, O, in0, nullptr, in3, hg, hd);
      for (int k = 0; k < 6; ++k) out[k] = rate[k] - M.total_mass * hd[k];
    } break;
    case PL_FN_GAPS_CV: {
      double hd[6];
      centroidal_full(M, O, in1, in2, nullptr, out, hd);
      for (int k = 0; k < 6; ++k) out[k] -= M.total_mass * in0[k];
    } break;
    case PL_FN_BASE_VEL_CV:
    case PL_FN_BASE_ACC_CV: {
      // A_b = A_G[:, :6]; base_vel: v_b = A_b^-1 (m h - A_j v_j);
      // base_acc: a_b = A_b^-1 (dh - dA_G v - A_j a_j), dh = [sum f + m g, sum (p - c) x f]
      double Ab[36], b[6], hd[6];
      for (int c = 0; c < 6; ++c) {
        for (int k = 0; k < nv; ++k) e[k] = (k == c) ? 1.0 : 0.0;
        double col[6];
        centroidal_full(M, O, fn == PL_FN_BASE_VEL_CV ? in1 : in0, e, nullptr, col, hd);
        for (int r = 0; r < 6; ++r) Ab[6 * r + c] = col[r];
      }
      double w[PL_MAXV];
      for (int k = 0; k < 6; ++k) w[k] = 0.0;
      if (fn == PL_FN_BASE_VEL_CV) {
        for (int k = 6; k < nv; ++k) w[k] = in2[k - 6];
        double aj[6];
        centroidal_full(M, O, in1, w, nullptr, aj, hd);
        for (int k = 0; k < 6; ++k) b[k] = M.total_mass * in0[k] - aj[k];
      } else {
        for (int k = 6; k < nv; ++k) w[k] = in2[k - 6];
        double rate[6], hg[6];
        momentum_rate(M, in0, in1, w, rate);
        centroidal_full(M, O, in0, nullptr, in3, hg, hd);
        for (int k = 0; k < 6; ++k) b[k] = M.total_mass * hd[k] - rate[k];
      }
      solve6(Ab, b);
      for (int k = 0; k < 6; ++k) out[k] = b[k];
    } break;
    case PL_FN_CRBA: {
      double t0[PL_MAXV], tc[PL_MAXV];
      rnea_full(M, O, in0, z, z, nullptr, t0);
      for (int c = 0; c < nv; ++c) {
        for (int k = 0; k < nv; ++k) e[k] = (k == c) ? 1.0 : 0.0;
        rnea_full(M, O, in0, z, e, nullptr, tc);
        for (int r = 0; r < nv; ++r) out[r * nv + c] = tc[r] - t0[r];
      }
    } break;
    case PL_FN_NLE:
      rnea_full(M, O, in0, in1, z, nullptr, out);
      break;
    case PL_FN_FRAME_JAC: {
      for (int c = 0; c < nv; ++c) {
        for (int k = 0; k < nv; ++k) e[k] = (k == c) ? 1.0 : 0.0;
        FkAll K;
        fk_all(M, in0, e, K);
        double col[6];
        frame_vel_lwa(K, F, col);
        for (int r = 0; r < 6; ++r) out[r * nv + c] = col[r];
      }
    } break;
    case PL_FN_CMAP: {
      double hd[6];
      for (int c = 0; c < nv; ++c) {
        for (int k = 0; k < nv; ++k) e[k] = (k == c) ? 1.0 : 0.0;
        double col[6];
        centroidal_full(M, O, in0, e, nullptr, col, hd);
        for (int r = 0; r < 6; ++r) out[r * nv + c] = col[r];
      }
    } break;
    case PL_FN_COM: {
      FkAll K;
      fk_all(M, in0, nullptr, K);
      double mc[3] = {0, 0, 0};
      for (int j = 1; j < M.njoints; ++j) {
        double lc[3];
        matvec(K.oR[j], M.lever[j], lc);
        for (int k = 0; k < 3; ++k) mc[k] += M.mass[j] * (K.op[j][k] + lc[k]);
      }
      for (int k = 0; k < 3; ++k) out[k] = mc[k] / M.total_mass;
    } break;
    case PL_FN_INTEGRATE_WB: {
      VecIn<double> acc{in1, nullptr, 0.0, -1};
      integrate_q<double>(M, in0, acc, out);
      for (int k = 0; k < nv; ++k) out[nq + k] = in0[nq + k] + in1[nv + k];
    } break;
    case PL_FN_DIFFERENCE_WB:
      difference_q(M, in0, in1, out);
      for (int k = 0; k < nv; ++k) out[nv + k] = in1[nq + k] - in0[nq + k];
      break;
    case PL_FN_INTEGRATE_CV: {
      VecIn<double> acc{in1 + 6, nullptr, 0.0, -1};
      for (int k = 0; k < 6; ++k) out[k] = in0[k] + in1[k];
      integrate_q<double>(M, in0 + 6, acc, out + 6);
    } break;
    case PL_FN_DIFFERENCE_CV:
      for (int k = 0; k < 6; ++k) out[k] = in1[k] - in0[k];
      difference_q(M, in0 + 6, in1 + 6, out + 6);
      break;
    default:
      break;
  }
}

}  // namespace pl
