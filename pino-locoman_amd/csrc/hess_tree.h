// Lagrangian-Hessian tree sweeps of the whole_body_rnea / whole_body_acc state pairs (k_hess.hip), on
// the host and the device (PL_HD: tests/native/hess_host.cpp builds the same code for the CPU).
//
// phi = lambda_tau^T tau(q, v, a, f) + sum_e mu_e . v_foot,e(q, v) is one forward sweep over a chain
// (virtual work, k_hess.hip k_lag_hess_tree); its curvature in the state is wanted for the
// (dq, dq) and (dq, dv) pairs of every node block.
//   tree_pair   one hyper-dual sweep seeded on both columns of a pair (the r05 kernel);
//   tree_col    forward-over-reverse (r06): a dual sweep seeded on the column j, then the reverse
//               (adjoint) sweep of the same chain in dual numbers, whose tangents are the whole
//               column d^2 phi / d x_j d x_k over the chain's coordinates at once.
#pragma once
#include <stdint.h>
#include "rows.h"

namespace hess {

using pl::VecIn;

template <class S> PL_HD void crossd(const double* a, const S* b, S* o) {  // a x b, a constant
  o[0] = a[1] * b[2] - a[2] * b[1];
  o[1] = a[2] * b[0] - a[0] * b[2];
  o[2] = a[0] * b[1] - a[1] * b[0];
}
template <class S, class C> PL_HD void rot_core_t(const PlModel& M, int j, const C& s, const C& c, const S* e, S* out) {
  switch (M.axis_kind[j]) {  // out = Rot(axis_j, q)^T e
    case PL_AX_X:
      out[0] = e[0]; out[1] = c * e[1] + s * e[2]; out[2] = c * e[2] - s * e[1];
      break;
    case PL_AX_Y:
      out[0] = c * e[0] - s * e[2]; out[1] = e[1]; out[2] = s * e[0] + c * e[2];
      break;
    case PL_AX_Z:
      out[0] = c * e[0] + s * e[1]; out[1] = c * e[1] - s * e[0]; out[2] = e[2];
      break;
    default: {  // Rodrigues I + s [a]x + (1 - c) [a]x^2, transposed
      const double* a = M.axis[j];
      const double K[9] = {0, -a[2], a[1], a[2], 0, -a[0], -a[1], a[0], 0};
      const C oc = 1.0 - c;
      for (int r = 0; r < 3; ++r) {
        S t = e[r];
        for (int q = 0; q < 3; ++q) {
          const double kk = K[3 * q] * K[r] + K[3 * q + 1] * K[3 + r] + K[3 * q + 2] * K[6 + r];  // ([a]x^2)_qr
          t += (s * K[3 * q + r] + oc * kk) * e[q];
        }
        out[r] = t;
      }
    }
  }
}
// out = R_j^T d for the revolute joint rotation R_j = jR Rot(axis, q_j) (rbd.h rev_rot), applied as
// Rot^T (jR^T d) so that no hyper-dual 3x3 matrix is formed (jR constant; Rot a plane rotation for
// the axis-aligned joints)
template <class S, class C> PL_HD void rot_t(const PlModel& M, int j, const C& s, const C& c, const S* d, S* out) {
  S e[3];
  pl::mattvec(M.jR[j], d, e);
  rot_core_t(M, j, s, c, e, out);
}
// out = R_j d (the inverse of rot_t: Rot(q) = Rot(-q)^T, then jR)
template <class S, class C> PL_HD void rot_j(const PlModel& M, int j, const C& s, const C& c, const S* d, S* out) {
  S e[3];
  const C ms = -s;
  rot_core_t(M, j, ms, c, d, e);
  pl::matvec(M.jR[j], e, out);
}
// actInv of a motion through joint j: [R^T (m_lin - p x m_ang); R^T m_ang], p the joint placement
template <class S, class C> PL_HD void act_inv_j(const PlModel& M, int j, const C& s, const C& c, const S* m, S* out) {
  S pxw[3];
  crossd(M.jp[j], m + 3, pxw);
  S d[3] = {m[0] - pxw[0], m[1] - pxw[1], m[2] - pxw[2]};
  rot_t(M, j, s, c, d, out);
  rot_t(M, j, s, c, m + 3, out + 3);
}
// f = I a + v x* I v  (body axes; inertia (m, c, Ic) constant)
template <class S> PL_HD void body_wrench(double m, const double* c, const double* Ic, const S* a, const S* v,
                                               S* f) {
  S t[3], h[6];
  crossd(c, v + 3, t);
  for (int k = 0; k < 3; ++k) h[k] = m * (v[k] - t[k]);
  crossd(c, h, t);
  for (int k = 0; k < 3; ++k) h[3 + k] = Ic[3 * k] * v[3] + Ic[3 * k + 1] * v[4] + Ic[3 * k + 2] * v[5] + t[k];
  pl::motion_cross_force(v, h, f);
  crossd(c, a + 3, t);
  S fl[3];
  for (int k = 0; k < 3; ++k) fl[k] = m * (a[k] - t[k]);
  crossd(c, fl, t);
  for (int k = 0; k < 3; ++k) {
    f[k] += fl[k];
    f[3 + k] += Ic[3 * k] * a[3] + Ic[3 * k + 1] * a[4] + Ic[3 * k + 2] * a[5] + t[k];
  }
}
PL_HD int block_row(const PlOcpConst& O, int type, int kind, int arg) {  // first row of a block, -1: none
  int r = 0;
  for (int bi = 0; bi < O.nblk[type]; ++bi) {
    const PlRowBlock B = O.blk[type][bi];
    if (B.kind == kind && (arg < 0 || B.arg == arg)) return r;
    r += B.count;
  }
  return -1;
}
// The sweep's view of one node: the root pose, the state accessors and the world-axis vectors it
// rotates into a body's axes (oR_b^T x, by a walk from the root: R0^T, then R_j^T joint by joint)
struct TreeSweep {
  const PlModel& M;
  const HDual* qb;
  const pl::RevQ<HDual, VecIn<HDual>>& qrev;
  // two vectors in one walk (a foot's force and its velocity rows' multipliers)
  template <class X> PL_HD void to_body2(int first, int kk, const X* xw, const double* yw, HDual* ox,
                                              HDual* oy) const {
    HDual R0[9];
    pl::quat_to_R(qb + 3, R0);
    pl::mattvec(R0, xw, ox);
    pl::mattvec(R0, yw, oy);
    for (int k2 = 0; k2 <= kk; ++k2) {
      const int j2 = first + k2;
      HDual s2, c2, t[3];
      sincos_s(qrev(M.idx_q[j2]), &s2, &c2);
      rot_t(M, j2, s2, c2, ox, t);
      for (int q = 0; q < 3; ++q) ox[q] = t[q];
      rot_t(M, j2, s2, c2, oy, t);
      for (int q = 0; q < 3; ++q) oy[q] = t[q];
    }
  }
  template <class X> PL_HD void to_body(int first, int kk, const X* xw, HDual* out) const {
    HDual R0[9];
    pl::quat_to_R(qb + 3, R0);
    pl::mattvec(R0, xw, out);
    for (int k2 = 0; k2 <= kk; ++k2) {
      const int j2 = first + k2;
      HDual s2, c2, t[3];
      sincos_s(qrev(M.idx_q[j2]), &s2, &c2);
      rot_t(M, j2, s2, c2, out, t);
      for (int q = 0; q < 3; ++q) out[q] = t[q];
    }
  }
};

// contact forces on body j (f_b -= [fl; p x fl], fl = oR^T f_world) and its feet's velocity rows
// (phi += (v_lin + w x p) . oR^T mu); first / kk: body j's place in its chain (first = -1: the root)
// (fx: the contact forces; f(e, c): the external frame's, plain or seeded -- k_lag_hess_tree<true>;
// frame ef's force and multipliers arrive already in body axes: cf, cg (cg only if has_mu))
PL_HD void foot_mu(const PlOcpConst& O, int type, int node, int e, const double* lam, const double* p,
                        double* mu, bool* has) {  // a foot's velocity-row multipliers times coefficients
  const int rxy = e < O.nfeet ? block_row(O, type, PL_RB_FVXY, e) : -1;
  const int rz = e < O.nfeet ? block_row(O, type, PL_RB_FVZ, e) : -1;
  *has = rxy >= 0 || rz >= 0;
  const double c = e < O.nfeet ? p[O.P.contact + 4 * node + e] : 0.0;
  mu[0] = rxy >= 0 ? c * lam[rxy] : 0.0;
  mu[1] = rxy >= 0 ? c * lam[rxy + 1] : 0.0;
  mu[2] = rz >= 0 ? lam[rz] : 0.0;
}
template <class F3>
PL_HD void body_frames(const PlOcpConst& O, const TreeSweep& T, int first, int kk, int j, int type, int node,
                            const HDual* vj, const double* fx, const F3& f, const double* lam, const double* p,
                            HDual* fb, HDual& phi, int ef = -1, const HDual* cf = nullptr, const HDual* cg = nullptr,
                            bool has_mu = false) {
  for (int e = 0; e < O.nee; ++e) {
    const PlFrameRef& F = (e < O.nfeet) ? O.feet[e] : O.ext;
    if (F.joint != j) continue;
    HDual fl[3], t[3];
    if (e == ef) {  // carried along the chain
      for (int k = 0; k < 3; ++k) fl[k] = cf[k];
      if (has_mu) {
        HDual wxp[3];
        crossd(F.p, vj + 3, wxp);  // p x w = -(w x p)
        for (int k = 0; k < 3; ++k) phi += (vj[k] - wxp[k]) * cg[k];
      }
      crossd(F.p, fl, t);
      for (int k = 0; k < 3; ++k) { fb[k] -= fl[k]; fb[3 + k] -= t[k]; }
      continue;
    }
    const int rxy = e < O.nfeet ? block_row(O, type, PL_RB_FVXY, e) : -1;
    const int rz = e < O.nfeet ? block_row(O, type, PL_RB_FVZ, e) : -1;
    if (e >= O.nfeet) {  // the external force frame (seeded in k_lag_hess_tree<true>)
      const decltype(f(0, 0)) fw[3] = {f(e, 0), f(e, 1), f(e, 2)};
      T.to_body(first, kk, fw, fl);
    } else if (rxy >= 0 || rz >= 0) {
      const double c = p[O.P.contact + 4 * node + e];
      const double mu[3] = {rxy >= 0 ? c * lam[rxy] : 0.0, rxy >= 0 ? c * lam[rxy + 1] : 0.0,
                            rz >= 0 ? lam[rz] : 0.0};
      HDual g[3], wxp[3];
      T.to_body2(first, kk, fx + 3 * e, mu, fl, g);
      crossd(F.p, vj + 3, wxp);  // p x w = -(w x p)
      for (int k = 0; k < 3; ++k) phi += (vj[k] - wxp[k]) * g[k];
    } else {
      T.to_body(first, kk, fx + 3 * e, fl);
    }
    crossd(F.p, fl, t);
    for (int k = 0; k < 3; ++k) { fb[k] -= fl[k]; fb[3 + k] -= t[k]; }
  }
}

// The root pose for the state pairs: nothing downstream reads the base position (translation
// invariance: it is set to 0), and the orientation is q0 (x) exp(w / 2), w = dq_3..5, whose
// rotation matrix is R(q0) Exp(w) -- what integrate_ff's SE3 exponential, R -> quaternion and
// renormalisation give (the last two are the identity on rotations: their derivatives cancel
// analytically), without carrying them in hyper-duals.  Below the exp6 series threshold
// (rbd.h PL_TAYLOR_PREC3) sin(t/2)/t and cos(t/2) are their series in t^2 through t^4.
template <class S> PL_HD void base_pose(const double* xi, const VecIn<S>& dx, S* qb) {
  const S w[3] = {dx[3], dx[4], dx[5]};
  const S t2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  S f, g;
  if (val(t2) < PL_TAYLOR_PREC3 * PL_TAYLOR_PREC3) {
    f = 0.5 - t2 * (1.0 / 48.0) + (t2 * t2) * (1.0 / 3840.0);
    g = 1.0 - t2 * 0.125 + (t2 * t2) * (1.0 / 384.0);
  } else {
    const S th = sqrt_s(t2);
    S sh, ch;
    sincos_s(th * 0.5, &sh, &ch);
    f = sh / th;
    g = ch;
  }
  const S u[3] = {f * w[0], f * w[1], f * w[2]};  // exp(w / 2) = [u; g]
  const double* q0 = xi + 3;                           // [x y z w]
  S cr[3];
  crossd(q0, u, cr);
  for (int k = 0; k < 3; ++k) qb[3 + k] = q0[3] * u[k] + q0[k] * g + cr[k];
  qb[6] = q0[3] * g - (q0[0] * u[0] + q0[1] * u[1] + q0[2] * u[2]);
  for (int k = 0; k < 3; ++k) qb[k] = S(0.0);
}


// One (j, k) state pair of node i (j <= k, dx indices; only_ch: the pair's chain, -1 the whole tree):
// the entry of the node block the r05 kernel k_lag_hess_tree wrote.  SF: the (dq, f_ext) pairs with
// the external force seeded instead of dx_k.
template <bool SF>
PL_HD double tree_pair(const PlModel& M, const PlOcpConst& O, int i, int only_ch, int j, int k, const double* x,
                       const double* p, const double* lam) {
  if (j < 3) return 0.0;  // the RNEA and the frame velocities do not read the base position (rows.h seed_pos)
  const double* xi = p + O.P.x_init;
  const int nv = O.nv, ndx = O.ndx, type = pl::node_type(O, i);
  const VecIn<HDual> dx{x, nullptr, 0.0, j, k};
  HDual qb[7];
  base_pose(xi, dx, qb);
  const pl::RevQ<HDual, VecIn<HDual>> qrev{xi, dx};
  const pl::VelAcc<HDual, VecIn<HDual>> vel{xi + O.nq, pl::sub_in(dx, nv)};
  const double* a = x + ndx;           // u = [a | f | tau_j]: constants for a state pair
  const double* fx = x + ndx + O.na;
  const int fk = k - ndx - O.na;  // SF: the seeded force component
  const auto f = [&](int e, int c) {
    if constexpr (SF) return HDual(fx[3 * e + c], 0.0, 3 * e + c == fk ? 1.0 : 0.0, 0.0);
    else return fx[3 * e + c];
  };
  const int rb = block_row(O, type, PL_RB_RNEA_BASE, -1), rt = block_row(O, type, PL_RB_TAU_EQ, -1);
  HDual phi(0.0);
  // the sweep's carried state is v, a and L of the current body; the root's pose and motion are
  // recomputed per chain from q_b, and a body's world rotation (its frames) by a walk from the root
  const double mg[3] = {-M.gravity[0], -M.gravity[1], -M.gravity[2]};
  const TreeSweep T{M, qb, qrev};
  if (only_ch < 0 && rb >= 0) {  // the root body's own term (base coordinates only)
    HDual v1[6], a1[6], f1[6];
    for (int c = 0; c < 6; ++c) v1[c] = vel[c];
    T.to_body(0, -1, mg, a1);
    for (int c = 0; c < 3; ++c) { a1[c] = a1[c] + a[c]; a1[3 + c] = HDual(a[3 + c]); }
    body_wrench(M.mass[1], M.lever[1], M.Ic[1], a1, v1, f1);
    body_frames(O, T, 0, -1, 1, type, i, v1, fx, f, lam, p, f1, phi);
    for (int c = 0; c < 6; ++c) phi += lam[rb + c] * f1[c];
  }
  for (int ch = 0; ch < M.nchains; ++ch) {
    if (only_ch >= 0 && ch != only_ch) continue;
    const int first = M.chain_first[ch], L = M.chain_len[ch];
    // the chain's first frame (a foot, or the external force frame): its world force and
    // velocity-row multipliers are rotated into body axes joint by joint with the sweep's own
    // rotations (cf, cg) instead of a walk from the root at the frame
    int ef = -1, ej = -1;
    for (int e = 0; e < O.nee && ef < 0; ++e) {
      const int fj = e < O.nfeet ? O.feet[e].joint : O.ext.joint;
      if (fj >= first && fj < first + L) { ef = e; ej = fj; }
    }
    HDual pv[6], pa[6], pL[6], cf[3], cg[3];
    bool has_mu = false;
    {
      HDual R0[9];
      pl::quat_to_R(qb + 3, R0);
      pl::mattvec(R0, mg, pa);
      if (ef >= 0) {
        const decltype(f(0, 0)) fw[3] = {f(ef, 0), f(ef, 1), f(ef, 2)};
        pl::mattvec(R0, fw, cf);
        double mu[3];
        foot_mu(O, type, i, ef, lam, p, mu, &has_mu);
        if (has_mu) pl::mattvec(R0, mu, cg);
      }
    }
    for (int c = 0; c < 3; ++c) { pa[c] = pa[c] + a[c]; pa[3 + c] = HDual(a[3 + c]); }
    for (int c = 0; c < 6; ++c) { pv[c] = vel[c]; pL[c] = HDual(rb >= 0 ? lam[rb + c] : 0.0); }
    for (int kk = 0; kk < L; ++kk) {
      const int jt = first + kk;
      HDual s, c;
      sincos_s(qrev(M.idx_q[jt]), &s, &c);
      if (ef >= 0 && jt <= ej) {
        HDual t3[3];
        rot_t(M, jt, s, c, cf, t3);
        for (int q = 0; q < 3; ++q) cf[q] = t3[q];
        if (has_mu) {
          rot_t(M, jt, s, c, cg, t3);
          for (int q = 0; q < 3; ++q) cg[q] = t3[q];
        }
      }
      const double* ax = M.axis[jt];
      const int iv = M.idx_v[jt];
      const HDual qd = vel[iv];
      HDual vj[6], aj[6], t[3];
      act_inv_j(M, jt, s, c, pv, vj);
      for (int q = 0; q < 3; ++q) vj[3 + q] += ax[q] * qd;
      act_inv_j(M, jt, s, c, pa, aj);
      // + S qdd + v x vJ, vJ = [0; ax qd]:  [v_lin x ax; w x ax] qd
      crossd(ax, vj, t);
      for (int q = 0; q < 3; ++q) aj[q] -= t[q] * qd;
      crossd(ax, vj + 3, t);
      for (int q = 0; q < 3; ++q) aj[3 + q] += ax[q] * a[iv] - t[q] * qd;
      for (int q = 0; q < 6; ++q) { pv[q] = vj[q]; pa[q] = aj[q]; }
      act_inv_j(M, jt, s, c, pL, aj);  // L_j (aj: scratch)
      const double lj = rt >= 0 ? lam[rt + iv - 6] : 0.0;
      for (int q = 0; q < 3; ++q) aj[3 + q] += ax[q] * lj;
      for (int q = 0; q < 6; ++q) pL[q] = aj[q];
      HDual fj[6];
      body_wrench(M.mass[jt], M.lever[jt], M.Ic[jt], pa, pv, fj);
      body_frames(O, T, first, kk, jt, type, i, pv, fx, f, lam, p, fj, phi, ef, cf, cg, has_mu);
      for (int q = 0; q < 6; ++q) phi += pL[q] * fj[q];
    }
  }
  return phi.c;
}

// ---- forward-over-reverse columns (r06) -------------------------------------------------------
// Local coordinates of a chain's state block (the coordinates its sweep reads) = the bits of a
// work item's mask:
//   0..2  dq of the base position   3..5  dq of the base rotation   6..11  dv of the base
//   12 + kk   dq of the chain's joint kk        12 + L + kk   dv of joint kk
// (only_ch < 0, the whole tree: the base coordinates 0..11 only).
PL_HD int col_coord(const PlModel& M, const PlOcpConst& O, int only_ch, int loc) {
  if (loc < 6) return loc;
  if (loc < 12) return O.nv + loc - 6;
  const int L = M.chain_len[only_ch], first = M.chain_first[only_ch];
  const int kk = loc - 12;
  return kk < L ? M.idx_v[first + kk] : O.nv + M.idx_v[first + kk - L];
}

// spatial inertia (body axes, mass m, CoM c, rotational inertia Ic at the CoM) times a motion
template <class S> PL_HD void inertia_mul(double m, const double* c, const double* Ic, const S* v, S* h) {
  S t[3];
  crossd(c, v + 3, t);
  for (int k = 0; k < 3; ++k) h[k] = m * (v[k] - t[k]);
  crossd(c, h, t);
  for (int k = 0; k < 3; ++k) h[3 + k] = Ic[3 * k] * v[3] + Ic[3 * k + 1] * v[4] + Ic[3 * k + 2] * v[5] + t[k];
}
// adjoint of body_wrench, f = I a + v x* (I v) (I symmetric):  ab += I fb,
//   vb += [h_l x fb_a; h_l x fb_l + h_a x fb_a] + I [fb_l x w + fb_a x v_l; fb_a x w],  h = I v
template <class S> PL_HD void body_wrench_adj(double m, const double* c, const double* Ic, const S* v, const S* fb,
                                             S* ab, S* vb) {
  S h[6], t[3], u[3], hb[6];
  inertia_mul(m, c, Ic, fb, hb);
  for (int k = 0; k < 6; ++k) ab[k] += hb[k];
  inertia_mul(m, c, Ic, v, h);
  pl::cross3(h, fb, t);
  pl::cross3(h + 3, fb + 3, u);
  for (int k = 0; k < 3; ++k) vb[3 + k] += t[k] + u[k];
  pl::cross3(h, fb + 3, t);
  for (int k = 0; k < 3; ++k) vb[k] += t[k];
  pl::cross3(fb, v + 3, t);
  pl::cross3(fb + 3, v, u);
  for (int k = 0; k < 3; ++k) hb[k] = t[k] + u[k];
  pl::cross3(fb + 3, v + 3, t);
  for (int k = 0; k < 3; ++k) hb[3 + k] = t[k];
  inertia_mul(m, c, Ic, hb, h);
  for (int k = 0; k < 6; ++k) vb[k] += h[k];
}
// act of a motion through joint j (the inverse of act_inv_j): [R m_l + p x (R m_a); R m_a]
template <class S, class C> PL_HD void act_j(const PlModel& M, int j, const C& s, const C& c, const S* m, S* out) {
  S t[3];
  rot_j(M, j, s, c, m + 3, out + 3);
  rot_j(M, j, s, c, m, t);
  S pxw[3];
  crossd(M.jp[j], out + 3, pxw);
  for (int k = 0; k < 3; ++k) out[k] = t[k] + pxw[k];
}
// adjoint of act_inv_j (a force transform): mbar = [R ybar_l; R ybar_a + p x (R ybar_l)]
template <class S, class C> PL_HD void act_inv_adj(const PlModel& M, int j, const C& s, const C& c, const S* yb, S* out) {
  S t[3];
  rot_j(M, j, s, c, yb, out);
  rot_j(M, j, s, c, yb + 3, t);
  S pxr[3];
  crossd(M.jp[j], out, pxr);
  for (int k = 0; k < 3; ++k) out[3 + k] = t[k] + pxr[k];
}
// theta-derivative of y = R_j^T d (R_j = jR Rot(axis, theta)): dy/dtheta = y x axis, so the angle's
// adjoint takes ybar . (y x axis) = y . (axis x ybar)
template <class S> PL_HD S ang_adj(const double* ax, const S* y, const S* yb) {
  S t[3];
  crossd(ax, yb, t);
  return y[0] * t[0] + y[1] * t[1] + y[2] * t[2];
}

// The column j (a dq coordinate, dx index) of the curvature of the tree rows of node i over the
// chain only_ch (-1: root and every chain), written for the local coordinates in `mask`:
// Hnode[max(j, k) (max + 1) / 2 + min(j, k)] for k = col_coord(loc), loc a bit of mask.  Same
// function phi as tree_pair<false> (the root / frame layout checked on the host: no frame on the
// root, at most one frame per chain), differentiated as: one forward sweep in Dual numbers seeded
// on dx_j, then the reverse sweep of the same chain (adjoints in Dual numbers; the forward values
// of each joint recovered from its outputs by the inverse motion transforms), whose tangents are
// d^2 phi / dx_j dx_k for every coordinate k of the chain at once.  The base rotation's adjoint
// goes through R0: d phi / dw_k = Rbar0 : dR0 / dw_k with dR0 / dw_k and d^2 R0 / dw_j dw_k from
// a hyper-dual evaluation of the root pose.
// WHOLE: the whole-tree base columns (only_ch < 0: the root term, every chain and the base rotation's
// adjoint); otherwise one chain, whose columns never write a base-rotation entry (the register
// budget of the chain items then holds no R0 adjoint).
template <bool WHOLE, class W>
PL_HD void tree_col(const PlModel& M, const PlOcpConst& O, int i, int only_ch, int j, uint32_t mask, const double* x,
                    const double* p, const double* lam, W&& write) {
  const auto kidx = [&](int loc) { return col_coord(M, O, only_ch, loc); };
  if (j < 3) {  // the RNEA and the frame velocities do not read the base position
    for (int loc = 0; loc < 32; ++loc)
      if (mask >> loc & 1u) write(kidx(loc), 0.0);
    return;
  }
  const double* xi = p + O.P.x_init;
  const int nv = O.nv, ndx = O.ndx, type = pl::node_type(O, i);
  const VecIn<Dual> dx{x, nullptr, 0.0, j};
  Dual R0[9];
  {
    Dual qb[7];
    base_pose(xi, dx, qb);
    pl::quat_to_R(qb + 3, R0);
  }
  const pl::RevQ<Dual, VecIn<Dual>> qrev{xi, dx};
  const pl::VelAcc<Dual, VecIn<Dual>> vel{xi + O.nq, pl::sub_in(dx, nv)};
  const double* a = x + ndx;
  const double* fx = x + ndx + O.na;
  const int rb = block_row(O, type, PL_RB_RNEA_BASE, -1), rt = block_row(O, type, PL_RB_TAU_EQ, -1);
  const double mg[3] = {-M.gravity[0], -M.gravity[1], -M.gravity[2]};
  Dual R0b[WHOLE ? 9 : 1], v0b[6];  // adjoints of R0 (whole-tree columns) and of the base velocity
  for (int q = 0; q < (WHOLE ? 9 : 1); ++q) R0b[q] = Dual(0.0);
  for (int q = 0; q < 6; ++q) v0b[q] = Dual(0.0);
  if (WHOLE && rb >= 0) {  // the root body's own term: phi += lam_b . body_wrench(a1, v1)
    Dual v1[6], a1b[6], v1b[6], fb[6];
    for (int c = 0; c < 6; ++c) { v1[c] = vel[c]; a1b[c] = Dual(0.0); v1b[c] = Dual(0.0); fb[c] = Dual(lam[rb + c]); }
    body_wrench_adj(M.mass[1], M.lever[1], M.Ic[1], v1, fb, a1b, v1b);
    for (int c = 0; c < 6; ++c) v0b[c] += v1b[c];
    for (int r = 0; r < 3; ++r)  // a1_lin = R0^T mg + a
      for (int c = 0; c < 3; ++c) R0b[3 * r + c] += mg[r] * a1b[c];
  }
  for (int ch = WHOLE ? 0 : only_ch; ch < (WHOLE ? M.nchains : only_ch + 1); ++ch) {
    const int first = M.chain_first[ch], L = M.chain_len[ch];
    int ef = -1, ej = -1;
    for (int e = 0; e < O.nee && ef < 0; ++e) {
      const int fj = e < O.nfeet ? O.feet[e].joint : O.ext.joint;
      if (fj >= first && fj < first + L) { ef = e; ej = fj; }
    }
    double fw[3] = {0.0, 0.0, 0.0}, mu[3] = {0.0, 0.0, 0.0};
    bool has_mu = false;
    Dual pv[6], pa[6], pL[6], cf[3], cg[3];
    pl::mattvec(R0, mg, pa);
    if (ef >= 0) {
      for (int c = 0; c < 3; ++c) fw[c] = fx[3 * ef + c];
      pl::mattvec(R0, fw, cf);
      foot_mu(O, type, i, ef, lam, p, mu, &has_mu);
      pl::mattvec(R0, mu, cg);
    } else {
      for (int c = 0; c < 3; ++c) cf[c] = cg[c] = Dual(0.0);
    }
    for (int c = 0; c < 3; ++c) { pa[c] = pa[c] + a[c]; pa[3 + c] = Dual(a[3 + c]); }
    for (int c = 0; c < 6; ++c) { pv[c] = vel[c]; pL[c] = Dual(rb >= 0 ? lam[rb + c] : 0.0); }
    // ---- forward (values and d / dx_j), keeping only the chain's last state
    for (int kk = 0; kk < L; ++kk) {
      const int jt = first + kk;
      Dual s, c, t3[3];
      sincos_s(qrev(M.idx_q[jt]), &s, &c);
      if (ef >= 0 && jt <= ej) {
        rot_t(M, jt, s, c, cf, t3);
        for (int q = 0; q < 3; ++q) cf[q] = t3[q];
        rot_t(M, jt, s, c, cg, t3);
        for (int q = 0; q < 3; ++q) cg[q] = t3[q];
      }
      const double* ax = M.axis[jt];
      const int iv = M.idx_v[jt];
      const Dual qd = vel[iv];
      Dual y[6], t[3];
      act_inv_j(M, jt, s, c, pv, y);
      for (int q = 0; q < 3; ++q) y[3 + q] += ax[q] * qd;
      for (int q = 0; q < 6; ++q) pv[q] = y[q];
      act_inv_j(M, jt, s, c, pa, y);
      crossd(ax, pv, t);
      for (int q = 0; q < 3; ++q) y[q] -= t[q] * qd;
      crossd(ax, pv + 3, t);
      for (int q = 0; q < 3; ++q) y[3 + q] += ax[q] * a[iv] - t[q] * qd;
      for (int q = 0; q < 6; ++q) pa[q] = y[q];
      act_inv_j(M, jt, s, c, pL, y);
      const double lj = rt >= 0 ? lam[rt + iv - 6] : 0.0;
      for (int q = 0; q < 3; ++q) y[3 + q] += ax[q] * lj;
      for (int q = 0; q < 6; ++q) pL[q] = y[q];
    }
    // ---- reverse: adjoints (d phi / d state and their d / dx_j) from the last joint to the root
    Dual vb[6], ab[6], Lb[6], cfb[3], cgb[3];
    for (int q = 0; q < 6; ++q) vb[q] = ab[q] = Lb[q] = Dual(0.0);
    for (int q = 0; q < 3; ++q) cfb[q] = cgb[q] = Dual(0.0);
    for (int kk = L - 1; kk >= 0; --kk) {
      const int jt = first + kk;
      const double* ax = M.axis[jt];
      const int iv = M.idx_v[jt];
      Dual s, c;
      sincos_s(qrev(M.idx_q[jt]), &s, &c);
      const Dual qd = vel[iv];
      const double lj = rt >= 0 ? lam[rt + iv - 6] : 0.0;
      // body jt: phi += L_j . f_j (+ its frame), f_j = body_wrench(a_j, v_j) - [cf; p x cf]
      {
        Dual fj[6], fb[6];
        body_wrench(M.mass[jt], M.lever[jt], M.Ic[jt], pa, pv, fj);
        for (int q = 0; q < 6; ++q) fb[q] = pL[q];
        if (jt == ej) {
          const double* pe = ef < O.nfeet ? O.feet[ef].p : O.ext.p;
          Dual t[3];
          for (int q = 0; q < 3; ++q) fj[q] -= cf[q];
          crossd(pe, cf, t);
          for (int q = 0; q < 3; ++q) fj[3 + q] -= t[q];
          crossd(pe, fb + 3, t);  // cf enters as -[cf; p x cf]: cfbar += -fb_l + p x fb_a
          for (int q = 0; q < 3; ++q) cfb[q] += t[q] - fb[q];
          if (has_mu) {  // phi += (v_l - p x w) . cg
            Dual u[3];
            crossd(pe, cg, u);
            crossd(pe, pv + 3, t);
            for (int q = 0; q < 3; ++q) {
              vb[q] += cg[q];
              vb[3 + q] += u[q];
              cgb[q] += pv[q] - t[q];
            }
          }
        }
        for (int q = 0; q < 6; ++q) Lb[q] += fj[q];
        body_wrench_adj(M.mass[jt], M.lever[jt], M.Ic[jt], pv, fb, ab, vb);
      }
      Dual thb(0.0), qdb(0.0), y[6], t[3], nb[6];
      // a_j = act_inv(a_in) + [-(ax x v_l) qd; ax a_iv - (ax x w) qd]  (v = v_j)
      crossd(ax, pv, t);
      for (int q = 0; q < 3; ++q) y[q] = pa[q] + t[q] * qd;
      qdb -= ab[0] * t[0] + ab[1] * t[1] + ab[2] * t[2];
      crossd(ax, pv + 3, t);
      for (int q = 0; q < 3; ++q) y[3 + q] = pa[3 + q] - ax[q] * a[iv] + t[q] * qd;
      qdb -= ab[3] * t[0] + ab[4] * t[1] + ab[5] * t[2];
      crossd(ax, ab, t);
      for (int q = 0; q < 3; ++q) vb[q] += qd * t[q];
      crossd(ax, ab + 3, t);
      for (int q = 0; q < 3; ++q) vb[3 + q] += qd * t[q];
      thb += ang_adj(ax, y, ab) + ang_adj(ax, y + 3, ab + 3);
      act_j(M, jt, s, c, y, pa);
      act_inv_adj(M, jt, s, c, ab, nb);
      for (int q = 0; q < 6; ++q) ab[q] = nb[q];
      // v_j = act_inv(v_in) + [0; ax qd]
      qdb += vb[3] * ax[0] + vb[4] * ax[1] + vb[5] * ax[2];
      for (int q = 0; q < 3; ++q) { y[q] = pv[q]; y[3 + q] = pv[3 + q] - ax[q] * qd; }
      thb += ang_adj(ax, y, vb) + ang_adj(ax, y + 3, vb + 3);
      act_j(M, jt, s, c, y, pv);
      act_inv_adj(M, jt, s, c, vb, nb);
      for (int q = 0; q < 6; ++q) vb[q] = nb[q];
      // L_j = act_inv(L_in) + [0; ax lj]
      for (int q = 0; q < 3; ++q) { y[q] = pL[q]; y[3 + q] = pL[3 + q] - ax[q] * lj; }
      thb += ang_adj(ax, y, Lb) + ang_adj(ax, y + 3, Lb + 3);
      act_j(M, jt, s, c, y, pL);
      act_inv_adj(M, jt, s, c, Lb, nb);
      for (int q = 0; q < 6; ++q) Lb[q] = nb[q];
      // the frame's force and multipliers rotated into the body axes: cf_j = R_j^T cf_in
      if (ef >= 0 && jt <= ej) {
        thb += ang_adj(ax, cf, cfb) + ang_adj(ax, cg, cgb);
        rot_j(M, jt, s, c, cf, t);
        for (int q = 0; q < 3; ++q) cf[q] = t[q];
        rot_j(M, jt, s, c, cg, t);
        for (int q = 0; q < 3; ++q) cg[q] = t[q];
        rot_j(M, jt, s, c, cfb, t);
        for (int q = 0; q < 3; ++q) cfb[q] = t[q];
        rot_j(M, jt, s, c, cgb, t);
        for (int q = 0; q < 3; ++q) cgb[q] = t[q];
      }
      if (!WHOLE) {
        if (mask >> (12 + kk) & 1u) write(iv, thb.d);            // dq of joint jt
        if (mask >> (12 + L + kk) & 1u) write(nv + iv, qdb.d);   // dv of joint jt
      }
    }
    // the chain's root state: v_0 = vel (base), a_0 = R0^T mg + a, cf_0 = R0^T f, cg_0 = R0^T mu
    for (int q = 0; q < 6; ++q) v0b[q] += vb[q];
    if constexpr (WHOLE)
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) R0b[3 * r + c] += mg[r] * ab[c] + fw[r] * cfb[c] + mu[r] * cgb[c];
  }
  for (int c = 0; c < 6; ++c)
    if (mask >> (6 + c) & 1u) write(nv + c, v0b[c].d);
  if constexpr (!WHOLE) return;
  for (int k = 3; k < 6; ++k) {  // the base rotation (whole-tree columns)
    if (!(mask >> k & 1u)) continue;
    const VecIn<HDual> hx{x, nullptr, 0.0, j, k};
    HDual qh[7], Rh[9];
    base_pose(xi, hx, qh);
    pl::quat_to_R(qh + 3, Rh);
    double acc = 0.0;
    for (int q = 0; q < 9; ++q) acc += R0b[q].d * Rh[q].b + R0b[q].v * Rh[q].c;
    write(k, acc);
  }
}

}  // namespace hess
