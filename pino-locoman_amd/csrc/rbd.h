// Rigid-body kernels (host+device, templated on the scalar: double or Dual).
//
// Restates the Pinocchio routines the reference calls through pinocchio.casadi:
//  * integrate / difference on the free-flyer Lie group
//    (dynamics_whole_body_torque.py:11-40; pinocchio SE3 LieGroup integrate_impl:
//    M0 * exp6(v), matrix->quaternion, hemisphere alignment, first-order renorm);
//  * RNEA with contact wrenches mapped to joint-local f_ext
//    (dynamics_whole_body_torque.py:42-71, dynamics/dynamics.py:33-65);
//  * frame velocities in LOCAL_WORLD_ALIGNED, optionally relative to the base
//    (dynamics/dynamics.py:77-118);
//  * ABA with the same f_ext (dynamics_whole_body_torque.py:73-103).
//
// The RNEA walks the tree chain by chain in the WORLD frame: each body's force is
// pushed to world coordinates as soon as it is computed, and a joint's torque is
// S_w^T (F_chain_total - prefix_before_joint).  Only three scalars per chain body
// (prefix projection, sin, cos) stay live across the chain, which keeps the
// dual-number Jacobian kernel in registers.
#pragma once
#include <type_traits>

#include "ad.h"
#include "model.h"

namespace pl {

template <class S> PL_HD void cross3(const S* a, const S* b, S* o) {
  S x = a[1] * b[2] - a[2] * b[1];
  S y = a[2] * b[0] - a[0] * b[2];
  S z = a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z;
}
template <class S> PL_HD S dot3(const S* a, const S* b) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
template <class S, class T, class X> PL_HD void matvec(const T* R, const X* x, S* o) {   // o = R x
  S a = R[0] * x[0] + R[1] * x[1] + R[2] * x[2];
  S b = R[3] * x[0] + R[4] * x[1] + R[5] * x[2];
  S c = R[6] * x[0] + R[7] * x[1] + R[8] * x[2];
  o[0] = a; o[1] = b; o[2] = c;
}
template <class S, class T, class X> PL_HD void mattvec(const T* R, const X* x, S* o) {  // o = R^T x
  S a = R[0] * x[0] + R[3] * x[1] + R[6] * x[2];
  S b = R[1] * x[0] + R[4] * x[1] + R[7] * x[2];
  S c = R[2] * x[0] + R[5] * x[1] + R[8] * x[2];
  o[0] = a; o[1] = b; o[2] = c;
}
template <class S, class T, class U> PL_HD void matmul3(const T* A, const U* B, S* C) {  // C = A B
  S t[9];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c)
      t[3 * r + c] = A[3 * r] * B[c] + A[3 * r + 1] * B[3 + c] + A[3 * r + 2] * B[6 + c];
  for (int k = 0; k < 9; ++k) C[k] = t[k];
}

// ---------------------------------------------------------------- quaternions / SE3
template <class S> PL_HD void quat_to_R(const S* qv, S* R) {  // Eigen toRotationMatrix, q = [x y z w]
  S tx = 2.0 * qv[0], ty = 2.0 * qv[1], tz = 2.0 * qv[2];
  S twx = tx * qv[3], twy = ty * qv[3], twz = tz * qv[3];
  S txx = tx * qv[0], txy = ty * qv[0], txz = tz * qv[0];
  S tyy = ty * qv[1], tyz = tz * qv[1], tzz = tz * qv[2];
  R[0] = 1.0 - (tyy + tzz); R[1] = txy - twz; R[2] = txz + twy;
  R[3] = txy + twz; R[4] = 1.0 - (txx + tzz); R[5] = tyz - twx;
  R[6] = txz - twy; R[7] = tyz + twx; R[8] = 1.0 - (txx + tyy);
}

// trace <= 0 branch for the largest diagonal entry I (compile-time indices: a run-time
// index into R / q would put both arrays in scratch)
template <int I, class S> PL_HD void R_to_quat_diag(const S* R, S* q) {
  constexpr int J = (I + 1) % 3, K = (J + 1) % 3;
  S s = sqrt_s(R[4 * I] - R[4 * J] - R[4 * K] + 1.0);
  q[I] = 0.5 * s;
  S inv = 0.5 / s;
  q[3] = (R[3 * K + J] - R[3 * J + K]) * inv;
  q[J] = (R[3 * J + I] + R[3 * I + J]) * inv;
  q[K] = (R[3 * K + I] + R[3 * I + K]) * inv;
}

template <class S> PL_HD void R_to_quat(const S* R, S* q) {  // Eigen quaternionbase_assign_impl
  // every branch fills its own local quaternion; one store per component at the end
  // (stores from several branches into q kept its tangents in scratch)
  S o[4];
  S t = R[0] + R[4] + R[8];
  if (val(t) > 0.0) {
    S s = sqrt_s(t + 1.0);
    o[3] = 0.5 * s;
    S inv = 0.5 / s;
    o[0] = (R[7] - R[5]) * inv;
    o[1] = (R[2] - R[6]) * inv;
    o[2] = (R[3] - R[1]) * inv;
  } else {
    int i = 0;
    if (val(R[4]) > val(R[0])) i = 1;
    if (val(R[8]) > val(R[4 * i])) i = 2;
    if (i == 0) R_to_quat_diag<0>(R, o);
    else if (i == 1) R_to_quat_diag<1>(R, o);
    else R_to_quat_diag<2>(R, o);
  }
  for (int k = 0; k < 4; ++k) q[k] = o[k];
}

#define PL_TAYLOR_PREC3 1.2207031250000000e-04  // eps^(1/4), pinocchio TaylorSeriesExpansion<double>::precision<3>()

// pinocchio exp6: R, t of the SE3 exponential of nu = [v; w]
template <class S> PL_HD void exp6(const S* nu, S* R, S* t) {
  const S* v = nu;
  const S* w = nu + 3;
  S t2 = w[0] * w[0] + w[1] * w[1] + w[2] * w[2];
  S a_wxv, a_v, a_w, diag;
  if (val(t2) < PL_TAYLOR_PREC3 * PL_TAYLOR_PREC3) {
    a_wxv = 0.5 - t2 / 24.0;
    a_v = 1.0 - t2 / 6.0;
    a_w = 1.0 / 6.0 - t2 / 120.0;
    diag = 1.0 - t2 / 2.0;
  } else {
    S th = sqrt_s(t2);
    S st, ct;
    sincos_s(th, &st, &ct);
    S inv_t2 = 1.0 / t2;
    a_wxv = (1.0 - ct) * inv_t2;
    a_v = st / th;
    a_w = (1.0 - a_v) * inv_t2;
    diag = ct;
  }
  S wxv[3];
  cross3(w, v, wxv);
  S wv = dot3(w, v);
  for (int k = 0; k < 3; ++k) t[k] = a_v * v[k] + (a_w * wv) * w[k] + a_wxv * wxv[k];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) R[3 * r + c] = a_wxv * w[r] * w[c];
  R[1] -= a_v * w[2]; R[3] += a_v * w[2];
  R[2] += a_v * w[1]; R[6] -= a_v * w[1];
  R[5] -= a_v * w[0]; R[7] += a_v * w[0];
  R[0] += diag; R[4] += diag; R[8] += diag;
}

// Free-flyer integrate (pinocchio SE3 LieGroup integrate_impl); q0 is a plain
// double configuration (x_init), dq the tangent (may be dual).
template <class S, class In> PL_HD void integrate_ff(const double* q0, const In& dq, S* qout) {
  double R0[9];
  quat_to_R(q0 + 3, R0);
  S Rx[9], tx[3];
  S nu[6];
  for (int k = 0; k < 6; ++k) nu[k] = dq[k];
  exp6(nu, Rx, tx);
  S R1[9];
  matmul3(R0, Rx, R1);
  S p1[3];
  matvec(R0, tx, p1);
  for (int k = 0; k < 3; ++k) qout[k] = q0[k] + p1[k];
  S qu[4];
  R_to_quat(R1, qu);
  double dot = val(qu[0]) * q0[3] + val(qu[1]) * q0[4] + val(qu[2]) * q0[5] + val(qu[3]) * q0[6];
  if (dot < 0.0)
    for (int k = 0; k < 4; ++k) qu[k] = -qu[k];
  S n2 = qu[0] * qu[0] + qu[1] * qu[1] + qu[2] * qu[2] + qu[3] * qu[3];
  S alpha = (3.0 - n2) / 2.0;
  for (int k = 0; k < 4; ++k) qout[3 + k] = qu[k] * alpha;
}

// pinocchio::integrate for free-flyer root + revolute joints.
template <class S, class In> PL_HD void integrate_q(const PlModel& M, const double* q0, const In& dq, S* q) {
  integrate_ff<S>(q0, dq, q);
  for (int j = 2; j < M.njoints; ++j) q[M.idx_q[j]] = q0[M.idx_q[j]] + dq[M.idx_v[j]];
}

// Revolute joint rotation R = jR * Rot(axis, theta), given sin/cos.
template <class S> PL_HD void rev_rot(const PlModel& M, int j, const S& s, const S& c, S* R) {
  const double* A = M.jR[j];
  switch (M.axis_kind[j]) {
    case PL_AX_X:
      for (int r = 0; r < 3; ++r) {
        R[3 * r + 0] = S(A[3 * r + 0]);
        R[3 * r + 1] = A[3 * r + 1] * c + A[3 * r + 2] * s;
        R[3 * r + 2] = A[3 * r + 2] * c - A[3 * r + 1] * s;
      }
      break;
    case PL_AX_Y:
      for (int r = 0; r < 3; ++r) {
        R[3 * r + 0] = A[3 * r + 0] * c - A[3 * r + 2] * s;
        R[3 * r + 1] = S(A[3 * r + 1]);
        R[3 * r + 2] = A[3 * r + 0] * s + A[3 * r + 2] * c;
      }
      break;
    case PL_AX_Z:
      for (int r = 0; r < 3; ++r) {
        R[3 * r + 0] = A[3 * r + 0] * c + A[3 * r + 1] * s;
        R[3 * r + 1] = A[3 * r + 1] * c - A[3 * r + 0] * s;
        R[3 * r + 2] = S(A[3 * r + 2]);
      }
      break;
    default: {
      const double* a = M.axis[j];
      S K[9];
      S oc = 1.0 - c;
      S Rr[9];
      // Rodrigues: I + s [a]x + (1-c) [a]x^2
      double ax[9] = {0, -a[2], a[1], a[2], 0, -a[0], -a[1], a[0], 0};
      for (int r = 0; r < 3; ++r)
        for (int cc = 0; cc < 3; ++cc) {
          double kk = ax[3 * r] * ax[cc] + ax[3 * r + 1] * ax[3 + cc] + ax[3 * r + 2] * ax[6 + cc];
          K[3 * r + cc] = s * ax[3 * r + cc] + oc * kk;
          Rr[3 * r + cc] = K[3 * r + cc] + (r == cc ? 1.0 : 0.0);
        }
      matmul3(A, Rr, R);
    }
  }
}

// Spatial helpers (Motion [v; w], Force [f; n]).
// actInv of a motion: out = [R^T (v - p x w); R^T w]
template <class S, class T, class U> PL_HD void act_inv_motion(const T* R, const U* p, const S* m, S* out) {
  S pxw[3];
  S pp[3] = {S(p[0]), S(p[1]), S(p[2])};
  cross3(pp, m + 3, pxw);
  S d[3] = {m[0] - pxw[0], m[1] - pxw[1], m[2] - pxw[2]};
  S o1[3], o2[3];
  mattvec(R, d, o1);
  mattvec(R, m + 3, o2);
  for (int k = 0; k < 3; ++k) { out[k] = o1[k]; out[3 + k] = o2[k]; }
}
// act of a force: out = [R f; R n + p x (R f)]
template <class S, class T, class U> PL_HD void act_force(const T* R, const U* p, const S* f, S* out) {
  S fl[3], nl[3];
  matvec(R, f, fl);
  matvec(R, f + 3, nl);
  S pp[3] = {S(p[0]), S(p[1]), S(p[2])};
  S pxf[3];
  cross3(pp, fl, pxf);
  for (int k = 0; k < 3; ++k) { out[k] = fl[k]; out[3 + k] = nl[k] + pxf[k]; }
}
// Y * v for inertia (m, c, Ic)
template <class S> PL_HD void inertia_mul(double m, const double* c, const double* Ic, const S* v, S* out) {
  S cc[3] = {S(c[0]), S(c[1]), S(c[2])};
  S cxw[3];
  cross3(cc, v + 3, cxw);
  S fl[3] = {m * (v[0] - cxw[0]), m * (v[1] - cxw[1]), m * (v[2] - cxw[2])};
  S Iw[3];
  matvec(Ic, v + 3, Iw);
  S cxf[3];
  cross3(cc, fl, cxf);
  for (int k = 0; k < 3; ++k) { out[k] = fl[k]; out[3 + k] = Iw[k] + cxf[k]; }
}
// v x* f (motion cross force)
template <class S> PL_HD void motion_cross_force(const S* v, const S* f, S* out) {
  S a[3], b[3], c[3];
  cross3(v + 3, f, a);
  cross3(v + 3, f + 3, b);
  cross3(v, f, c);
  for (int k = 0; k < 3; ++k) { out[k] = a[k]; out[3 + k] = b[k] + c[k]; }
}

// Per-node kinematic/dynamic outputs requested by the row function.  The arrays
// the rows index at run time (joint torques, foot velocities) live in caller
// storage (LDS on the device, interleaved with a stride), so no thread keeps a
// dynamically indexed register array (which the compiler would put in scratch).
#define PL_KIN_STORE (PL_MAXV - 6 + 3 * PL_MAXFEET + 7 * PL_MAXCL)  // entries of a NodeKin store
#define PL_KIN_STORE_DUAL PL_KIN_STORE
#ifndef PL_CHAIN_UNROLL
#define PL_CHAIN_UNROLL 1  // chain loops of tree_pass: rolled (register pressure of the dual pass)
#endif
template <class S> struct NodeKin {
  S tau[6];    // RNEA base torques (if want_tau)
  S arm_vel[3];  // relative arm velocity rows (ocp.py:177-179)
  S* store;    // [PL_KIN_STORE] x stride: joint torques, foot velocities, chain scratch
  int stride;
  PL_HD S& tau_j(int k) { return store[k * stride]; }                          // tau[6 + k]
  PL_HD S& foot_vel(int e, int c) { return store[(PL_MAXV - 6 + 3 * e + c) * stride]; }  // LWA lin. vel.
  // per joint of the current chain: world motion subspace S_w (6) and S_w . prefix
  PL_HD S& sw(int kk, int c) { return store[(PL_MAXV - 6 + 3 * PL_MAXFEET + 7 * kk + c) * stride]; }
  PL_HD S& alpha(int kk) { return store[(PL_MAXV - 6 + 3 * PL_MAXFEET + 7 * kk + 6) * stride]; }
  PL_HD void clear(int k) { store[k * stride] = S(0.0); }
};

// Dual-number store with the value and the tangent of an entry at separate addresses.
// The Jacobian kernel's 64 lanes evaluate the same primal (one tangent each), so the
// values go to one shared slot per entry (every writing lane stores identical bits)
// and only the tangents are per lane: half the LDS of an interleaved Dual store,
// which lets two single-wave workgroups share a SIMD.  The plain C++ callers point
// both at an interleaved Dual array (vstride = dstride = 2 x stride).
struct DualRef {
  double* v;
  double* d;
  PL_HD operator Dual() const { return Dual(*v, *d); }
  PL_HD DualRef& operator=(const Dual& x) {
    *v = x.v;
    *d = x.d;
    return *this;
  }
};
template <> struct NodeKin<Dual> {
  Dual tau[6];
  Dual arm_vel[3];
  double* vst;  // values   [PL_KIN_STORE_DUAL] x vstride
  double* dst;  // tangents [PL_KIN_STORE_DUAL] x dstride
  int vstride, dstride;
  PL_HD DualRef at(int k) { return DualRef{vst + k * vstride, dst + k * dstride}; }
  PL_HD DualRef tau_j(int k) { return at(k); }
  PL_HD DualRef foot_vel(int e, int c) { return at(PL_MAXV - 6 + 3 * e + c); }
  PL_HD DualRef sw(int kk, int c) { return at(PL_MAXV - 6 + 3 * PL_MAXFEET + 7 * kk + c); }
  PL_HD DualRef alpha(int kk) { return at(PL_MAXV - 6 + 3 * PL_MAXFEET + 7 * kk + 6); }
  // a skipped tree pass: zero tangent (the shared value slot belongs to the lanes that ran it)
  PL_HD void clear(int k) { dst[k * dstride] = 0.0; }
};

// q / v accessors over x_init + dx (ocp_whole_body_rnea.py:173-181): the free-flyer
// part of q comes from integrate_ff, every revolute coordinate is x_init + dx.
template <class S, class In> struct RevQ {
  const double* q0;
  In dq;
  PL_HD S operator()(int k) const { return q0[k] + dq[k - 1]; }  // revolute q index k >= 7
};
template <class S, class In> struct VelAcc {
  const double* v0;
  In dv;
  PL_HD S operator[](int k) const { return v0[k] + dv[k]; }
};
template <class S> struct RevQArr {  // same interface over a full q array
  const S* q;
  PL_HD S operator()(int k) const { return q[k]; }
};

// One pass over the tree: RNEA with contact forces (world frame, point forces at
// the frames in `ee`) plus foot / arm frame velocities.
//   q, v, a: full configuration / velocity / acceleration (a unused if !want_tau)
//   forces: 3 * nee world-frame forces (FR, FL, RR, RL[, ee])
//   qb: free-flyer q[0..7); qrev(k): revolute coordinate q[k]; v[k]: velocity
// Composite-body sums of tree_pass (kComp): about the root origin p0, world axes,
//   comp[6..8]  = sum_j m_j (c_j - p0),
//   comp[9..14] = sum_j R_j I_c,j R_j^T + m_j (|r_j|^2 1 - r_j r_j^T)  (xx xy xz yy yz zz),
// and comp[0..5] = the total body wrench sum_j X_j^* f_j at the world origin (world
// axes; gravity enters through the base acceleration, contact forces subtracted).
template <class S>
PL_HD void comp_add(S* comp, double m, const double* lever, const double* Ic, const S* oR, const S* op, const S* p0) {
  S lw[3];
  matvec(oR, lever, lw);
  S r[3];
  for (int k = 0; k < 3; ++k) r[k] = op[k] + lw[k] - p0[k];
  for (int k = 0; k < 3; ++k) comp[6 + k] += m * r[k];
  S T[9];  // R Ic
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T[3 * i + j] = oR[3 * i] * Ic[j] + oR[3 * i + 1] * Ic[3 + j] + oR[3 * i + 2] * Ic[6 + j];
  const S rr = r[0] * r[0] + r[1] * r[1] + r[2] * r[2];
  constexpr int II[6] = {0, 0, 0, 1, 1, 2}, JJ[6] = {0, 1, 2, 1, 2, 2};
  for (int q = 0; q < 6; ++q) {
    const int i = II[q], j = JJ[q];
    S t = T[3 * i] * oR[3 * j] + T[3 * i + 1] * oR[3 * j + 1] + T[3 * i + 2] * oR[3 * j + 2];
    t = t - m * (r[i] * r[j]);
    if (i == j) t = t + m * rr;
    comp[9 + q] += t;
  }
}

template <class S, class QR, class VA, class InA, class InF, bool kComp = false>
PL_HD void tree_pass(const PlModel& M, const PlOcpConst& O, const S* qb, const QR& qrev, const VA& v, const InA& a,
                     const InF& forces, bool want_tau, bool want_vel, NodeKin<S>& out, S* comp = nullptr,
                     std::integral_constant<bool, kComp> = {}, int only_ch = -1) {
  // ---- root (free-flyer, joint 1)
  S R0[9];
  quat_to_R(qb + 3, R0);
  S p0[3] = {qb[0], qb[1], qb[2]};
  S v1[6], a1[6], f1[6];
  for (int k = 0; k < 6; ++k) v1[k] = v[k];
  if (want_tau) {
    // a_gf[1] = actInv(M0, -g) + a_base  (v x vJ = 0 for the root)
    S g0[6] = {S(-M.gravity[0]), S(-M.gravity[1]), S(-M.gravity[2]), S(0.0), S(0.0), S(0.0)};
    act_inv_motion(R0, p0, g0, a1);
    for (int k = 0; k < 6; ++k) a1[k] += a[k];
    S h[6], vxh[6];
    inertia_mul(M.mass[1], M.lever[1], M.Ic[1], a1, f1);
    inertia_mul(M.mass[1], M.lever[1], M.Ic[1], v1, h);
    motion_cross_force(v1, h, vxh);
    for (int k = 0; k < 6; ++k) f1[k] += vxh[k];
  }
  // contact forces on the root body (e.g. a payload frame on the trunk)
  for (int e = 0; e < O.nee; ++e) {
    const PlFrameRef& F = (e < O.nfeet) ? O.feet[e] : O.ext;
    if (F.joint != 1 || !want_tau) continue;
    S fw[3] = {forces[3 * e], forces[3 * e + 1], forces[3 * e + 2]};
    S fl[3];
    mattvec(R0, fw, fl);
    S pf[3] = {S(F.p[0]), S(F.p[1]), S(F.p[2])};
    S fa[3];
    cross3(pf, fl, fa);
    for (int k = 0; k < 3; ++k) { f1[k] -= fl[k]; f1[3 + k] -= fa[k]; }
  }
  if constexpr (kComp) {
    for (int k = 0; k < 15; ++k) comp[k] = S(0.0);
    comp_add(comp, M.mass[1], M.lever[1], M.Ic[1], R0, p0, p0);
  }
  // world-frame force accumulated from every chain (at world origin)
  S Fw[6];
  for (int k = 0; k < 6; ++k) Fw[k] = S(0.0);
  // arm frame world data (for the relative velocity)
  S arm_lin[3], arm_pos[3];
  bool arm_skipped = false;  // the arm's chain skipped (only_ch): its velocity rows are zero

  for (int ch = 0; ch < M.nchains; ++ch) {
    const int first = M.chain_first[ch];
    const int L = M.chain_len[ch];
    if (only_ch >= 0 && ch != only_ch) {
      // only_ch: the caller differentiates along coordinates of chain only_ch (and of the
      // base) alone, so the other chains' outputs have zero tangents: they are skipped and
      // their outputs zeroed, values included (k_eval_jac_lin: the a / f columns at v = 0 and
      // zero gravity, where the other chains carry no acceleration and no force; k_lag_hess_pb:
      // a pair with a chain coordinate, whose mixed part only that chain's terms carry)
      if (want_tau)
        for (int kk = 0; kk < L; ++kk) out.tau_j(M.idx_v[first + kk] - 6) = S(0.0);
      if (want_vel) {
        for (int e = 0; e < O.nfeet; ++e)
          if (O.feet[e].joint >= first && O.feet[e].joint < first + L)
            for (int c = 0; c < 3; ++c) out.foot_vel(e, c) = S(0.0);
        if (O.arm.valid && O.arm.joint >= first && O.arm.joint < first + L) {
          arm_skipped = true;
          for (int k = 0; k < 3; ++k) {
            arm_lin[k] = S(0.0);
            arm_pos[k] = S(0.0);
          }
        }
      }
      continue;
    }
    S pv[6], pa[6], oR[9], op[3];
    for (int k = 0; k < 6; ++k) { pv[k] = v1[k]; if (want_tau) pa[k] = a1[k]; }
    for (int k = 0; k < 9; ++k) oR[k] = R0[k];
    for (int k = 0; k < 3; ++k) op[k] = p0[k];
    S P[6];
    for (int k = 0; k < 6; ++k) P[k] = S(0.0);
    // chain scratch (S_w, S_w . prefix per joint) in the NodeKin store (LDS on the
    // device; for the dual numbers only the tangents are per lane)
    auto SW = [&](int kk, int c) -> decltype(auto) { return out.sw(kk, c); };
    auto AL = [&](int kk) -> decltype(auto) { return out.alpha(kk); };
#pragma unroll PL_CHAIN_UNROLL
    for (int kk = 0; kk < PL_MAXCL; ++kk) {
      if (kk >= L) break;
      const int j = first + kk;
      S qj = qrev(M.idx_q[j]);
      S s, c;
      sincos_s(qj, &s, &c);
      S Rl[9];
      rev_rot(M, j, s, c, Rl);
      const double* pl = M.jp[j];
      S vj[6];
      act_inv_motion(Rl, pl, pv, vj);
      S qd = v[M.idx_v[j]];
      const double* ax = M.axis[j];
      S vJ[6] = {S(0.0), S(0.0), S(0.0), ax[0] * qd, ax[1] * qd, ax[2] * qd};
      for (int k = 0; k < 3; ++k) vj[3 + k] += vJ[3 + k];
      // world pose of body j
      S oRj[9], opj[3], tmp3[3];
      matmul3(oR, Rl, oRj);
      matvec(oR, pl, tmp3);
      for (int k = 0; k < 3; ++k) opj[k] = op[k] + tmp3[k];
      if constexpr (kComp) comp_add(comp, M.mass[j], M.lever[j], M.Ic[j], oRj, opj, p0);
      if (want_tau) {
        S aj[6];
        act_inv_motion(Rl, pl, pa, aj);
        S qdd = a[M.idx_v[j]];
        // + S qdd + v x vJ   (c_J = 0 for revolute joints)
        S vxvJ[6];
        {
          // motion cross: [w x vJ_lin + v x vJ_ang ; w x vJ_ang], vJ_lin = 0
          S t1[3], t2[3];
          cross3(vj, vJ + 3, t1);
          cross3(vj + 3, vJ + 3, t2);
          for (int k = 0; k < 3; ++k) { vxvJ[k] = t1[k]; vxvJ[3 + k] = t2[k]; }
        }
        for (int k = 0; k < 3; ++k) { aj[k] += vxvJ[k]; aj[3 + k] += ax[k] * qdd + vxvJ[3 + k]; }
        S fj[6], h[6], vxh[6];
        inertia_mul(M.mass[j], M.lever[j], M.Ic[j], aj, fj);
        inertia_mul(M.mass[j], M.lever[j], M.Ic[j], vj, h);
        motion_cross_force(vj, h, vxh);
        for (int k = 0; k < 6; ++k) fj[k] += vxh[k];
        for (int e = 0; e < O.nee; ++e) {
          const PlFrameRef& F = (e < O.nfeet) ? O.feet[e] : O.ext;
          if (F.joint != j) continue;
          // f_lin = R_wj^T f_world; f_ang = p_frame x f_lin (joint-local)
          S fw[3] = {forces[3 * e], forces[3 * e + 1], forces[3 * e + 2]};
          S fl[3];
          mattvec(oRj, fw, fl);
          S pf[3] = {S(F.p[0]), S(F.p[1]), S(F.p[2])};
          S fa[3];
          cross3(pf, fl, fa);
          for (int k = 0; k < 3; ++k) { fj[k] -= fl[k]; fj[3 + k] -= fa[k]; }
        }
        // body force in world coordinates (at world origin)
        S fwj[6];
        act_force(oRj, opj, fj, fwj);
        // joint motion subspace in world coordinates: [op x w_ax; w_ax]
        S wax[3];
        matvec(oRj, ax, wax);
        S lax[3];
        cross3(opj, wax, lax);
        for (int k = 0; k < 3; ++k) { SW(kk, k) = lax[k]; SW(kk, 3 + k) = wax[k]; }
        AL(kk) = lax[0] * P[0] + lax[1] * P[1] + lax[2] * P[2] + wax[0] * P[3] + wax[1] * P[4] + wax[2] * P[5];
        for (int k = 0; k < 6; ++k) P[k] += fwj[k];
        for (int k = 0; k < 6; ++k) pa[k] = aj[k];
      }
      if (want_vel) {
        for (int e = 0; e < O.nfeet; ++e) {
          if (O.feet[e].joint != j) continue;
          S wxp[3];
          S pf[3] = {S(O.feet[e].p[0]), S(O.feet[e].p[1]), S(O.feet[e].p[2])};
          cross3(vj + 3, pf, wxp);
          S lv[3] = {vj[0] + wxp[0], vj[1] + wxp[1], vj[2] + wxp[2]};
          S fvw[3];
          matvec(oRj, lv, fvw);
          for (int k = 0; k < 3; ++k) out.foot_vel(e, k) = fvw[k];
        }
        if (O.arm.valid && O.arm.joint == j) {
          S wxp[3];
          S pf[3] = {S(O.arm.p[0]), S(O.arm.p[1]), S(O.arm.p[2])};
          cross3(vj + 3, pf, wxp);
          S lv[3] = {vj[0] + wxp[0], vj[1] + wxp[1], vj[2] + wxp[2]};
          matvec(oRj, lv, arm_lin);
          S t[3];
          matvec(oRj, pf, t);
          for (int k = 0; k < 3; ++k) arm_pos[k] = opj[k] + t[k];
        }
      }
      for (int k = 0; k < 6; ++k) pv[k] = vj[k];
      for (int k = 0; k < 9; ++k) oR[k] = oRj[k];
      for (int k = 0; k < 3; ++k) op[k] = opj[k];
    }
    if (want_tau) {
      // tau_j = S_w^T (F_total - prefix_before_j)
#pragma unroll PL_CHAIN_UNROLL
      for (int kk = 0; kk < PL_MAXCL; ++kk) {
        if (kk >= L) break;
        const int j = first + kk;
        S t = SW(kk, 0) * P[0] + SW(kk, 1) * P[1] + SW(kk, 2) * P[2] + SW(kk, 3) * P[3] + SW(kk, 4) * P[4] +
              SW(kk, 5) * P[5];
        out.tau_j(M.idx_v[j] - 6) = t - AL(kk);
      }
      for (int k = 0; k < 6; ++k) Fw[k] += P[k];
    }
  }
  if (want_tau) {
    if constexpr (kComp) {  // total wrench at the world origin: chains + the root body's own
      S f1w[6];
      act_force(R0, p0, f1, f1w);
      for (int k = 0; k < 6; ++k) comp[k] = Fw[k] + f1w[k];
    }
    // root: f1 += actInv_force(M0, Fw)  (world -> root-local)
    S d[3], pxf[3];
    cross3(p0, Fw, pxf);
    for (int k = 0; k < 3; ++k) d[k] = Fw[3 + k] - pxf[k];
    S fl[3], nl[3];
    mattvec(R0, Fw, fl);
    mattvec(R0, d, nl);
    for (int k = 0; k < 3; ++k) { out.tau[k] = f1[k] + fl[k]; out.tau[3 + k] = f1[3 + k] + nl[k]; }
  }
  if (want_vel && O.arm.valid && arm_skipped) {
    // a pass confined to another chain: the arm rows have zero tangents, value and all (as the
    // skipped chains' other outputs above), not the base-only remainder of the formula below
    for (int k = 0; k < 3; ++k) out.arm_vel[k] = S(0.0);
  } else if (want_vel && O.arm.valid) {
    // Dynamics.get_frame_velocity(relative_to_base=True) (dynamics/dynamics.py:86-113)
    // base frame on the root joint: LWA velocity = R0 (v + w x p_b), angular R0 w
    S pb[3] = {S(O.base.p[0]), S(O.base.p[1]), S(O.base.p[2])};
    S wxp[3];
    cross3(v1 + 3, pb, wxp);
    S lvb[3] = {v1[0] + wxp[0], v1[1] + wxp[1], v1[2] + wxp[2]};
    S bl[3], ba[3];
    matvec(R0, lvb, bl);
    matvec(R0, v1 + 3, ba);
    S Rb[9];
    matmul3(R0, O.base.R, Rb);
    S t[3], bpos[3];
    matvec(R0, pb, t);
    for (int k = 0; k < 3; ++k) bpos[k] = p0[k] + t[k];
    S rel[3] = {arm_pos[0] - bpos[0], arm_pos[1] - bpos[1], arm_pos[2] - bpos[2]};
    S corr[3];
    cross3(ba, rel, corr);
    S rl[3] = {arm_lin[0] - bl[0] - corr[0], arm_lin[1] - bl[1] - corr[1], arm_lin[2] - bl[2] - corr[2]};
    S rlb[3];
    mattvec(Rb, rl, rlb);
    out.arm_vel[0] = rlb[0];
    out.arm_vel[1] = rlb[1];
    out.arm_vel[2] = arm_lin[2];
  }
}

// ---------------------------------------------------------------- centroidal
// One pass over the tree for the centroidal model (DynamicsCentroidalVel,
// dynamics_centroidal_vel.py:43-71, 136-148):
//   hg   = A(q) v: pinocchio computeCentroidalMap applied to v, i.e. the total spatial
//          momentum sum_j X_j^* (I_j v_j) about the CoM in world axes (linear first);
//   hdot = com_dynamics(q, forces) = [sum_e f_e + (0, 0, -9.81 m), sum_e (p_e - com) x f_e] / m
//          over the contact frames FR, FL, RR, RL (+ the external-force frame).
// Bodies are pushed to world coordinates as they are visited (as in tree_pass), so
// only the running sums stay live.  want_h = false skips the velocity recursion.
// CI: also the CoM c -> cinfo[0, 3) and the composite rotational inertia about the CoM in
// world axes -> cinfo[3, 9) = (xx, xy, xz, yy, yz, zz), for the base-velocity solve (a
// compile-time switch, so the other instantiations compile exactly as without it).
template <class S, class QR, class VA, class InF, bool CI = false>
PL_HD void centroidal_pass(const PlModel& M, const PlOcpConst& O, const S* qb, const QR& qrev, const VA& v,
                           const InF& forces, bool want_h, bool want_hdot, S* hg, S* hdot,
                           S* cinfo = nullptr, std::integral_constant<bool, CI> = {}) {
  S R0[9];
  quat_to_R(qb + 3, R0);
  S p0[3] = {qb[0], qb[1], qb[2]};
  S mc[3], H[6], pe[PL_MAXFEET + 1][3], Io[CI ? 6 : 1];
  for (int k = 0; k < 3; ++k) mc[k] = S(0.0);
  if constexpr (CI)
    for (int k = 0; k < 6; ++k) Io[k] = S(0.0);
  for (int k = 0; k < 6; ++k) H[k] = S(0.0);
  for (int e = 0; e < PL_MAXFEET + 1; ++e)
    for (int k = 0; k < 3; ++k) pe[e][k] = S(0.0);
  // body j at world pose (oR, op) with local velocity vj: CoM moment, momentum, frames
  auto visit = [&](int j, const S* oR, const S* op, const S* vj) {
    S lc[3];
    matvec(oR, M.lever[j], lc);
    for (int k = 0; k < 3; ++k) mc[k] += M.mass[j] * (op[k] + lc[k]);
    if constexpr (CI) {  // inertia about the world origin: oR Ic oR^T + m (|p|^2 1 - p p^T)
      S T[9], Iw[9], pj[3];
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c)
          T[3 * r + c] = oR[3 * r] * M.Ic[j][c] + oR[3 * r + 1] * M.Ic[j][3 + c] + oR[3 * r + 2] * M.Ic[j][6 + c];
      for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) Iw[3 * r + c] = T[3 * r] * oR[3 * c] + T[3 * r + 1] * oR[3 * c + 1] + T[3 * r + 2] * oR[3 * c + 2];
      for (int k = 0; k < 3; ++k) pj[k] = op[k] + lc[k];
      const S pp = pj[0] * pj[0] + pj[1] * pj[1] + pj[2] * pj[2];
      const double mj = M.mass[j];
      Io[0] += Iw[0] + mj * (pp - pj[0] * pj[0]);
      Io[1] += Iw[1] - mj * pj[0] * pj[1];
      Io[2] += Iw[2] - mj * pj[0] * pj[2];
      Io[3] += Iw[4] + mj * (pp - pj[1] * pj[1]);
      Io[4] += Iw[5] - mj * pj[1] * pj[2];
      Io[5] += Iw[8] + mj * (pp - pj[2] * pj[2]);
    }
    if (want_h) {
      S hl[6], hw[6];
      inertia_mul(M.mass[j], M.lever[j], M.Ic[j], vj, hl);
      act_force(oR, op, hl, hw);
      for (int k = 0; k < 6; ++k) H[k] += hw[k];
    }
    if (want_hdot) {
#pragma unroll
      for (int e = 0; e < PL_MAXFEET + 1; ++e) {  // constant bound: pe stays in registers
        if (e >= O.nee) break;
        const PlFrameRef& F = (e < O.nfeet) ? O.feet[e] : O.ext;
        if (F.joint != j) continue;
        S t[3];
        matvec(oR, F.p, t);
        for (int k = 0; k < 3; ++k) pe[e][k] = op[k] + t[k];
      }
    }
  };
  S v1[6];
  for (int k = 0; k < 6; ++k) v1[k] = want_h ? S(v[k]) : S(0.0);
  visit(1, R0, p0, v1);
  for (int ch = 0; ch < M.nchains; ++ch) {
    const int first = M.chain_first[ch];
    const int L = M.chain_len[ch];
    S pv[6], oR[9], op[3];
    for (int k = 0; k < 6; ++k) pv[k] = v1[k];
    for (int k = 0; k < 9; ++k) oR[k] = R0[k];
    for (int k = 0; k < 3; ++k) op[k] = p0[k];
#pragma unroll
    for (int kk = 0; kk < PL_MAXCL; ++kk) {
      if (kk >= L) break;
      const int j = first + kk;
      S s, c;
      sincos_s(qrev(M.idx_q[j]), &s, &c);
      S Rl[9];
      rev_rot(M, j, s, c, Rl);
      const double* pl = M.jp[j];
      S vj[6];
      if (want_h) {
        act_inv_motion(Rl, pl, pv, vj);
        S qd = v[M.idx_v[j]];
        for (int k = 0; k < 3; ++k) vj[3 + k] += M.axis[j][k] * qd;
      }
      S oRj[9], t3[3];
      matmul3(oR, Rl, oRj);
      matvec(oR, pl, t3);
      for (int k = 0; k < 3; ++k) op[k] = op[k] + t3[k];
      for (int k = 0; k < 9; ++k) oR[k] = oRj[k];
      visit(j, oR, op, vj);
      if (want_h)
        for (int k = 0; k < 6; ++k) pv[k] = vj[k];
    }
  }
  const double m = M.total_mass;
  S com[3];
  for (int k = 0; k < 3; ++k) com[k] = mc[k] * (1.0 / m);
  if constexpr (CI) {  // parallel axis to the CoM: I_c = I_o - m (|c|^2 1 - c c^T)
    const S cc = com[0] * com[0] + com[1] * com[1] + com[2] * com[2];
    for (int k = 0; k < 3; ++k) cinfo[k] = com[k];
    cinfo[3] = Io[0] - m * (cc - com[0] * com[0]);
    cinfo[4] = Io[1] + m * com[0] * com[1];
    cinfo[5] = Io[2] + m * com[0] * com[2];
    cinfo[6] = Io[3] - m * (cc - com[1] * com[1]);
    cinfo[7] = Io[4] + m * com[1] * com[2];
    cinfo[8] = Io[5] - m * (cc - com[2] * com[2]);
  }
  if (want_h) {  // shift the angular momentum from the world origin to the CoM
    S cxl[3];
    cross3(com, H, cxl);
    for (int k = 0; k < 3; ++k) { hg[k] = H[k]; hg[3 + k] = H[3 + k] - cxl[k]; }
  }
  if (want_hdot) {
    S dp[3] = {S(0.0), S(0.0), S(-9.81 * m)}, dl[3] = {S(0.0), S(0.0), S(0.0)};
#pragma unroll
    for (int e = 0; e < PL_MAXFEET + 1; ++e) {
      if (e >= O.nee) break;
      S f[3] = {forces[3 * e], forces[3 * e + 1], forces[3 * e + 2]};
      S r[3] = {pe[e][0] - com[0], pe[e][1] - com[1], pe[e][2] - com[2]};
      S t[3];
      cross3(r, f, t);
      for (int k = 0; k < 3; ++k) { dp[k] += f[k]; dl[k] += t[k]; }
    }
    for (int k = 0; k < 3; ++k) { hdot[k] = dp[k] * (1.0 / m); hdot[3 + k] = dl[k] * (1.0 / m); }
  }
}

// base_vel_dynamics (dynamics_centroidal_vel.py:73-89): v_b = A_b^-1 (m h - A_j v_j).  A_b
// maps the local base twist to the momentum of the robot moving rigidly with the base:
// linear m (R0 v + w_w x (c - p0)), angular I_c w_w (w_w = R0 w).  hj = A_j v_j (the
// momentum at zero base velocity), ci = centroidal_pass's cinfo.
template <class S>
PL_HD void base_vel_solve(double m, const S* R0, const S* p0, const S* ci, const S* h, const S* hj, S* vb) {
  S b[6];
  for (int k = 0; k < 6; ++k) b[k] = m * h[k] - hj[k];
  const S* I = ci + 3;  // xx xy xz yy yz zz
  const S l00 = sqrt_s(I[0]);
  const S l10 = I[1] / l00, l20 = I[2] / l00;
  const S l11 = sqrt_s(I[3] - l10 * l10);
  const S l21 = (I[4] - l20 * l10) / l11;
  const S l22 = sqrt_s(I[5] - l20 * l20 - l21 * l21);
  const S y0 = b[3] / l00, y1 = (b[4] - l10 * y0) / l11, y2 = (b[5] - l20 * y0 - l21 * y1) / l22;
  const S w2 = y2 / l22, w1 = (y1 - l21 * w2) / l11, w0 = (y0 - l10 * w1 - l20 * w2) / l00;
  const S ww[3] = {w0, w1, w2};
  S d[3], wxd[3], lin[3];
  for (int k = 0; k < 3; ++k) d[k] = ci[k] - p0[k];
  cross3(ww, d, wxd);
  for (int k = 0; k < 3; ++k) lin[k] = b[k] * (1.0 / m) - wxd[k];
  mattvec(R0, lin, vb);
  mattvec(R0, ww, vb + 3);
}

// ---------------------------------------------------------------- base from the base rows
// The 6 base equations of the floating base, from tree_pass's composite sums:
//   M_bb = [[m 1, -[h]x], [[h]x, I]] in the root frame (h = R0^T sum m r, I = R0^T I_p0 R0);
//   base_solve: a_b = -M_bb^-1 tau_b (tau_b = RNEA base rows at a_b = 0), by the Schur
//   complement on the rotational block (the inertia about the CoM, 3x3 Cholesky).
template <class S>
PL_HD void base_solve(double m, const S* R0, const S* comp, const S* tau_b, S* a_b) {
  S h[3], Iw[9];
  mattvec(R0, comp + 6, h);
  const S* c = comp + 9;
  const S Ip[9] = {c[0], c[1], c[2], c[1], c[3], c[4], c[2], c[4], c[5]};
  // I = R0^T Ip R0
  S T[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T[3 * i + j] = R0[i] * Ip[j] + R0[3 + i] * Ip[3 + j] + R0[6 + i] * Ip[6 + j];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) Iw[3 * i + j] = T[3 * i] * R0[j] + T[3 * i + 1] * R0[3 + j] + T[3 * i + 2] * R0[6 + j];
  // Ic = I + (h h^T - |h|^2 1) / m ; rhs = -tau_ang + h x tau_lin / m
  const double im = 1.0 / m;
  const S hh = h[0] * h[0] + h[1] * h[1] + h[2] * h[2];
  S A[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) A[3 * i + j] = Iw[3 * i + j] + (h[i] * h[j] - (i == j ? hh : S(0.0))) * im;
  S hxt[3];
  cross3(h, tau_b, hxt);
  S r[3];
  for (int k = 0; k < 3; ++k) r[k] = hxt[k] * im - tau_b[3 + k];
  // Cholesky A = L L^T
  const S l00 = sqrt_s(A[0]);
  const S l10 = A[3] / l00, l20 = A[6] / l00;
  const S l11 = sqrt_s(A[4] - l10 * l10);
  const S l21 = (A[7] - l20 * l10) / l11;
  const S l22 = sqrt_s(A[8] - l20 * l20 - l21 * l21);
  const S y0 = r[0] / l00, y1 = (r[1] - l10 * y0) / l11, y2 = (r[2] - l20 * y0 - l21 * y1) / l22;
  const S w2 = y2 / l22, w1 = (y1 - l21 * w2) / l11, w0 = (y0 - l10 * w1 - l20 * w2) / l00;
  const S wa[3] = {w0, w1, w2};
  S hxw[3];
  cross3(h, wa, hxw);
  for (int k = 0; k < 3; ++k) {
    a_b[k] = (hxw[k] - tau_b[k]) * im;
    a_b[3 + k] = wa[k];
  }
}

// A a + dA v - dh(q, f) (DynamicsCentroidalAcc.dynamics_gaps): the total wrench of
// tree_pass moved from the world origin to the CoM, c = p0 + sum m r / m.
template <class S>
PL_HD void centroidal_gap(double m, const S* p0, const S* comp, S* gap) {
  S c[3];
  for (int k = 0; k < 3; ++k) c[k] = p0[k] + comp[6 + k] * (1.0 / m);
  S cxf[3];
  cross3(c, comp, cxf);
  for (int k = 0; k < 3; ++k) {
    gap[k] = comp[k];
    gap[3 + k] = comp[3 + k] - cxf[k];
  }
}

// ---------------------------------------------------------------- ABA
// pinocchio::aba(model, data, q, v, [0_6; tau_j], f_ext) (dynamics_whole_body_torque.py:73-103),
// articulated-body algorithm in local joint frames.  Generic per-body arrays
// (used by the whole_body_aba OCP only).
template <class S> PL_HD void inertia6(const PlModel& M, int j, S* Y) {
  const double m = M.mass[j];
  const double* c = M.lever[j];
  const double* I = M.Ic[j];
  double cx[9] = {0, -c[2], c[1], c[2], 0, -c[0], -c[1], c[0], 0};
  for (int r = 0; r < 6; ++r)
    for (int k = 0; k < 6; ++k) Y[6 * r + k] = S(0.0);
  for (int r = 0; r < 3; ++r) {
    Y[6 * r + r] = S(m);
    for (int k = 0; k < 3; ++k) {
      Y[6 * r + 3 + k] = S(-m * cx[3 * r + k]);
      Y[6 * (3 + r) + k] = S(m * cx[3 * r + k]);
      double cc = cx[3 * r] * cx[k] + cx[3 * r + 1] * cx[3 + k] + cx[3 * r + 2] * cx[6 + k];
      Y[6 * (3 + r) + 3 + k] = S(I[3 * r + k] - m * cc);
    }
  }
}

// Xm = 6x6 motion transform of actInv(R, p):  [[R^T, -R^T [p]x], [0, R^T]]
template <class S> PL_HD void actinv_matrix(const S* R, const S* p, S* X) {
  S px[9] = {S(0.0), -p[2], p[1], p[2], S(0.0), -p[0], -p[1], p[0], S(0.0)};
  for (int r = 0; r < 6; ++r)
    for (int k = 0; k < 6; ++k) X[6 * r + k] = S(0.0);
  for (int r = 0; r < 3; ++r)
    for (int k = 0; k < 3; ++k) {
      S rt = R[3 * k + r];
      X[6 * r + k] = rt;
      X[6 * (3 + r) + 3 + k] = rt;
      S acc = S(0.0);
      for (int l = 0; l < 3; ++l) acc += R[3 * l + r] * px[3 * l + k];
      X[6 * r + 3 + k] = -acc;
    }
}

template <class S, class InT, class InF>
PL_HD void aba_forward(const PlModel& M, const PlOcpConst& O, const S* q, const S* v, const InT& tau_j,
                       const InF& forces, S* ddq) {
  const int nb = M.njoints;
  S lR[PL_MAXJ][9], lp[PL_MAXJ][3], oR[PL_MAXJ][9];
  S vv[PL_MAXJ][6], cc[PL_MAXJ][6], pA[PL_MAXJ][6], Ia[PL_MAXJ][36];
  for (int j = 1; j < nb; ++j) {
    const int par = M.parent[j];
    S vJ[6];
    if (M.jtype[j] == PL_JT_FREEFLYER) {
      quat_to_R(q + M.idx_q[j] + 3, lR[j]);
      for (int k = 0; k < 3; ++k) lp[j][k] = q[M.idx_q[j] + k];
      for (int k = 0; k < 6; ++k) vJ[k] = v[M.idx_v[j] + k];
    } else {
      S s, c;
      sincos_s(q[M.idx_q[j]], &s, &c);
      rev_rot(M, j, s, c, lR[j]);
      for (int k = 0; k < 3; ++k) lp[j][k] = S(M.jp[j][k]);
      S qd = v[M.idx_v[j]];
      for (int k = 0; k < 3; ++k) { vJ[k] = S(0.0); vJ[3 + k] = M.axis[j][k] * qd; }
    }
    if (par == 0) {
      for (int k = 0; k < 9; ++k) oR[j][k] = lR[j][k];
      for (int k = 0; k < 6; ++k) vv[j][k] = vJ[k];
    } else {
      matmul3(oR[par], lR[j], oR[j]);
      act_inv_motion(lR[j], lp[j], vv[par], vv[j]);
      for (int k = 0; k < 6; ++k) vv[j][k] += vJ[k];
    }
    {
      S t1[3], t2[3], t3[3];
      cross3(vv[j] + 3, vJ, t1);
      cross3(vv[j], vJ + 3, t2);
      cross3(vv[j] + 3, vJ + 3, t3);
      for (int k = 0; k < 3; ++k) { cc[j][k] = t1[k] + t2[k]; cc[j][3 + k] = t3[k]; }
    }
    inertia6(M, j, Ia[j]);
    S h[6];
    inertia_mul(M.mass[j], M.lever[j], M.Ic[j], vv[j], h);
    motion_cross_force(vv[j], h, pA[j]);
    for (int e = 0; e < O.nee; ++e) {
      const PlFrameRef& F = (e < O.nfeet) ? O.feet[e] : O.ext;
      if (F.joint != j) continue;
      S fw[3] = {forces[3 * e], forces[3 * e + 1], forces[3 * e + 2]};
      S fl[3];
      mattvec(oR[j], fw, fl);
      S pf[3] = {S(F.p[0]), S(F.p[1]), S(F.p[2])};
      S fa[3];
      cross3(pf, fl, fa);
      for (int k = 0; k < 3; ++k) { pA[j][k] -= fl[k]; pA[j][3 + k] -= fa[k]; }
    }
  }
  S U[PL_MAXJ][6], Dinv[PL_MAXJ], uu[PL_MAXJ];
  S u_root[6];
  for (int j = nb - 1; j >= 1; --j) {
    const int par = M.parent[j];
    if (M.jtype[j] == PL_JT_FREEFLYER) {
      for (int k = 0; k < 6; ++k) u_root[k] = -pA[j][k];  // base torque = 0
      continue;                                           // root: parent is universe
    }
    const double* ax = M.axis[j];
    for (int r = 0; r < 6; ++r) U[j][r] = Ia[j][6 * r + 3] * ax[0] + Ia[j][6 * r + 4] * ax[1] + Ia[j][6 * r + 5] * ax[2];
    S D = U[j][3] * ax[0] + U[j][4] * ax[1] + U[j][5] * ax[2];
    Dinv[j] = 1.0 / D;
    uu[j] = tau_j[M.idx_v[j] - 6] - (pA[j][3] * ax[0] + pA[j][4] * ax[1] + pA[j][5] * ax[2]);
    if (par > 0) {
      S Iaa[36];
      for (int r = 0; r < 6; ++r)
        for (int k = 0; k < 6; ++k) Iaa[6 * r + k] = Ia[j][6 * r + k] - U[j][r] * Dinv[j] * U[j][k];
      S pa[6];
      S Udu = Dinv[j] * uu[j];
      for (int r = 0; r < 6; ++r) {
        S acc = pA[j][r] + U[j][r] * Udu;
        for (int k = 0; k < 6; ++k) acc += Iaa[6 * r + k] * cc[j][k];
        pa[r] = acc;
      }
      S X[36];
      actinv_matrix(lR[j], lp[j], X);
      // Ia[par] += X^T Iaa X
      S T[36];
      for (int r = 0; r < 6; ++r)
        for (int k = 0; k < 6; ++k) {
          S acc = S(0.0);
          for (int l = 0; l < 6; ++l) acc += Iaa[6 * r + l] * X[6 * l + k];
          T[6 * r + k] = acc;
        }
      for (int r = 0; r < 6; ++r)
        for (int k = 0; k < 6; ++k) {
          S acc = S(0.0);
          for (int l = 0; l < 6; ++l) acc += X[6 * l + r] * T[6 * l + k];
          Ia[par][6 * r + k] += acc;
        }
      S fo[6];
      act_force(lR[j], lp[j], pa, fo);
      for (int k = 0; k < 6; ++k) pA[par][k] += fo[k];
    }
  }
  // pass 3
  S acc_[PL_MAXJ][6];
  for (int j = 1; j < nb; ++j) {
    const int par = M.parent[j];
    S ai[6];
    if (par == 0) {
      S g0[6] = {S(-M.gravity[0]), S(-M.gravity[1]), S(-M.gravity[2]), S(0.0), S(0.0), S(0.0)};
      act_inv_motion(lR[j], lp[j], g0, ai);
    } else {
      act_inv_motion(lR[j], lp[j], acc_[par], ai);
    }
    for (int k = 0; k < 6; ++k) ai[k] += cc[j][k];
    if (M.jtype[j] == PL_JT_FREEFLYER) {
      // qdd = Ia^-1 (u - Ia a) ; solve 6x6 SPD by Gaussian elimination
      S A[36], b[6];
      for (int r = 0; r < 36; ++r) A[r] = Ia[j][r];
      for (int r = 0; r < 6; ++r) {
        S t = u_root[r];
        for (int k = 0; k < 6; ++k) t -= Ia[j][6 * r + k] * ai[k];
        b[r] = t;
      }
      for (int col = 0; col < 6; ++col) {
        S inv = 1.0 / A[6 * col + col];
        for (int r = col + 1; r < 6; ++r) {
          S f = A[6 * r + col] * inv;
          for (int k = col; k < 6; ++k) A[6 * r + k] -= f * A[6 * col + k];
          b[r] -= f * b[col];
        }
      }
      S x[6];
      for (int r = 5; r >= 0; --r) {
        S t = b[r];
        for (int k = r + 1; k < 6; ++k) t -= A[6 * r + k] * x[k];
        x[r] = t / A[6 * r + r];
      }
      for (int k = 0; k < 6; ++k) { ddq[M.idx_v[j] + k] = x[k]; acc_[j][k] = ai[k] + x[k]; }
    } else {
      const double* ax = M.axis[j];
      S Ua = U[j][0] * ai[0] + U[j][1] * ai[1] + U[j][2] * ai[2] + U[j][3] * ai[3] + U[j][4] * ai[4] + U[j][5] * ai[5];
      S qdd = Dinv[j] * (uu[j] - Ua);
      ddq[M.idx_v[j]] = qdd;
      for (int k = 0; k < 3; ++k) { acc_[j][k] = ai[k]; acc_[j][3 + k] = ai[3 + k] + ax[k] * qdd; }
    }
  }
}

// ---------------------------------------------------------------- difference (values only)
// pinocchio log3 / log6 and the free-flyer difference log6(M0^-1 M1)
// (used for dx_des = difference(x_init, x_des), ocp_whole_body_rnea.py:93-94).
PL_HD void log3_d(const double* R, double* w, double* theta_out) {
  double tr = R[0] + R[4] + R[8];
  double theta;
  if (tr >= 3.0) theta = 0.0;
  else if (tr <= -1.0) theta = M_PI;
  else theta = acos((tr - 1.0) / 2.0);
  double t;
  if (theta < PL_TAYLOR_PREC3) t = 1.0 + theta * theta / 6.0;
  else t = theta / sin(theta);
  w[0] = t / 2.0 * (R[7] - R[5]);
  w[1] = t / 2.0 * (R[2] - R[6]);
  w[2] = t / 2.0 * (R[3] - R[1]);
  *theta_out = theta;
}

PL_HD void log6_d(const double* R, const double* p, double* out) {
  double w[3], theta;
  log3_d(R, w, &theta);
  double t2 = theta * theta, alpha, beta;
  if (theta < PL_TAYLOR_PREC3) {
    alpha = 1.0 - t2 / 12.0 - t2 * t2 / 720.0;
    beta = 1.0 / 12.0 + t2 / 720.0;
  } else {
    double st = sin(theta), ct = cos(theta);
    alpha = theta * st / (2.0 * (1.0 - ct));
    beta = 1.0 / t2 - st / (2.0 * theta * (1.0 - ct));
  }
  double wxp[3];
  cross3(w, p, wxp);
  double wp = dot3(w, p);
  for (int k = 0; k < 3; ++k) out[k] = alpha * p[k] - 0.5 * wxp[k] + (beta * wp) * w[k];
  for (int k = 0; k < 3; ++k) out[3 + k] = w[k];
}

PL_HD void difference_q(const PlModel& M, const double* q0, const double* q1, double* dq) {
  double R0[9], R1[9];
  quat_to_R(q0 + 3, R0);
  quat_to_R(q1 + 3, R1);
  double R[9];
  for (int r = 0; r < 3; ++r)
    for (int c = 0; c < 3; ++c) R[3 * r + c] = R0[r] * R1[c] + R0[3 + r] * R1[3 + c] + R0[6 + r] * R1[6 + c];
  double d[3] = {q1[0] - q0[0], q1[1] - q0[1], q1[2] - q0[2]};
  double p[3];
  mattvec(R0, d, p);
  log6_d(R, p, dq);
  for (int j = 2; j < M.njoints; ++j) dq[M.idx_v[j]] = q1[M.idx_q[j]] - q0[M.idx_q[j]];
}

}  // namespace pl
