// Per-node constraint rows of the OCP, templated on the scalar (double / Dual).
//
// Emits g, lbg, ubg of one horizon node in the reference's subject_to order:
//   node 0 starts with DX_0 == 0                          (optimization/ocp.py:109)
//   setup_dynamics_constraints(i)                          (ocp_whole_body_rnea.py:138-171,
//                                                           ocp_whole_body_acc.py:90-112,
//                                                           ocp_whole_body_aba.py:86-106)
//   per foot FR, FL, RR, RL: friction cone, swing force, no-slip, swing height
//                                                          (ocp.py:121-157)
//   external force, arm velocity, joint limits             (ocp.py:165-190)
// The block list per node type is built on the host (api.cpp: build_blocks) so
// the row order has one definition shared by the layout code and this emitter.
#pragma once
#include <type_traits>

#include "rbd.h"

namespace pl {

// OCS2 cubic swing spline (utils/gait_sequence.py:96-133), evaluated in double
// (it depends on parameters only).
PL_HD double spline_vel_z(double phase, double period, double h_max, double v_lo, double v_td) {
  double mid = period / 2.0;
  double t = phase * period;
  double t0, dt, c1, c2, c3;
  if (phase < 0.5) {
    t0 = 0.0; dt = mid - 0.0;
    double p0 = 0.0, v0 = v_lo, p1 = h_max, v1 = 0.0;
    double dpos = p1 - p0, dvel = v1 - v0;
    c1 = v0 * dt; c2 = -(3.0 * v0 + dvel) * dt + 3.0 * dpos; c3 = (2.0 * v0 + dvel) * dt - 2.0 * dpos;
  } else {
    t0 = mid; dt = period - mid;
    double p0 = h_max, v0 = 0.0, p1 = 0.0, v1 = v_td;
    double dpos = p1 - p0, dvel = v1 - v0;
    c1 = v0 * dt; c2 = -(3.0 * v0 + dvel) * dt + 3.0 * dpos; c3 = (2.0 * v0 + dvel) * dt - 2.0 * dpos;
  }
  double tn = (t - t0) / dt;
  return (3.0 * c3 * tn * tn + 2.0 * c2 * tn + c1) / dt;
}

PL_HD int node_type(const PlOcpConst& O, int i) { return i == 0 ? 0 : (i < O.tau_nodes ? 1 : 2); }
PL_HD int node_nu(const PlOcpConst& O, int i) {
  if (PL_IS_RNEA(O.dyn)) return O.na + O.nf + (i < O.tau_nodes ? O.nj : 0);
  if (O.dyn == PL_DYN_ACC || O.dyn == PL_DYN_CA || O.dyn == PL_DYN_ACCNB) return O.na + O.nf;
  if (O.dyn == PL_DYN_CV) return O.nv + O.nf;
  return O.nj + O.nf;  // aba: [tau_j | f]; centroidal_vel without the base: [v_j | f]
}


// Geometric step size dt_i (ocp.py:71-74).
PL_HD double node_dt(const PlOcpConst& O, const double* p, int i) {
  double dt_min = p[O.P.dt_min], dt_max = p[O.P.dt_max];
  double gamma = pow(dt_max / dt_min, 1.0 / (double)(O.N - 1));
  return dt_min * pow(gamma, (double)i);
}

#define PL_INF (__builtin_inf())

// Input accessor over the node's local columns: x (+ alpha * step) with an
// optional dual seed.  dx = cols [0, ndx), u = [ndx, nw), dx_{i+1} = [nw, nw+ndx).
template <class S> struct VecIn;
template <> struct VecIn<double> {
  const double* x;
  const double* step;
  double alpha;
  int seed;
  PL_HD double operator[](int k) const { return step ? x[k] + alpha * step[k] : x[k]; }
};
template <> struct VecIn<Dual> {
  const double* x;
  const double* step;
  double alpha;
  int seed;
  PL_HD Dual operator[](int k) const { return Dual(x[k], k == seed ? 1.0 : 0.0); }
};
// two seeds: the e1 / e2 parts of column seed / seed2 (the Lagrangian Hessian, k_lag_hess)
template <> struct VecIn<HDual> {
  const double* x;
  const double* step;
  double alpha;
  int seed, seed2;
  PL_HD HDual operator[](int k) const { return HDual(x[k], k == seed ? 1.0 : 0.0, k == seed2 ? 1.0 : 0.0, 0.0); }
};
template <class S> PL_HD VecIn<S> sub_in(const VecIn<S>& a, int off) {
  VecIn<S> r = a;
  r.x = a.x + off;
  if (a.step) r.step = a.step + off;
  r.seed = a.seed - off;
  if constexpr (std::is_same<S, HDual>::value) r.seed2 = a.seed2 - off;
  return r;
}
// a seed of the input in [lo, hi) (for HDual: either seed -- a pass whose outputs do not
// depend on one seed's column has zero mixed second derivatives)
template <class S> PL_HD bool seeded(const VecIn<S>& a, int lo, int hi) {
  bool r = a.seed >= lo && a.seed < hi;
  if constexpr (std::is_same<S, HDual>::value) r = r || (a.seed2 >= lo && a.seed2 < hi);
  return r;
}

// Acceleration input of the tree pass for the include_base = False variants: the base
// acceleration zeroed (the base rows at a_b = 0 give the right-hand side of the base solve).
// whole_body_rnea with include_acc = False: a = (v_{i+1} - v_i) / dt with v = x_init.v + dv
// (get_a, ocp_whole_body_rnea.py:183-191), in the oracle's operation order.
template <class S> struct FdAcc {
  const double* xv;
  VecIn<S> dv, dvn;
  double dt;
  PL_HD S operator[](int k) const { return ((xv[k] + dvn[k]) - (xv[k] + dv[k])) / dt; }
};

template <class S> struct ZeroBaseAcc {
  VecIn<S> aj;
  PL_HD S operator[](int k) const { return k < 6 ? S(0.0) : aj[k - 6]; }
};

// kstore: caller storage for the run-time indexed kinematic outputs (NodeKin,
// PL_KIN_STORE entries spaced by kstride).
// Shared primal of the ABA Jacobian (k_eval_jac<ABA>): a = ABA(q, v, tau_j, f) in
// [0, PL_MAXV) and the Cholesky factor of the joint-space mass matrix M(q) (packed lower)
// from PL_MAXV on.
#define PL_ABA_SH (PL_MAXV + PL_MAXV * (PL_MAXV + 1) / 2)
struct ShAcc {  // the shared primal acceleration as a constant (zero tangent)
  const double* a;
  PL_HD Dual operator[](int k) const { return Dual(a[k], 0.0); }
};
// x <- L^-T L^-1 x (L packed lower, row i at i (i + 1) / 2)
PL_HD void chol_solve(const double* L, int n, double* x) {
  for (int i = 0; i < n; ++i) {
    const double* Li = L + i * (i + 1) / 2;
    double t = x[i];
    for (int k = 0; k < i; ++k) t -= Li[k] * x[k];
    x[i] = t / Li[i];
  }
  for (int i = n - 1; i >= 0; --i) {
    double t = x[i];
    for (int k = i + 1; k < n; ++k) t -= L[k * (k + 1) / 2 + i] * x[k];
    x[i] = t / L[i * (i + 1) / 2 + i];
  }
}

// kvals (Dual only): a shared value store for the kinematic outputs (NodeKin<Dual>);
// null keeps values and tangents interleaved in kstore.  aba_sh (Dual, ABA only): the
// node's shared primal (PL_ABA_SH); the ABA tangent then comes from the implicit
// function M a' = [0; tau_j'] - RNEA'(q', v', f' | a) instead of a dual ABA.
// lin_base (Dual, rnea, a column seeded on a or f only): the RNEA is linear in that input,
// so the caller took the torque tangent from a primal pass instead of the dual tree pass:
// lin_base holds the 6 base torques' tangents and the first nj tangent slots of kstore the
// joint torques' (k_eval_jac_lin); every other kinematic tangent of such a column is zero.
// An emitter may skip whole row blocks: emit.skip_block(n) returns true (and advances past the n
// rows) when none of them is wanted -- the Jacobian's column emitter, whose column has entries in
// a few rows only (k_eval.hip JacEmit).  Emitters without the member compute every row.
template <class E>
PL_HD auto emit_skip(E& e, int n, int) -> decltype(e.skip_block(n)) { return e.skip_block(n); }
template <class E>
PL_HD bool emit_skip(E&, int, long) { return false; }

template <class S, int DYN, class Emit>
PL_HD void node_rows(const PlModel& M, const PlOcpConst& O, int i, const double* p, const VecIn<S>& dx,
                     const VecIn<S>& u, const VecIn<S>& dxn, Emit& emit, S* kstore, int kstride,
                     double* kvals = nullptr, const double* aba_sh = nullptr, const double* lin_base = nullptr,
                     int only_ch = -1) {
  const int nv = O.nv, nq = O.nq, nj = O.nj;
  constexpr bool CV = PL_IS_CV(DYN);
  constexpr bool CVNB = (DYN == PL_DYN_CVNB);  // v = [base_vel_dynamics(h, q, v_j), v_j]
  const double* xi = p + O.P.x_init;
  const double dt = node_dt(O, p, i);
  const int type = node_type(O, i);
  // state: q = integrate(x_init.q, dq), v = x_init.v + dv   (ocp_whole_body_rnea.py:173-181);
  // centroidal_vel: x = [h, q], dx = [dh, dq], v = u[:nv]    (ocp_centroidal_vel.py:109-127);
  // the free-flyer part of q in registers, the rest read through accessors
  const double* xq = CV ? xi + 6 : xi;
  const VecIn<S> dq = CV ? sub_in(dx, 6) : dx;
  S qb[7];
  integrate_ff<S>(xq, dq, qb);
  const RevQ<S, VecIn<S>> qrev{xq, dq};
  // centroidal_vel without the base: one centroidal pass at v = [0, v_j] gives A_j v_j,
  // h_dot, the CoM and the composite inertia, then v_b = A_b^-1 (m h - A_j v_j)
  // (ocp_centroidal_vel.py:119-129, dynamics_centroidal_vel.py:73-89)
  S vnb[CVNB ? PL_MAXV : 1], hdot_nb[CVNB ? 6 : 1];
  if constexpr (CVNB) {
    bool run = true;
    if constexpr (!std::is_same<S, double>::value) run = !seeded(dxn, 0, O.ndx);
    if (run) {
      S hj[6], ci[9], hcur[6], R0[9];
      centroidal_pass<S>(M, O, qb, qrev, ZeroBaseAcc<S>{u}, sub_in(u, nj), true, true, hj, hdot_nb, ci,
                         std::true_type{});
      for (int k = 0; k < 6; ++k) hcur[k] = xi[k] + dx[k];
      quat_to_R(qb + 3, R0);
      base_vel_solve(M.total_mass, R0, qb, ci, hcur, hj, vnb);
    } else {
      for (int k = 0; k < 6; ++k) { vnb[k] = S(0.0); hdot_nb[k] = S(0.0); }
    }
    for (int k = 0; k < nj; ++k) vnb[6 + k] = u[k];
  }
  const auto vel = [&]() {
    if constexpr (CVNB) return static_cast<const S*>(vnb);
    else if constexpr (CV) return u;
    else return VelAcc<S, VecIn<S>>{xi + nq, sub_in(dx, nv)};
  }();
  // acc family: whole_body_acc (ACC), centroidal_acc (CA), their include_base = False form (ACCNB)
  constexpr bool ACCF = (DYN == PL_DYN_ACC || DYN == PL_DYN_CA || DYN == PL_DYN_ACCNB);
  constexpr bool NB = (DYN == PL_DYN_ACCNB);
  constexpr bool COMP = (DYN == PL_DYN_CA || DYN == PL_DYN_ACCNB);
  constexpr bool FD = (DYN == PL_DYN_RNEAFD);
  const int f_off = (PL_IS_RNEA(DYN) || ACCF) ? O.na : (DYN == PL_DYN_CV ? nv : nj);
  const VecIn<S> a = u;                                   // rnea / acc: a = u[0:nv]
  const FdAcc<S> afd{xi + nq, sub_in(dx, nv), sub_in(dxn, nv), dt};  // rnea, include_acc = False
  const VecIn<S> forces = sub_in(u, f_off);
  const VecIn<S> tau_j = sub_in(u, PL_IS_RNEA(DYN) ? O.na + O.nf : 0);
  // centroidal_vel keeps the state rows at node 0 (ocp.py:137-140, 170-173)
  const bool state_rows = CV || (type != 0);
  NodeKin<S> kin;
  if constexpr (std::is_same<S, Dual>::value) {
    double* raw = reinterpret_cast<double*>(kstore);
    if (kvals) {  // shared values, per-lane tangents (kstore holds kstride-strided doubles)
      kin.vst = kvals;
      kin.vstride = 1;
      kin.dst = raw;
      kin.dstride = kstride;
    } else {
      kin.vst = raw;
      kin.dst = raw + 1;
      kin.vstride = kin.dstride = 2 * kstride;
    }
  } else {
    (void)kvals;
    kin.store = kstore;
    kin.stride = kstride;
  }
  constexpr bool want_tau = (PL_IS_RNEA(DYN) || ACCF);
  // A Jacobian column seeded on dx_{i+1}, or (rnea) on tau_j, has a zero tangent in the
  // tree pass and the ABA: every row that reads them then has a zero derivative, so
  // the pass is skipped (its values are not emitted for such a column's pattern).
  // centroidal_vel: h and the forces do not enter the kinematics either; the
  // centroidal pass reads the forces but not h.
  bool tree = true, cen = CV;
  if constexpr (!std::is_same<S, double>::value) {
    // (FD: dv_{i+1} enters the pass through a)
    const bool seed_dxn = seeded(dxn, 0, FD ? nv : O.ndx);
    const bool seed_tau = PL_IS_RNEA(DYN) && seeded(u, O.na + O.nf, O.na + O.nf + nj);
    // (without the base, h enters the kinematics through v_b; its centroidal pass ran above)
    const bool seed_h = DYN == PL_DYN_CV && seeded(dx, 0, 6);
    const bool seed_f = CV && seeded(u, f_off, f_off + O.nf);
    // whole_body_rnea / _acc: the RNEA, the foot and arm velocities do not read the base
    // position (translation invariance), so a dq_0..2 column skips the pass (its exact
    // tangents there are 0; the dual pass left round-off)
    const bool seed_pos = (PL_IS_RNEA(DYN) || DYN == PL_DYN_ACC) && seeded(dx, 0, 3);
    tree = !(seed_dxn || seed_tau || seed_h || seed_f || seed_pos) && !lin_base;
    cen = DYN == PL_DYN_CV && !(seed_dxn || seed_h);
  } else {
    (void)lin_base;
  }
  S comp[COMP ? 15 : 1];
  S aba_a[DYN == PL_DYN_ABA ? PL_MAXV : 1];
  bool aba_done = false;
  if constexpr (DYN == PL_DYN_ABA && std::is_same<S, Dual>::value) {
    {  // aba_sh is required for the dual ABA rows (pl::aba_primal computes it)
      if (tree) {
        // one tree pass at the shared primal a: the RNEA tangent and the state rows
        tree_pass<S>(M, O, qb, qrev, vel, ShAcc{aba_sh}, forces, true, state_rows, kin);
        double r[PL_MAXV];
        for (int k = 0; k < 6; ++k) r[k] = -kin.tau[k].d;
        for (int k = 0; k < nj; ++k) {
          const Dual t = kin.tau_j(k);
          r[6 + k] = tau_j[k].d - t.d;
        }
        chol_solve(aba_sh + PL_MAXV, nv, r);
        for (int k = 0; k < nv; ++k) aba_a[k] = Dual(aba_sh[k], r[k]);
      } else {
        for (int k = 0; k < PL_KIN_STORE_DUAL; ++k) kin.clear(k);
        for (int k = 0; k < 3; ++k) kin.arm_vel[k] = S(0.0);
        for (int k = 0; k < nv; ++k) aba_a[k] = S(0.0);
      }
      aba_done = true;
    }
  }
  if (aba_done) {
  } else if (tree && (want_tau || state_rows)) {
    if constexpr (NB) {
      tree_pass<S>(M, O, qb, qrev, vel, ZeroBaseAcc<S>{a}, forces, want_tau, state_rows, kin, comp, std::true_type{});
    } else if constexpr (COMP) {
      tree_pass<S>(M, O, qb, qrev, vel, a, forces, want_tau, state_rows, kin, comp, std::true_type{});
    } else if constexpr (FD) {
      tree_pass<S>(M, O, qb, qrev, vel, afd, forces, want_tau, state_rows, kin, nullptr, std::false_type{}, only_ch);
    } else {
      tree_pass<S>(M, O, qb, qrev, vel, a, forces, want_tau, state_rows, kin, nullptr, std::false_type{}, only_ch);
    }
  } else {  // a skipped pass leaves zero (value and tangent) kinematic outputs
    for (int k = lin_base ? nj : 0; k < PL_KIN_STORE_DUAL; ++k) kin.clear(k);
    for (int k = 0; k < 3; ++k) kin.arm_vel[k] = S(0.0);
    for (int k = 0; k < 6; ++k) kin.tau[k] = S(0.0);
    if constexpr (COMP)
      for (int k = 0; k < 15; ++k) comp[k] = S(0.0);
    if constexpr (std::is_same<S, Dual>::value)
      if (lin_base)
        for (int k = 0; k < 6; ++k) kin.tau[k] = Dual(0.0, lin_base[k]);
  }
  // acc family: the base acceleration (include_base = False) or the centroidal gap
  S abase[NB ? 6 : 1], cgap[DYN == PL_DYN_CA ? 6 : 1];
  if constexpr (COMP) {
    if (tree) {
      S R0[9];
      quat_to_R(qb + 3, R0);
      if constexpr (NB) base_solve(M.total_mass, R0, comp, kin.tau, abase);
      else centroidal_gap(M.total_mass, qb, comp, cgap);
    } else {
      for (int k = 0; k < 6; ++k) {
        if constexpr (NB) abase[k] = S(0.0);
        else cgap[k] = S(0.0);
      }
    }
  }
  S hg[CV ? 6 : 1], hdot[CV ? 6 : 1];
  if constexpr (CVNB) {
    for (int k = 0; k < 6; ++k) hdot[k] = hdot_nb[k];
  } else if constexpr (CV) {
    if (cen) {
      centroidal_pass<S>(M, O, qb, qrev, vel, forces, true, true, hg, hdot);
    } else {
      for (int k = 0; k < 6; ++k) { hg[k] = S(0.0); hdot[k] = S(0.0); }
    }
  }
  if constexpr (DYN == PL_DYN_ABA && !std::is_same<S, Dual>::value) {
    if (aba_done) {
    } else if (tree) {
      S q[PL_MAXQ], v[PL_MAXV];
      for (int k = 0; k < 7; ++k) q[k] = qb[k];
      for (int k = 7; k < nq; ++k) q[k] = qrev(k);
      for (int k = 0; k < nv; ++k) v[k] = vel[k];
      aba_forward<S>(M, O, q, v, tau_j, forces, aba_a);
    } else {
      for (int k = 0; k < nv; ++k) aba_a[k] = S(0.0);
    }
  }

  const int nb = O.nblk[type];
  for (int bi = 0; bi < nb; ++bi) {
    const PlRowBlock B = O.blk[type][bi];
    const int k = B.arg;
    if (emit_skip(emit, B.count, 0)) continue;  // B.count: the rows the switch below emits
    switch (B.kind) {
      case PL_RB_INIT:
        for (int r = 0; r < O.ndx; ++r) emit(dx[r], 0.0, 0.0);
        break;
      case PL_RB_DYNQ:
        for (int r = 0; r < nv; ++r) emit(dxn[r] - (dx[r] + vel[r] * dt), 0.0, 0.0);
        break;
      case PL_RB_DYNV:
        for (int r = 0; r < nv; ++r) {
          S ar;
          if constexpr (DYN == PL_DYN_ABA) ar = aba_a[r];
          else if constexpr (NB) ar = r < 6 ? abase[r] : a[r - 6];
          else ar = a[r];
          emit(dxn[nv + r] - (dx[nv + r] + ar * dt), 0.0, 0.0);
        }
        break;
      case PL_RB_RNEA_BASE:
        for (int r = 0; r < 6; ++r) emit(kin.tau[r], 0.0, 0.0);
        break;
      case PL_RB_TAU_EQ:
        for (int r = 0; r < nj; ++r) emit(kin.tau_j(r) - tau_j[r], 0.0, 0.0);
        break;
      case PL_RB_TAU_BND:
        for (int r = 0; r < nj; ++r) emit(tau_j[r], -O.tau_max[r], O.tau_max[r]);
        break;
      case PL_RB_FZ: {
        double c = p[O.P.contact + 4 * i + k];
        emit(c * forces[3 * k + 2], 0.0, PL_INF);
      } break;
      case PL_RB_CONE: {
        double c = p[O.P.contact + 4 * i + k];
        S f0 = forces[3 * k], f1 = forces[3 * k + 1], f2 = forces[3 * k + 2];
        emit(c * (f0 * f0 + f1 * f1) - (c * O.mu * O.mu) * (f2 * f2), -PL_INF, 0.0);
      } break;
      case PL_RB_SWINGF: {
        double c = p[O.P.contact + 4 * i + k];
        for (int r = 0; r < 3; ++r) emit((1.0 - c) * forces[3 * k + r], 0.0, 0.0);
      } break;
      case PL_RB_FVXY: {
        double c = p[O.P.contact + 4 * i + k];
        emit(c * kin.foot_vel(k, 0), 0.0, 0.0);
        emit(c * kin.foot_vel(k, 1), 0.0, 0.0);
      } break;
      case PL_RB_FVZ: {
        double c = p[O.P.contact + 4 * i + k];
        double ph = p[O.P.swing + 4 * i + k];
        double vz_des = spline_vel_z(ph, p[O.P.swing_period], p[O.P.swing_height], p[O.P.swing_vel_limits],
                                     p[O.P.swing_vel_limits + 1]);
        S vz = kin.foot_vel(k, 2);
        emit(c * vz + (1.0 - c) * (vz - vz_des), 0.0, 0.0);
      } break;
      case PL_RB_EXT:
        for (int r = 0; r < 3; ++r) emit(forces[3 * O.nfeet + r] - p[O.P.ext_force_des + r], 0.0, 0.0);
        break;
      case PL_RB_ARM:
        for (int r = 0; r < 3; ++r) emit(kin.arm_vel[r] - p[O.P.arm_vel_des + r], 0.0, 0.0);
        break;
      case PL_RB_QJ:
        for (int r = 0; r < nj; ++r) emit(qrev(7 + r), O.pos_min[r], O.pos_max[r]);
        break;
      case PL_RB_VJ:
        for (int r = 0; r < nj; ++r) emit(vel[6 + r], -O.vel_max[r], O.vel_max[r]);
        break;
      case PL_RB_CV_DYNH:
        if constexpr (CV)
          for (int r = 0; r < 6; ++r) emit(dxn[r] - (dx[r] + hdot[r] * dt), 0.0, 0.0);
        break;
      case PL_RB_CV_DYNQ:
        for (int r = 0; r < nv; ++r) emit(dxn[6 + r] - (dx[6 + r] + vel[r] * dt), 0.0, 0.0);
        break;
      case PL_RB_CV_GAP:
        if constexpr (CV)
          for (int r = 0; r < 6; ++r) emit(hg[r] - M.total_mass * (xi[r] + dx[r]), 0.0, 0.0);
        break;
      case PL_RB_CA_GAP:
        if constexpr (DYN == PL_DYN_CA)
          for (int r = 0; r < 6; ++r) emit(cgap[r], 0.0, 0.0);
        break;
    }
  }
}

}  // namespace pl
