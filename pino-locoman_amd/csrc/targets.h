// Tracking targets and objective terms (host+device, doubles).
//
// x_des = [q0, base_vel_des, 0], dx_des = difference(x_init, x_des)
//   (ocp_whole_body_rnea.py:91-94, ocp_whole_body_acc.py:73-76, ocp_whole_body_aba.py:69-72;
//   centroidal_vel: x_des = [base_vel_des, q0], ocp_centroidal_vel.py:60-63);
// f_des = 0.8 / 1.2 * m g / n_contacts on front / rear feet, 0 on the end effector,
// u_des = [0_a, f_des, 0_tau] (ocp_whole_body_rnea.py:96-106 and siblings);
// objective sum_i |dx_i - dx_des|_Q^2 + |u_i - u_des|_R^2 (+ |tau_0 - tau_prev|_W^2)
//   + |dx_N - dx_des|_Q^2 (ocp.py:80-101, ocp_whole_body_rnea.py:108-136).
#pragma once
#include "rbd.h"
#include "rows.h"

namespace pl {

PL_HD void compute_dx_des(const PlModel& M, const PlOcpConst& O, const double* p, double* dxd) {
  const double* xi = p + O.P.x_init;
  if (PL_IS_CV(O.dyn)) {
    // x_des = [base_vel_des, q0], dx_des = [h_des - h, difference(q, q0)] (ocp_centroidal_vel.py:61-63)
    for (int k = 0; k < 6; ++k) dxd[k] = p[O.P.base_vel_des + k] - xi[k];
    difference_q(M, xi + 6, O.q0, dxd + 6);
    return;
  }
  difference_q(M, xi, O.q0, dxd);
  for (int k = 0; k < O.nv; ++k) {
    double vd = (k < 6) ? p[O.P.base_vel_des + k] : 0.0;
    dxd[O.nv + k] = vd - xi[O.nq + k];
  }
}

// Force target of component c (0..nf-1) of the stacked end-effector forces.
PL_HD double f_des_comp(const PlModel& M, const PlOcpConst& O, const double* p, int c) {
  int foot = c / 3, ax = c % 3;
  if (foot >= O.nfeet || ax != 2) return 0.0;
  double fg = 9.81 * M.total_mass;
  double nc = p[O.P.n_contacts];
  return (foot < 2 ? 0.8 : 1.2) * fg / nc;
}

// Offset of the forces inside u for the dynamics kind.
PL_HD int u_force_off(const PlOcpConst& O) {
  if (PL_IS_RNEA(O.dyn) || O.dyn == PL_DYN_ACC || O.dyn == PL_DYN_CA || O.dyn == PL_DYN_ACCNB) return O.na;
  return O.dyn == PL_DYN_CV ? O.nv : O.nj;
}

// u_des[k] (k indexes the padded input of length nu_0).
PL_HD double u_des(const PlModel& M, const PlOcpConst& O, const double* p, int k) {
  int fo = u_force_off(O);
  if (k >= fo && k < fo + O.nf) return f_des_comp(M, O, p, k - fo);
  return 0.0;
}

// Gait schedule (utils/gait_sequence.py:26-77) for one problem.
PL_HD void gait_schedule(const PlOcpConst& O, int gait_type, double period, double swing_period, double t_cur,
                              const double* p, double* contact, double* swing) {
  const int N = O.N;
  double t = t_cur;
  for (int i = 0; i < N; ++i) {
    if (i > 0) t += pl::node_dt(O, p, i - 1);
    for (int f = 0; f < 4; ++f) {
      contact[4 * i + f] = 1.0;
      swing[4 * i + f] = 0.0;
    }
    if (gait_type == 2) continue;
    double gp = fmod(t, period) / period;
    double sp = fmod(t, swing_period) / swing_period;
    int f0 = -1, f1 = -1;
    if (gait_type == 0) {
      if (gp < 0.5) { f0 = 0; f1 = 3; } else { f0 = 1; f1 = 2; }
    } else {
      f0 = gp < 0.25 ? 1 : gp < 0.5 ? 2 : gp < 0.75 ? 0 : 3;
    }
    contact[4 * i + f0] = 0.0;
    swing[4 * i + f0] = sp;
    if (f1 >= 0) {
      contact[4 * i + f1] = 0.0;
      swing[4 * i + f1] = sp;
    }
  }
}

}  // namespace pl
