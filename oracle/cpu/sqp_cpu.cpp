// CPU BASELINE (test infrastructure; never linked into the product) -- a compiled C++
// restatement of the reference's CPU solve path, timed beside the GPU in bench.py.
//
// One MPC step of one problem, as run_mpc.py:127-143 drives the OSQP branch of
// OCP.solve() (optimization/ocp.py:375-422):
//   gait schedule + x_init update + warm start   (ocp.py:231-242, ocp_whole_body_rnea.py:207-235)
//   sqp_data: constraint values, Jacobian (forward-mode duals), objective gradient
//   osqp.update + osqp.solve: OSQP 0.6 -- Ruiz equilibration, rho vector, the
//     quasi-definite KKT [P + sigma I, A^T; A, -diag(rho)^-1] factored by a sparse
//     up-looking LDL^T (the QDLDL algorithm OSQP ships) in a node-interleaved
//     ordering, ADMM with relaxation, termination / infeasibility checks every 25
//     iterations, the x10 "approximate" check at max_iter, warm-started iterates
//   _armijo_line_search (ocp.py:430-480), _constraint_violation_max
//   x_state <- integrate(x_state, DX[1])          (run_mpc.py:142)
// The per-node row math is the product's templated row code (csrc/rows.h) compiled
// for the host with g++; everything else here is a separate restatement that
// follows oracle/osqp_ref.py and oracle/ocp.py line by line.  Problems are
// independent: OpenMP runs one problem per thread.
#include <math.h>
#include <omp.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <vector>

#include "dyn.h"
#include "rows.h"
#include "targets.h"

namespace {

constexpr double OSQP_INFTY = 1e30, MIN_SCALING = 1e-4, MAX_SCALING = 1e4, RHO_MIN = 1e-6, RHO_TOL = 1e-4;
constexpr double RHO_EQ = 1e3, DIV_TOL = 1e-30;
enum { SOLVED = 1, SOLVED_INACC = 2, MAX_ITER = -2, PRIM_INF = -3, PRIM_INF_INACC = 3, DUAL_INF = -4,
       DUAL_INF_INACC = 4, NON_CVX = -7, UNSOLVED = -10 };

struct Settings {
  double rho, sigma, alpha, eps_abs, eps_rel, eps_pinf, eps_dinf;
  int max_iter, check_termination, scaling, gait_type;
  double gait_period, swing_period;
};

struct VEmit {
  double* g; double* l; double* u; int r;
  void operator()(double v, double lb, double ub) { g[r] = v; l[r] = lb; u[r] = ub; ++r; }
};
struct TEmit {
  double* t; int r;
  void operator()(const Dual& v, double, double) { t[r++] = v.d; }
};
struct ViolEmit {
  double ss, mx;
  void operator()(double v, double l, double u) {
    const double a = fmax(0.0, l - v), c = fmax(0.0, v - u);
    ss += a * a + c * c;
    mx = fmax(mx, fmax(a, c));
  }
};

inline double limit(double v) { return v < MIN_SCALING ? 1.0 : (v > MAX_SCALING ? MAX_SCALING : v); }

// Upper-triangular CSC pattern of a symmetric K x K matrix and its symbolic LDL^T.
struct Kkt {
  int K = 0;
  std::vector<int> Kp, Ki;
  std::vector<int> etree, Lnz, Lp;
};

struct LdlWork {  // numeric LDL^T of one Kkt
  std::vector<double> Kx, Lx, Dd, Dinv, buf;
  std::vector<int> Li, yMark, yIdx, elim, nextc;
  void init(const Kkt& k) {
    Kx.assign(k.Ki.size(), 0.0);
    Lx.assign(k.Lp[k.K], 0.0);
    Li.assign(k.Lp[k.K], 0);
    for (auto* v : {&Dd, &Dinv, &buf}) v->assign(k.K, 0.0);
    for (auto* v : {&yMark, &yIdx, &elim, &nextc}) v->assign(k.K, 0);
  }
};

// Shared (read-only) structure of one OCP: layout, A pattern (CSC), KKT pattern.
struct Problem {
  PlModel M;
  PlOcpConst O;
  Settings S;
  int N, n, m, nnz, np;
  std::vector<int> x_off, row_off, nrow, nw;   // per node (N + 1)
  std::vector<int> colnode;                    // global column -> node
  // A in CSC over the library pattern; per node and local column: (local row, CSC slot)
  std::vector<int> Ap, Ai;
  std::vector<std::vector<std::pair<int, int>>> jcol;  // [node][local col] flattened below
  std::vector<int> jc_ptr;                     // node-local column lists: offsets per (node, lc)
  std::vector<int> jc_node_base;               // first (node, lc) index of node i
  std::vector<std::pair<int, int>> jc_list;    // (local row, CSC slot)
  // KKT: permuted index of x_j and of row r; upper-triangular CSC pattern; value maps
  std::vector<int> perm_x, perm_z;
  Kkt kkt;
  std::vector<int> kdiag_x, kdiag_z, kA;      // KKT slot of (x_j, x_j), (z_r, z_r), A entry e
  // interior point (built by cpu_ip_prepare): Lagrangian Hessian pairs per node type and the
  // KKT [H + H_L + d I, J^T; J, -W^-1] with the w_i blocks of H_L in its pattern
  bool ip_ready = false;
  // its own KKT ordering: per node the node's rows, then its variables (ip_prepare)
  std::vector<int> iperm_x, iperm_z;
  std::vector<std::pair<int, int>> hpairs[3];  // (j, k), j <= k, structurally non-zero (probe)
  Kkt ipk;
  std::vector<int> ik_diag_x, ik_diag_z, ik_A;
  std::vector<int> ik_H_off, ik_H;            // per node: first slot index into ik_H; KKT slot per pair
};

struct Work {  // per-thread scratch
  std::vector<double> g, lbg, ubg, grad, Ax, A, tan, P, q, l, u, xs_, zs_, ys_, D, E, rho, rinv, rhs, sol, xt, zt, dx,
      dy, x_prev, z_prev, Axv, Aty, step, xtrial, buf;
  LdlWork ldl;
  void init(const Problem& pr) {
    const int n = pr.n, m = pr.m, K = pr.kkt.K;
    for (auto* v : {&g, &lbg, &ubg, &l, &u, &zs_, &ys_, &E, &rho, &rinv, &zt, &dy, &z_prev, &Axv})
      v->assign(m, 0.0);
    for (auto* v : {&grad, &P, &q, &xs_, &D, &xt, &dx, &x_prev, &Aty, &step, &xtrial}) v->assign(n, 0.0);
    Ax.assign(pr.nnz, 0.0);
    A.assign(pr.nnz, 0.0);
    tan.assign(512, 0.0);
    ldl.init(pr.kkt);
    rhs.assign(K, 0.0);
    sol.assign(K, 0.0);
    buf.assign(std::max(K, m), 0.0);
  }
};

// ---------------------------------------------------------------- evaluation
template <int DYN>
void eval_values(const Problem& pr, const double* p, const double* x, const double* step, double alpha, double* g,
                 double* lb, double* ub) {
  double kst[PL_KIN_STORE];
  for (int i = 0; i < pr.N; ++i) {
    const int xo = pr.x_off[i], xn = pr.x_off[i + 1], ndx = pr.O.ndx;
    pl::VecIn<double> dx{x + xo, step ? step + xo : nullptr, alpha, -1};
    pl::VecIn<double> u{x + xo + ndx, step ? step + xo + ndx : nullptr, alpha, -1};
    pl::VecIn<double> dxn{x + xn, step ? step + xn : nullptr, alpha, -1};
    VEmit e{g + pr.row_off[i], lb + pr.row_off[i], ub + pr.row_off[i], 0};
    pl::node_rows<double, DYN>(pr.M, pr.O, i, p, dx, u, dxn, e, kst, 1);
  }
}

template <int DYN>
void violation(const Problem& pr, const double* p, const double* x, const double* step, double alpha, double* metric,
               double* vmax) {
  double kst[PL_KIN_STORE];
  ViolEmit e{0.0, 0.0};
  for (int i = 0; i < pr.N; ++i) {
    const int xo = pr.x_off[i], xn = pr.x_off[i + 1], ndx = pr.O.ndx;
    pl::VecIn<double> dx{x + xo, step ? step + xo : nullptr, alpha, -1};
    pl::VecIn<double> u{x + xo + ndx, step ? step + xo + ndx : nullptr, alpha, -1};
    pl::VecIn<double> dxn{x + xn, step ? step + xn : nullptr, alpha, -1};
    pl::node_rows<double, DYN>(pr.M, pr.O, i, p, dx, u, dxn, e, kst, 1);
  }
  *metric = sqrt(e.ss);
  *vmax = e.mx;
}

// J values on the CSC pattern: one dual pass per local column.
template <int DYN>
void eval_jac(const Problem& pr, const double* p, const double* x, Work& w, double* Ax) {
  Dual kst[PL_KIN_STORE];
  double aba_sh[PL_ABA_SH];
  const int ndx = pr.O.ndx;
  for (int i = 0; i < pr.N; ++i) {
    const int xo = pr.x_off[i], xn = pr.x_off[i + 1], ncol = pr.nw[i] + ndx;
    if (DYN == PL_DYN_ABA) pl::aba_primal(pr.M, pr.O, p, x + xo, aba_sh);  // ABA tangent by implicit function
    for (int lc = 0; lc < ncol; ++lc) {
      const int c = pr.jc_node_base[i] + lc;
      if (pr.jc_ptr[c] == pr.jc_ptr[c + 1]) continue;
      pl::VecIn<Dual> dx{x + xo, nullptr, 0.0, lc};
      pl::VecIn<Dual> u{x + xo + ndx, nullptr, 0.0, lc - ndx};
      pl::VecIn<Dual> dxn{x + xn, nullptr, 0.0, lc - pr.nw[i]};
      TEmit e{w.tan.data(), 0};
      pl::node_rows<Dual, DYN>(pr.M, pr.O, i, p, dx, u, dxn, e, kst, 1, nullptr, aba_sh);
      for (int q = pr.jc_ptr[c]; q < pr.jc_ptr[c + 1]; ++q) Ax[pr.jc_list[q].second] = w.tan[pr.jc_list[q].first];
    }
  }
}

// objective (ocp.py:80-101; ocp_whole_body_rnea.py:108-136), at x + alpha step
double objective(const Problem& pr, const double* p, const double* x, const double* step, double alpha, double* grad) {
  const PlOcpConst& O = pr.O;
  double dxd[2 * PL_MAXV];
  pl::compute_dx_des(pr.M, O, p, dxd);
  const double* Q = p + O.P.Q_diag;
  const double* R = p + O.P.R_diag;
  double f = 0.0;
  for (int j = 0; j < pr.n; ++j) {
    const int i = pr.colnode[j], lc = j - pr.x_off[i];
    const double xj = step ? x[j] + alpha * step[j] : x[j];
    double gj;
    if (lc < O.ndx) {
      const double e = xj - dxd[lc];
      f += e * (Q[lc] * e);
      gj = 2.0 * Q[lc] * e;
    } else {
      const int k = lc - O.ndx;
      const double e = xj - pl::u_des(pr.M, O, p, k);
      f += e * (R[k] * e);
      gj = 2.0 * R[k] * e;
      if (PL_IS_RNEA(O.dyn) && i == 0 && k >= O.na + O.nf) {
        const int t = k - O.na - O.nf;
        const double W = p[O.P.W_diag + t], et = xj - p[O.P.tau_prev + t];
        f += et * (W * et);
        gj += 2.0 * W * et;
      }
    }
    if (grad) grad[j] = gj;
  }
  return f;
}

// ---------------------------------------------------------------- LDL^T (QDLDL algorithm)
void ldl_symbolic(Kkt& kk) {
  const int K = kk.K;
  std::vector<int> work(K);
  kk.etree.assign(K, -1);
  kk.Lnz.assign(K, 0);
  for (int j = 0; j < K; ++j) {
    work[j] = j;
    for (int q = kk.Kp[j]; q < kk.Kp[j + 1]; ++q) {
      int i = kk.Ki[q];
      if (i == j) continue;
      while (work[i] != j) {
        if (kk.etree[i] == -1) kk.etree[i] = j;
        kk.Lnz[i]++;
        work[i] = j;
        i = kk.etree[i];
      }
    }
  }
  kk.Lp.assign(K + 1, 0);
  for (int i = 0; i < K; ++i) kk.Lp[i + 1] = kk.Lp[i] + kk.Lnz[i];
}

// Up-looking numeric factorization of the upper-triangular CSC (Kp, Ki, Kx).
bool ldl_numeric(const Kkt& kk, LdlWork& w) {
  const int K = kk.K;
  double* y = w.buf.data();
  for (int i = 0; i < K; ++i) { w.yMark[i] = 0; y[i] = 0.0; w.nextc[i] = kk.Lp[i]; }
  for (int k = 0; k < K; ++k) {
    int nnzY = 0;
    w.Dd[k] = 0.0;
    for (int q = kk.Kp[k]; q < kk.Kp[k + 1]; ++q) {
      const int b = kk.Ki[q];
      if (b == k) { w.Dd[k] = w.Kx[q]; continue; }
      y[b] = w.Kx[q];
      int nx = b;
      if (!w.yMark[nx]) {
        w.yMark[nx] = 1;
        w.elim[0] = nx;
        int ne = 1;
        nx = kk.etree[b];
        while (nx != -1 && nx < k) {
          if (w.yMark[nx]) break;
          w.yMark[nx] = 1;
          w.elim[ne++] = nx;
          nx = kk.etree[nx];
        }
        while (ne) w.yIdx[nnzY++] = w.elim[--ne];
      }
    }
    for (int t = nnzY - 1; t >= 0; --t) {
      const int c = w.yIdx[t];
      const int tmp = w.nextc[c];
      const double yc = y[c];
      for (int j = kk.Lp[c]; j < tmp; ++j) y[w.Li[j]] -= w.Lx[j] * yc;
      w.Li[tmp] = k;
      w.Lx[tmp] = yc * w.Dinv[c];
      w.Dd[k] -= yc * w.Lx[tmp];
      w.nextc[c]++;
      y[c] = 0.0;
      w.yMark[c] = 0;
    }
    if (w.Dd[k] == 0.0) return false;
    w.Dinv[k] = 1.0 / w.Dd[k];
  }
  return true;
}

void ldl_solve(const Kkt& kk, const LdlWork& w, double* x) {
  const int K = kk.K;
  for (int i = 0; i < K; ++i)
    for (int j = kk.Lp[i]; j < kk.Lp[i + 1]; ++j) x[w.Li[j]] -= w.Lx[j] * x[i];
  for (int i = 0; i < K; ++i) x[i] *= w.Dinv[i];
  for (int i = K - 1; i >= 0; --i)
    for (int j = kk.Lp[i]; j < kk.Lp[i + 1]; ++j) x[i] -= w.Lx[j] * x[w.Li[j]];
}

// ---------------------------------------------------------------- OSQP 0.6
struct OsqpState {
  std::vector<double> x, z, y;  // scaled iterates (warm start)
};

struct OsqpInfo {
  int status, iter;
  double pri, dua;
};

double inf_norm(const double* v, int n) {
  double r = 0.0;
  for (int k = 0; k < n; ++k) r = fmax(r, fabs(v[k]));
  return r;
}

// osqp.update(q, Ax, l, u) + osqp.solve() (ocp.py:391-401); dx (unscaled) in w.step.
OsqpInfo osqp_update_solve(const Problem& pr, Work& w, OsqpState& st, const double* Pd, const double* qraw,
                           const double* Araw, const double* lraw, const double* uraw) {
  const Settings& S = pr.S;
  const int n = pr.n, m = pr.m, nnz = pr.nnz;
  double* P = w.P.data();
  double* q = w.q.data();
  double* A = w.A.data();
  double* D = w.D.data();
  double* E = w.E.data();
  for (int j = 0; j < n; ++j) { P[j] = Pd[j]; q[j] = qraw[j]; D[j] = 1.0; }
  for (int r = 0; r < m; ++r) E[r] = 1.0;
  for (int e = 0; e < nnz; ++e) A[e] = Araw[e];
  double c = 1.0;
  std::vector<double>& Dt = w.dx;  // scratch
  std::vector<double>& Et = w.dy;
  for (int pass = 0; pass < S.scaling; ++pass) {  // Ruiz (oracle/osqp_ref.py:_scale)
    for (int j = 0; j < n; ++j) {
      double mx = fabs(P[j]);
      for (int q2 = pr.Ap[j]; q2 < pr.Ap[j + 1]; ++q2) mx = fmax(mx, fabs(A[q2]));
      Dt[j] = 1.0 / sqrt(limit(mx));
    }
    for (int r = 0; r < m; ++r) Et[r] = 0.0;
    for (int j = 0; j < n; ++j)
      for (int q2 = pr.Ap[j]; q2 < pr.Ap[j + 1]; ++q2) Et[pr.Ai[q2]] = fmax(Et[pr.Ai[q2]], fabs(A[q2]));
    for (int r = 0; r < m; ++r) Et[r] = 1.0 / sqrt(limit(Et[r]));
    double psum = 0.0, qn = 0.0;
    for (int j = 0; j < n; ++j) {
      P[j] = Dt[j] * P[j] * Dt[j];
      for (int q2 = pr.Ap[j]; q2 < pr.Ap[j + 1]; ++q2) A[q2] = Et[pr.Ai[q2]] * A[q2] * Dt[j];
      q[j] = Dt[j] * q[j];
      D[j] *= Dt[j];
      psum += fabs(P[j]);
      qn = fmax(qn, fabs(q[j]));
    }
    for (int r = 0; r < m; ++r) E[r] *= Et[r];
    double ct = fmax(psum / n, limit(qn));
    ct = 1.0 / limit(ct);
    for (int j = 0; j < n; ++j) { P[j] *= ct; q[j] *= ct; }
    c *= ct;
  }
  const double cinv = 1.0 / c;
  double* ls = w.l.data();
  double* us = w.u.data();
  double* rho = w.rho.data();
  double* rinv = w.rinv.data();
  for (int r = 0; r < m; ++r) {
    ls[r] = E[r] * fmax(lraw[r], -OSQP_INFTY);
    us[r] = E[r] * fmin(uraw[r], OSQP_INFTY);
    const bool loose = ls[r] < -OSQP_INFTY * MIN_SCALING && us[r] > OSQP_INFTY * MIN_SCALING;
    const bool eq = !loose && us[r] - ls[r] < RHO_TOL;
    rho[r] = loose ? RHO_MIN : (eq ? RHO_EQ * S.rho : S.rho);
    rinv[r] = 1.0 / rho[r];
  }
  // KKT values + LDL^T
  std::vector<double>& Kx = w.ldl.Kx;
  std::fill(Kx.begin(), Kx.end(), 0.0);
  for (int j = 0; j < n; ++j) Kx[pr.kdiag_x[j]] = P[j] + S.sigma;
  for (int r = 0; r < m; ++r) Kx[pr.kdiag_z[r]] = -rinv[r];
  for (int e = 0; e < nnz; ++e) Kx[pr.kA[e]] = A[e];
  OsqpInfo info{UNSOLVED, 0, 0.0, 0.0};
  if (!ldl_numeric(pr.kkt, w.ldl)) {
    info.status = NON_CVX;
  }
  double* x = st.x.data();
  double* z = st.z.data();
  double* y = st.y.data();
  double* xt = w.xt.data();
  double* zt = w.zt.data();
  double* dxv = w.dx.data();
  double* dyv = w.dy.data();
  double* rhs = w.sol.data();
  const double sig = S.sigma, al = S.alpha;
  auto compute_info = [&](double& pri, double& dua, double& nz, double& nax, double& nq, double& naty, double& npx) {
    double* Axv = w.Axv.data();
    double* Aty = w.Aty.data();
    for (int r = 0; r < m; ++r) Axv[r] = 0.0;
    for (int j = 0; j < n; ++j) {
      double s2 = 0.0;
      for (int q2 = pr.Ap[j]; q2 < pr.Ap[j + 1]; ++q2) {
        Axv[pr.Ai[q2]] += A[q2] * x[j];
        s2 += A[q2] * y[pr.Ai[q2]];
      }
      Aty[j] = s2;
    }
    pri = 0.0; nz = 0.0; nax = 0.0;
    for (int r = 0; r < m; ++r) {
      const double ei = 1.0 / E[r];
      pri = fmax(pri, fabs(ei * (Axv[r] - z[r])));
      nz = fmax(nz, fabs(ei * z[r]));
      nax = fmax(nax, fabs(ei * Axv[r]));
    }
    dua = 0.0; nq = 0.0; naty = 0.0; npx = 0.0;
    for (int j = 0; j < n; ++j) {
      const double di = 1.0 / D[j];
      const double px = P[j] * x[j];
      dua = fmax(dua, fabs(di * (q[j] + px + Aty[j])));
      nq = fmax(nq, fabs(di * q[j]));
      naty = fmax(naty, fabs(di * Aty[j]));
      npx = fmax(npx, fabs(di * px));
    }
    dua *= cinv;
  };
  auto check = [&](double pri, double dua, double nz, double nax, double nq, double naty, double npx,
                   bool approx) -> int {
    const double mul = approx ? 10.0 : 1.0;
    const double ea = S.eps_abs * mul, er = S.eps_rel * mul, epi = S.eps_pinf * mul, edi = S.eps_dinf * mul;
    if (pri > OSQP_INFTY || dua > OSQP_INFTY) return NON_CVX;
    const double eps_prim = ea + er * fmax(nz, nax);
    const bool prim_ok = pri < eps_prim;
    bool prim_inf = false, dual_inf = false;
    if (!prim_ok) {  // primal infeasibility certificate
      const double big = OSQP_INFTY * MIN_SCALING;
      double ndy = 0.0, ineq = 0.0;
      for (int r = 0; r < m; ++r) {
        double d2 = dyv[r];
        const bool ui = us[r] > big, li = ls[r] < -big;
        if (ui && li) d2 = 0.0;
        else if (ui) d2 = fmin(d2, 0.0);
        else if (li) d2 = fmax(d2, 0.0);
        w.buf[r] = d2;
        ndy = fmax(ndy, fabs(E[r] * d2));
      }
      if (ndy > DIV_TOL) {
        for (int r = 0; r < m; ++r) ineq += us[r] * fmax(w.buf[r], 0.0) + ls[r] * fmin(w.buf[r], 0.0);
        if (ineq < epi * ndy) {
          double nat = 0.0;
          for (int j = 0; j < n; ++j) {
            double s2 = 0.0;
            for (int q2 = pr.Ap[j]; q2 < pr.Ap[j + 1]; ++q2) s2 += A[q2] * w.buf[pr.Ai[q2]];
            nat = fmax(nat, fabs(s2 / D[j]));
          }
          prim_inf = nat < epi * ndy;
        }
      }
    }
    const double eps_dual = ea + er * cinv * fmax(nq, fmax(naty, npx));
    const bool dual_ok = dua < eps_dual;
    if (!dual_ok) {  // dual infeasibility certificate
      double ndx = 0.0, qdx = 0.0, npdx = 0.0;
      for (int j = 0; j < n; ++j) {
        ndx = fmax(ndx, fabs(D[j] * dxv[j]));
        qdx += q[j] * dxv[j];
        npdx = fmax(npdx, fabs(P[j] * dxv[j] / D[j]));
      }
      if (ndx > DIV_TOL && qdx < c * edi * ndx && npdx < c * edi * ndx) {
        double* Adx = w.Axv.data();
        for (int r = 0; r < m; ++r) Adx[r] = 0.0;
        for (int j = 0; j < n; ++j)
          for (int q2 = pr.Ap[j]; q2 < pr.Ap[j + 1]; ++q2) Adx[pr.Ai[q2]] += A[q2] * dxv[j];
        const double big = OSQP_INFTY * MIN_SCALING;
        bool bad = false;
        for (int r = 0; r < m; ++r) {
          const double a = Adx[r] / E[r];
          if ((us[r] < big && a > edi * ndx) || (ls[r] > -big && a < -edi * ndx)) bad = true;
        }
        dual_inf = !bad;
      }
    }
    if (prim_ok && dual_ok) return approx ? SOLVED_INACC : SOLVED;
    if (prim_inf) return approx ? PRIM_INF_INACC : PRIM_INF;
    if (dual_inf) return approx ? DUAL_INF_INACC : DUAL_INF;
    return UNSOLVED;
  };
  double pri = 0, dua = 0, nz = 0, nax = 0, nq = 0, naty = 0, npx = 0;
  bool can_check = false;
  int it = 0;
  if (info.status == UNSOLVED) {
    for (it = 1; it <= S.max_iter; ++it) {
      // rhs = [sigma x - q; z - rho^-1 y] in the KKT ordering
      for (int j = 0; j < n; ++j) rhs[pr.perm_x[j]] = sig * x[j] - q[j];
      for (int r = 0; r < m; ++r) rhs[pr.perm_z[r]] = z[r] - rinv[r] * y[r];
      ldl_solve(pr.kkt, w.ldl, rhs);
      for (int j = 0; j < n; ++j) {
        xt[j] = rhs[pr.perm_x[j]];
        const double xn = al * xt[j] + (1.0 - al) * x[j];
        dxv[j] = xn - x[j];
        x[j] = xn;
      }
      for (int r = 0; r < m; ++r) {
        zt[r] = (z[r] - rinv[r] * y[r]) + rinv[r] * rhs[pr.perm_z[r]];
        const double zr = al * zt[r] + (1.0 - al) * z[r];
        const double zn = fmin(fmax(zr + rinv[r] * y[r], ls[r]), us[r]);
        dyv[r] = rho[r] * (zr - zn);
        y[r] += dyv[r];
        z[r] = zn;
      }
      can_check = S.check_termination > 0 && it % S.check_termination == 0;
      if (can_check) {
        compute_info(pri, dua, nz, nax, nq, naty, npx);
        info.status = check(pri, dua, nz, nax, nq, naty, npx, false);
        if (info.status != UNSOLVED) break;
      }
    }
    if (it > S.max_iter) it = S.max_iter;
    if (!can_check) {
      compute_info(pri, dua, nz, nax, nq, naty, npx);
      info.status = check(pri, dua, nz, nax, nq, naty, npx, false);
    }
    if (info.status == UNSOLVED) {
      const int s2 = check(pri, dua, nz, nax, nq, naty, npx, true);
      info.status = s2 != UNSOLVED ? s2 : MAX_ITER;
    }
  }
  info.iter = it;
  info.pri = pri;
  info.dua = dua;
  const bool bad = info.status == PRIM_INF || info.status == PRIM_INF_INACC || info.status == DUAL_INF ||
                   info.status == DUAL_INF_INACC || info.status == NON_CVX;
  for (int j = 0; j < n; ++j) {
    w.step[j] = bad ? NAN : D[j] * x[j];
    if (bad) x[j] = 0.0;
  }
  if (bad)
    for (int r = 0; r < m; ++r) { z[r] = 0.0; y[r] = 0.0; }
  return info;
}

// ---------------------------------------------------------------- one SQP iteration
struct StepStats {
  int status, iter, branch, trials, accepted;
  double alpha, viol_max;
};

template <int DYN>
StepStats sqp_step(const Problem& pr, Work& w, OsqpState& st, const double* p, const double* Pd, double* x) {
  const int n = pr.n, m = pr.m;
  const double f0 = objective(pr, p, x, nullptr, 0.0, w.grad.data());
  eval_values<DYN>(pr, p, x, nullptr, 0.0, w.g.data(), w.lbg.data(), w.ubg.data());
  eval_jac<DYN>(pr, p, x, w, w.Ax.data());
  for (int r = 0; r < m; ++r) { w.lbg[r] -= w.g[r]; w.ubg[r] -= w.g[r]; }  // l - g, u - g (ocp.py:395)
  OsqpInfo oi = osqp_update_solve(pr, w, st, Pd, w.grad.data(), w.Ax.data(), w.lbg.data(), w.ubg.data());
  StepStats s{oi.status, oi.iter, 0, 0, 0, 0.0, 0.0};
  const double* dxs = w.step.data();
  bool nan_step = false;
  for (int j = 0; j < n; ++j) nan_step |= std::isnan(dxs[j]);
  // _armijo_line_search (ocp.py:430-480), incl. f / g_metric overwritten by every trial
  double f = f0, gm, vmax0;
  violation<DYN>(pr, p, x, nullptr, 0.0, &gm, &vmax0);
  double arm = 0.0;
  for (int j = 0; j < n; ++j) arm += w.grad[j] * dxs[j];
  const double armijo_factor = 1e-4, a_min = 1e-4, a_decay = 0.5, g_max = 1e-3, g_min = 1e-5, gamma = 1e-5;
  double a = 1.0, new_f = f, new_gm = gm, vmax = vmax0;
  bool accepted = false;
  int branch = 0, trials = 0;
  if (nan_step) {
    trials = 14;
  } else {
    while (!accepted && a > a_min) {
      new_f = objective(pr, p, x, dxs, a, nullptr);
      violation<DYN>(pr, p, x, dxs, a, &new_gm, &vmax);
      ++trials;
      if (new_gm > g_max) {
        if (new_gm < (1.0 - gamma) * gm) { accepted = true; branch = 1; }
      } else if (fmax(new_gm, gm) < g_min && arm < 0.0) {
        if (new_f <= f + armijo_factor * arm) { accepted = true; branch = 2; }
      } else if (new_f <= f - gamma * new_gm || new_gm < (1.0 - gamma) * gm) {
        accepted = true;
        branch = 3;
      }
      a *= a_decay;
      f = new_f;
      gm = new_gm;
    }
  }
  const double a_acc = a / a_decay;
  if (accepted)
    for (int j = 0; j < n; ++j) x[j] = x[j] + a_acc * dxs[j];
  s.accepted = accepted;
  s.branch = branch;
  s.trials = trials;
  s.alpha = accepted ? a_acc : 0.0;
  s.viol_max = accepted ? vmax : vmax0;
  return s;
}

// Constant Hessian diagonal (ocp.py:293-296).
void hess_diag(const Problem& pr, const double* p, double* Pd) {
  const PlOcpConst& O = pr.O;
  for (int j = 0; j < pr.n; ++j) {
    const int i = pr.colnode[j], lc = j - pr.x_off[i];
    double h;
    if (lc < O.ndx) {
      h = 2.0 * p[O.P.Q_diag + lc];
    } else {
      const int k = lc - O.ndx;
      h = 2.0 * p[O.P.R_diag + k];
      if (PL_IS_RNEA(O.dyn) && i == 0 && k >= O.na + O.nf) h += 2.0 * p[O.P.W_diag + k - O.na - O.nf];
    }
    Pd[j] = h;
  }
}

// MPC step k (k_mpc_prepare / k_mpc_finish): parameters, warm start, solve, state update.
template <int DYN>
StepStats mpc_step(const Problem& pr, Work& w, OsqpState& st, double* p, const double* Pd, double* x, double* xs,
                   double t0, int k) {
  const PlOcpConst& O = pr.O;
  for (int j = 0; j < O.nx; ++j) p[O.P.x_init + j] = xs[j];
  pl::gait_schedule(O, pr.S.gait_type, pr.S.gait_period, pr.S.swing_period, t0 + k * p[O.P.dt_min], p,
                    p + O.P.contact, p + O.P.swing);
  if (k > 0) {
    const int fo = pl::u_force_off(O);
    for (int i = 0; i < pr.N; ++i) {
      const int base = pr.x_off[i] + O.ndx + fo;
      for (int c = 0; c < O.nf; ++c) {
        double fd = pl::f_des_comp(pr.M, O, p, c);
        if (c / 3 < 4 && p[O.P.contact + 4 * i + c / 3] == 0.0) fd = 0.0;
        x[base + c] = fd;
      }
    }
  }
  StepStats s = sqp_step<DYN>(pr, w, st, p, Pd, x);
  const double* dx1 = x + pr.x_off[1];
  double qn[PL_MAXQ];
  if (PL_IS_CV(O.dyn)) {
    pl::VecIn<double> acc{dx1 + 6, nullptr, 0.0, -1};
    pl::integrate_q<double>(pr.M, xs + 6, acc, qn);
    for (int j = 0; j < 6; ++j) xs[j] += dx1[j];
    for (int j = 0; j < O.nq; ++j) xs[6 + j] = qn[j];
  } else {
    pl::VecIn<double> acc{dx1, nullptr, 0.0, -1};
    pl::integrate_q<double>(pr.M, xs, acc, qn);
    for (int j = 0; j < O.nq; ++j) xs[j] = qn[j];
    for (int j = 0; j < O.nv; ++j) xs[O.nq + j] += dx1[O.nv + j];
  }
  return s;
}

template <int DYN>
void run_problem(const Problem& pr, Work& w, const double* P0, const double* X0, const double* XS0, double t0,
                 int steps, double* xs_out, int* stats_out) {
  std::vector<double> p(P0, P0 + pr.np), x(X0, X0 + pr.n), xs(XS0, XS0 + pr.O.nx), Pd(pr.n);
  OsqpState st;
  st.x.assign(pr.n, 0.0);
  st.z.assign(pr.m, 0.0);
  st.y.assign(pr.m, 0.0);
  hess_diag(pr, p.data(), Pd.data());  // init_solver (excluded from nothing: cheap)
  for (int k = 0; k < steps; ++k) {
    StepStats s = mpc_step<DYN>(pr, w, st, p.data(), Pd.data(), x.data(), xs.data(), t0, k);
    if (stats_out) {
      int* o = stats_out + 4 * k;
      o[0] = s.status; o[1] = s.iter; o[2] = s.branch; o[3] = s.trials;
    }
  }
  for (int j = 0; j < pr.O.nx; ++j) xs_out[j] = xs[j];
}


// ---------------------------------------------------------------- interior point (Fatrop branch)
// A compiled restatement of oracle/ip_ref.py (the IPOPT-style primal-dual barrier method
// with a filter line search that stands in for Fatrop, run_mpc.py:34-37, ocp.py:248-263,
// 360-373): same settings, slack formulation, reduced Newton system, inertia correction,
// monotone barrier rule, filter line search and termination.  The Newton system is solved
// through the quasi-definite KKT [H + H_L + d_w I, J^T; J, -W^-1] by the QDLDL LDL^T (the
// reduced matrix H + H_L + d_w I + J^T W J is positive definite iff the KKT has exactly n
// positive pivots, Sylvester's law of inertia); H_L = sum_r lam_r d^2 g_r / dw_i^2 by
// hyper-dual node passes over the structurally non-zero column pairs of each w_i block (the
// same technique as the GPU's k_lag_hess).  Fatrop itself is not available: this is a
// restatement, timed as the CPU baseline of bench.py --solver fatrop.
constexpr double IP_KAPPA_EPS = 10.0, IP_KAPPA_MU = 0.2, IP_THETA_MU = 1.5, IP_TAU_MIN = 0.99, IP_S_MAX = 100.0;
constexpr double IP_KAPPA_SIGMA = 1e10, IP_GAMMA_THETA = 1e-5, IP_GAMMA_PHI = 1e-8, IP_DELTA = 1.0, IP_S_THETA = 1.1;
constexpr double IP_S_PHI = 2.3, IP_ETA_PHI = 1e-8, IP_W_MIN = 1e-20;
enum { IP_CONVERGED = 1, IP_MAX_ITER = -1, IP_LS_FAIL = -2, IP_NONFINITE = -3 };

struct IpSettings {
  double tol, mu_init, bound_push, bound_frac, warm_push, delta_w, delta_c;
  int max_iter, ls_max, n_refine, inertia_cap;
  int kkt_exact;  // 1: refinement on the unregularised KKT (ip_ref.py kkt_refine="exact"), 0: "regularized"
  int mpc_lam;    // MPC loop: 1 carries lam_g across steps (the Opti branch), 0 cold multipliers per solve
                  // (the reference's default compiled-solver driver, run_mpc.py:34-37, 50-111)
};

struct HEmit {
  const double* lam;
  double acc;
  int r;
  void operator()(const HDual& v, double, double) {
    acc = fma(lam[r], v.c, acc);
    ++r;
  }
};

template <int DYN>
void probe_pairs(const Problem& pr, int i, std::vector<std::pair<int, int>>& out) {
  const PlOcpConst& O = pr.O;
  uint64_t st = 0x2545f4914f6cdd1dull ^ (uint64_t)(i + 7);
  auto rnd = [&]() {  // uniform in (0.5, 1.5)
    st ^= st >> 12; st ^= st << 25; st ^= st >> 27;
    return 0.5 + (double)((st * 0x2545f4914f6cdd1dull) >> 11) / 9007199254740992.0;
  };
  std::vector<double> p(O.P.np);
  for (double& v : p) v = rnd();
  p[O.P.dt_min] = 0.02;
  p[O.P.dt_max] = 0.05;
  for (int k = 0; k < 4 * O.N; ++k) { p[O.P.contact + k] = 0.5; p[O.P.swing + k] = 0.3; }
  p[O.P.n_contacts] = 2.0;
  p[O.P.swing_period] = 0.4;
  p[O.P.swing_vel_limits + 1] = -0.2;
  const int qo = PL_IS_CV(O.dyn) ? 9 : 3;
  double qn = 0.0;
  for (int k = 0; k < 4; ++k) qn += p[O.P.x_init + qo + k] * p[O.P.x_init + qo + k];
  for (int k = 0; k < 4; ++k) p[O.P.x_init + qo + k] /= sqrt(qn);
  const int nw = pr.nw[i], ndx = O.ndx;
  std::vector<double> xw(nw + ndx), lam(pr.nrow[i]);
  for (double& v : xw) v = 0.2 * (rnd() - 1.0);
  for (size_t r = 0; r < lam.size(); ++r) lam[r] = (r & 1) ? rnd() : -rnd();
  HDual kst[PL_KIN_STORE];
  out.clear();
  for (int k = 0; k < nw; ++k)
    for (int j = 0; j <= k; ++j) {
      pl::VecIn<HDual> dx{xw.data(), nullptr, 0.0, j, k};
      pl::VecIn<HDual> u{xw.data() + ndx, nullptr, 0.0, j - ndx, k - ndx};
      pl::VecIn<HDual> dxn{xw.data() + nw, nullptr, 0.0, j - nw, k - nw};
      HEmit e{lam.data(), 0.0, 0};
      pl::node_rows<HDual, DYN>(pr.M, O, i, p.data(), dx, u, dxn, e, kst, 1);
      if (e.acc != 0.0) out.push_back({j, k});
    }
}

// whole_body_rnea: the (dq, a) and (dq, f_feet) blocks of node i from two dual tree passes per
// dq column (d/dq_k of M(q) lambda_tau and of -J_e(q) lambda_tau; the same restatement of the
// linearity in a and f as the GPU's k_lag_hess_lin).  lin[k * nlin + c] for the columns
// c = 0 .. na + 3 nfeet - 1 after dx.
struct ZeroInH {
  Dual operator[](int) const { return Dual(0.0, 0.0); }
};
struct LamInH {
  const double* lb;
  const double* lt;
  Dual operator[](int k) const { return Dual(k < 6 ? lb[k] : (lt ? lt[k - 6] : 0.0), 0.0); }
};
void rnea_lin_block(const Problem& pr, const PlModel& M0, const double* p, const double* x, const double* lam, int i,
                    double* lin) {
  const PlOcpConst& O = pr.O;
  const int t = pl::node_type(O, i);
  int rbb = -1, rbt = -1, r = 0;
  for (int bi = 0; bi < O.nblk[t]; ++bi) {
    if (O.blk[t][bi].kind == PL_RB_RNEA_BASE) rbb = r;
    if (O.blk[t][bi].kind == PL_RB_TAU_EQ) rbt = r;
    r += O.blk[t][bi].count;
  }
  const double* ln = lam + pr.row_off[i];
  const LamInH lt{ln + rbb, rbt >= 0 ? ln + rbt : nullptr};
  const double* xi = p + O.P.x_init;
  const int nv = O.nv, nlin = O.na + 3 * O.nfeet;
  Dual kst[PL_KIN_STORE];
  for (int k = 0; k < nv; ++k) {
    double* row = lin + (size_t)k * nlin;
    if (k < 3) {  // RNEA and the foot velocities ignore the base position
      for (int c = 0; c < nlin; ++c) row[c] = 0.0;
      continue;
    }
    const pl::VecIn<Dual> dq{x + pr.x_off[i], nullptr, 0.0, k};
    Dual qb[7];
    pl::integrate_ff<Dual>(xi, dq, qb);
    const pl::RevQ<Dual, pl::VecIn<Dual>> qrev{xi, dq};
    pl::NodeKin<Dual> kin;
    kin.vst = reinterpret_cast<double*>(kst);
    kin.dst = kin.vst + 1;
    kin.vstride = kin.dstride = 2;
    pl::tree_pass<Dual>(M0, O, qb, qrev, ZeroInH{}, lt, ZeroInH{}, true, false, kin);
    for (int j = 0; j < nv; ++j) row[j] = j < 6 ? kin.tau[j].d : Dual(kin.tau_j(j - 6)).d;
    pl::tree_pass<Dual>(pr.M, O, qb, qrev, lt, ZeroInH{}, ZeroInH{}, false, true, kin);
    for (int e = 0; e < O.nfeet; ++e)
      for (int c = 0; c < 3; ++c) row[O.na + 3 * e + c] = -Dual(kin.foot_vel(e, c)).d;
  }
}

// H_L blocks at (x, lam): hv[pair] = sum_r lam_r g_r.c over the node's rows (whole_body_rnea:
// the (dq, a) / (dq, f_feet) pairs from rnea_lin_block instead)
template <int DYN>
void lag_hess(const Problem& pr, const double* p, const double* x, const double* lam, double* hv) {
  HDual kst[PL_KIN_STORE];
  const int ndx = pr.O.ndx;
  const bool lin = DYN == PL_DYN_RNEA;
  const int nlin = pr.O.na + 3 * pr.O.nfeet;
  std::vector<double> linb(lin ? (size_t)pr.O.nv * nlin : 0);
  PlModel M0 = pr.M;
  for (int k = 0; k < 3; ++k) M0.gravity[k] = 0.0;
  for (int i = 0; i < pr.N; ++i) {
    const auto& pl_ = pr.hpairs[pl::node_type(pr.O, i)];
    const int xo = pr.x_off[i], xn = pr.x_off[i + 1], nw = pr.nw[i];
    if (lin) rnea_lin_block(pr, M0, p, x, lam, i, linb.data());
    for (size_t q = 0; q < pl_.size(); ++q) {
      const int j = pl_[q].first, k = pl_[q].second;
      if (lin && j < pr.O.nv && k >= ndx && k < ndx + nlin) {
        hv[pr.ik_H_off[i] + q] = linb[(size_t)j * nlin + (k - ndx)];
        continue;
      }
      pl::VecIn<HDual> dx{x + xo, nullptr, 0.0, j, k};
      pl::VecIn<HDual> u{x + xo + ndx, nullptr, 0.0, j - ndx, k - ndx};
      pl::VecIn<HDual> dxn{x + xn, nullptr, 0.0, j - nw, k - nw};
      HEmit e{lam + pr.row_off[i], 0.0, 0};
      pl::node_rows<HDual, DYN>(pr.M, pr.O, i, p, dx, u, dxn, e, kst, 1);
      hv[pr.ik_H_off[i] + q] = e.acc;
    }
  }
}

template <int DYN>
void ip_prepare(Problem& pr) {
  const int n = pr.n, m = pr.m, N = pr.N;
  for (int i = 0; i < N; ++i) {
    const int t = pl::node_type(pr.O, i);
    if (pr.hpairs[t].empty()) probe_pairs<DYN>(pr, i, pr.hpairs[t]);
  }
  // KKT pattern: diagonal + A plus the H_L pairs, in a rows-first order: per node its rows
  // (pivots -1 / W_r), then its variables.  Eliminating the rows first adds W_r J_r^T J_r to the
  // variables, so their pivots are those of the reduced SPD matrix H + H_L + J^T W J the oracle
  // factors (oracle/ip_ref.py).  The OSQP branch's variables-first order put the objective's
  // diagonal (down to delta_w = 1e-8 on the unweighted base coordinates) first: its pivots
  // lost the directions' accuracy (1e-3 at B2G's first iteration) and the inertia count
  // (shifts of 1e6 where the reduced matrix is positive definite), so the restatement failed
  // line searches the oracle and the GPU pass (17 of 64 headline problems, r05).
  pr.iperm_x.assign(n, 0);
  pr.iperm_z.assign(m, 0);
  {
    int idx = 0;
    for (int i = 0; i <= N; ++i) {
      const int nri = pr.nrow[i];
      for (int r = 0; r < nri; ++r) pr.iperm_z[pr.row_off[i] + r] = idx++;
      if (i == 0) {  // the initial rows DX_0 = 0 (before node 0's own rows in g)
        for (int r = 0; r < pr.row_off[0]; ++r) pr.iperm_z[r] = idx++;
      }
      for (int c = 0; c < pr.nw[i]; ++c) pr.iperm_x[pr.x_off[i] + c] = idx++;
    }
  }
  Kkt& kk = pr.ipk;
  kk.K = n + m;
  std::vector<std::vector<std::pair<int, int>>> cols(kk.K);  // (row, tag)
  for (int j = 0; j < n; ++j) cols[pr.iperm_x[j]].push_back({pr.iperm_x[j], -1 - j});
  for (int r = 0; r < m; ++r) cols[pr.iperm_z[r]].push_back({pr.iperm_z[r], -1 - n - r});
  for (int j = 0; j < n; ++j)
    for (int k = pr.Ap[j]; k < pr.Ap[j + 1]; ++k) {
      const int a = pr.iperm_x[j], b = pr.iperm_z[pr.Ai[k]];
      cols[std::max(a, b)].push_back({std::min(a, b), k});
    }
  const int tagH = 1 << 30;  // pair tags: tagH + running pair index
  pr.ik_H_off.assign(N + 1, 0);
  int npair = 0;
  for (int i = 0; i < N; ++i) {
    pr.ik_H_off[i] = npair;
    for (auto& jk : pr.hpairs[pl::node_type(pr.O, i)]) {
      const int a = pr.iperm_x[pr.x_off[i] + jk.first], b = pr.iperm_x[pr.x_off[i] + jk.second];
      cols[std::max(a, b)].push_back({std::min(a, b), tagH + npair});
      ++npair;
    }
  }
  pr.ik_H_off[N] = npair;
  pr.ik_H.assign(npair, 0);
  pr.ik_diag_x.assign(n, 0);
  pr.ik_diag_z.assign(m, 0);
  pr.ik_A.assign(pr.nnz, 0);
  kk.Kp.assign(kk.K + 1, 0);
  kk.Ki.clear();
  for (int c = 0; c < kk.K; ++c) {
    std::sort(cols[c].begin(), cols[c].end());
    int last = -1, slot = -1;
    for (auto& e : cols[c]) {
      if (e.first != last) {  // a diagonal pair (j, j) shares the (x_j, x_j) slot
        slot = (int)kk.Ki.size();
        kk.Ki.push_back(e.first);
        last = e.first;
      }
      if (e.second >= tagH) pr.ik_H[e.second - tagH] = slot;
      else if (e.second >= 0) pr.ik_A[e.second] = slot;
      else if (-1 - e.second < n) pr.ik_diag_x[-1 - e.second] = slot;
      else pr.ik_diag_z[-1 - e.second - n] = slot;
    }
    kk.Kp[c + 1] = (int)kk.Ki.size();
  }
  ldl_symbolic(kk);
  pr.ip_ready = true;
}

struct IpStats {
  int status, iter, trials;
  double err, f;
};

struct IpWork {
  LdlWork ldl;
  std::vector<double> g, lbg, ubg, grad, gt, lt, ut, J, H, s, sl, su, zl, zu, lam, c, rx, W, bs, rhat, rhs, dx, dl, ds,
      dzl, dzu, sol, jdx, res, xt, st, tmp, hv;
  std::vector<char> eq, hl, hu;
  void init(const Problem& pr) {
    const int n = pr.n, m = pr.m;
    ldl.init(pr.ipk);
    for (auto* v : {&g, &lbg, &ubg, &gt, &lt, &ut, &s, &sl, &su, &zl, &zu, &lam, &c, &W, &bs, &rhat, &dl, &ds, &dzl,
                    &dzu, &jdx, &st})
      v->assign(m, 0.0);
    for (auto* v : {&grad, &H, &rhs, &dx, &res, &xt, &tmp, &rx}) v->assign(n, 0.0);
    J.assign(pr.nnz, 0.0);
    sol.assign(pr.ipk.K, 0.0);
    hv.assign(pr.ik_H_off.back(), 0.0);
    eq.assign(m, 0);
    hl.assign(m, 0);
    hu.assign(m, 0);
  }
};

// J (CSC over pr.Ap / pr.Ai) products
void jt_mul(const Problem& pr, const double* J, const double* v, double* out) {  // out = J^T v
  for (int j = 0; j < pr.n; ++j) {
    double a = 0.0;
    for (int q = pr.Ap[j]; q < pr.Ap[j + 1]; ++q) a += J[q] * v[pr.Ai[q]];
    out[j] = a;
  }
}
void j_mul(const Problem& pr, const double* J, const double* v, double* out) {  // out = J v
  for (int r = 0; r < pr.m; ++r) out[r] = 0.0;
  for (int j = 0; j < pr.n; ++j)
    for (int q = pr.Ap[j]; q < pr.Ap[j + 1]; ++q) out[pr.Ai[q]] += J[q] * v[j];
}

// fraction to the boundary: max alpha in (0, 1] with v + alpha dv >= (1 - tau) v on the mask
double ftb(const std::vector<double>& v, const std::vector<double>& dv, double sgn, double tau,
           const std::vector<char>& mask) {
  double a = 1.0;
  for (size_t r = 0; r < v.size(); ++r)
    if (mask[r] && sgn * dv[r] < 0) a = std::min(a, -tau * v[r] / (sgn * dv[r]));
  return a;
}

// One interior-point solve from x (in / out); lam (in / out) is the lam_g warm start when warm.
template <int DYN>
IpStats ip_solve(const Problem& pr, Work& w, IpWork& iw, const IpSettings& S, const double* p, const double* Pd,
                 double* x, double* lam_io, bool warm) {
  const int n = pr.n, m = pr.m;
  double mu = S.mu_init;
  const double tol = S.tol, dc = S.delta_c;
  double dw_last = 0.0;
  std::vector<double>& H = iw.H;
  for (int j = 0; j < n; ++j) H[j] = Pd[j] + S.delta_w;
  eval_values<DYN>(pr, p, x, nullptr, 0.0, iw.g.data(), iw.lbg.data(), iw.ubg.data());
  const double* lbg = iw.lbg.data();
  const double* ubg = iw.ubg.data();
  auto& eq = iw.eq;
  auto& hl = iw.hl;
  auto& hu = iw.hu;
  int nb = 0;
  for (int r = 0; r < m; ++r) {
    eq[r] = lbg[r] == ubg[r];
    hl[r] = !eq[r] && std::isfinite(lbg[r]);
    hu[r] = !eq[r] && std::isfinite(ubg[r]);
    nb += hl[r] + hu[r];
  }
  auto lbv = [&](int r) { return hl[r] ? lbg[r] : 0.0; };
  auto ubv = [&](int r) { return hu[r] ? ubg[r] : 0.0; };
  // slacks pushed into the interior (push_slacks)
  for (int r = 0; r < m; ++r) {
    const double lb = lbv(r), ub = ubv(r);
    double pl_ = S.bound_push * fmax(1.0, fabs(lb)), pu = S.bound_push * fmax(1.0, fabs(ub));
    if (hl[r] && hu[r]) {
      pl_ = fmin(pl_, S.bound_frac * (ub - lb));
      pu = fmin(pu, S.bound_frac * (ub - lb));
    }
    double sv = iw.g[r];
    if (hl[r]) sv = fmax(sv, lb + pl_);
    if (hu[r]) sv = fmin(sv, ub - pu);
    iw.s[r] = eq[r] ? 0.0 : sv;
    iw.sl[r] = hl[r] ? iw.s[r] - lb : 1.0;
    iw.su[r] = hu[r] ? ub - iw.s[r] : 1.0;
  }
  double* lam = iw.lam.data();
  for (int r = 0; r < m; ++r) {
    if (!warm) {
      lam[r] = 0.0;
      iw.zl[r] = hl[r] ? mu / iw.sl[r] : 0.0;
      iw.zu[r] = hu[r] ? mu / iw.su[r] : 0.0;
    } else {
      lam[r] = lam_io[r];
      iw.zl[r] = hl[r] ? fmax(fmax(-lam[r], 0.0), S.warm_push) : 0.0;
      iw.zu[r] = hu[r] ? fmax(fmax(lam[r], 0.0), S.warm_push) : 0.0;
    }
  }
  auto cval = [&](const double* g, const double* s_, int r) { return eq[r] ? g[r] - (eq[r] ? lbg[r] : 0.0) : g[r] - s_[r]; };
  double theta0 = 0.0;
  for (int r = 0; r < m; ++r) theta0 += fabs(cval(iw.g.data(), iw.s.data(), r));
  const double theta_max = 1e4 * fmax(1.0, theta0), theta_min = 1e-4 * fmax(1.0, theta0);
  auto phi_of = [&](double f, const double* sl, const double* su) {
    double a = 0.0, b = 0.0;
    for (int r = 0; r < m; ++r) if (hl[r]) a += log(sl[r]);
    for (int r = 0; r < m; ++r) if (hu[r]) b += log(su[r]);
    return f - mu * (a + b);
  };
  std::vector<std::pair<double, double>> filt;
  static const bool ip_debug = getenv("CPU_IP_DEBUG") != nullptr;  // per-trial trace (debugging aid)
  IpStats out{IP_MAX_ITER, 0, 0, INFINITY, NAN};
  double f = NAN, err = INFINITY;
  for (int k = 0; k <= S.max_iter; ++k) {
    out.iter = k;
    f = objective(pr, p, x, nullptr, 0.0, iw.grad.data());
    eval_values<DYN>(pr, p, x, nullptr, 0.0, iw.g.data(), iw.lt.data(), iw.ut.data());
    eval_jac<DYN>(pr, p, x, w, iw.J.data());
    for (int r = 0; r < m; ++r) iw.c[r] = cval(iw.g.data(), iw.s.data(), r);
    jt_mul(pr, iw.J.data(), lam, iw.rx.data());
    for (int j = 0; j < n; ++j) iw.rx[j] += iw.grad[j];
    double sum_lam = 0.0, sum_z = 0.0;
    for (int r = 0; r < m; ++r) { sum_lam += fabs(lam[r]); sum_z += iw.zl[r] + iw.zu[r]; }
    const double sd = fmax(IP_S_MAX, (sum_lam + sum_z) / std::max(m + nb, 1)) / IP_S_MAX;
    const double sc = fmax(IP_S_MAX, sum_z / std::max(nb, 1)) / IP_S_MAX;
    auto nlp_err = [&](double mu_) {
      double comp = 0.0, erx = 0.0, ers = 0.0, ec = 0.0;
      for (int r = 0; r < m; ++r) {
        if (hl[r]) comp = fmax(comp, fabs(iw.sl[r] * iw.zl[r] - mu_));
        if (hu[r]) comp = fmax(comp, fabs(iw.su[r] * iw.zu[r] - mu_));
        if (!eq[r]) ers = fmax(ers, fabs(-lam[r] - iw.zl[r] + iw.zu[r]));
        ec = fmax(ec, fabs(iw.c[r]));
      }
      for (int j = 0; j < n; ++j) erx = fmax(erx, fabs(iw.rx[j]));
      return fmax(fmax(erx / sd, ers / sd), fmax(ec, comp / sc));
    };
    err = nlp_err(0.0);
    if (!std::isfinite(err)) { out.status = IP_NONFINITE; break; }
    if (err <= tol) { out.status = IP_CONVERGED; break; }
    if (k == S.max_iter) { out.status = IP_MAX_ITER; break; }
    for (int t = 0; t < 4; ++t) {  // monotone barrier update
      if (nlp_err(mu) > IP_KAPPA_EPS * mu) break;
      const double mu_new = fmax(tol / 10.0, fmin(IP_KAPPA_MU * mu, pow(mu, IP_THETA_MU)));
      if (mu_new == mu) break;
      mu = mu_new;
      filt.clear();
    }
    // reduced Newton system through the quasi-definite KKT
    for (int r = 0; r < m; ++r) {
      const double sig = (hl[r] ? iw.zl[r] / iw.sl[r] : 0.0) + (hu[r] ? iw.zu[r] / iw.su[r] : 0.0);
      double Wr = eq[r] ? 1.0 / dc : sig / (1.0 + dc * sig);
      iw.W[r] = fmax(Wr, IP_W_MIN);
      iw.bs[r] = eq[r] ? 0.0 : lam[r] + (hl[r] ? mu / iw.sl[r] : 0.0) - (hu[r] ? mu / iw.su[r] : 0.0);
      const double sig_safe = eq[r] ? 1.0 : sig;
      iw.rhat[r] = eq[r] ? iw.c[r] : iw.c[r] - iw.bs[r] / sig_safe;
    }
    std::vector<double>& Kx = iw.ldl.Kx;
    lag_hess<DYN>(pr, p, x, lam, iw.hv.data());
    auto assemble = [&](double dwi) {
      std::fill(Kx.begin(), Kx.end(), 0.0);
      for (int j = 0; j < n; ++j) Kx[pr.ik_diag_x[j]] += H[j] + dwi;
      for (int r = 0; r < m; ++r) Kx[pr.ik_diag_z[r]] = -1.0 / iw.W[r];
      for (int e = 0; e < pr.nnz; ++e) Kx[pr.ik_A[e]] = iw.J[e];
      for (size_t q = 0; q < iw.hv.size(); ++q) Kx[pr.ik_H[q]] += iw.hv[q];
    };
    auto inertia_ok = [&]() {
      if (!ldl_numeric(pr.ipk, iw.ldl)) return false;
      int pos = 0;
      for (int q = 0; q < pr.ipk.K; ++q) pos += iw.ldl.Dd[q] > 0.0;
      return pos == n;
    };
    double dwi = 0.0;
    int tries = 0;
    assemble(0.0);
    while (true) {  // inertia correction (ip_ref.py)
      if (inertia_ok()) {
        if (dwi > 0.0) dw_last = dwi;
        break;
      }
      if (tries >= S.inertia_cap) break;
      dwi = dwi == 0.0 ? (dw_last == 0.0 ? 1e-4 : fmax(1e-20, dw_last / 3.0)) : dwi * (dw_last == 0.0 ? 100.0 : 8.0);
      ++tries;
      assemble(dwi);
    }
    if (ip_debug) fprintf(stderr, " it %d: inertia shift %.3e after %d tries (dw_last %.3e) mu %.3e\n", k, dwi, tries, dw_last, mu);
    auto kkt_solve = [&](const double* r_x, double* out_x) {
      for (int j = 0; j < n; ++j) iw.sol[pr.iperm_x[j]] = r_x[j];
      for (int r = 0; r < m; ++r) iw.sol[pr.iperm_z[r]] = 0.0;
      ldl_solve(pr.ipk, iw.ldl, iw.sol.data());
      for (int j = 0; j < n; ++j) out_x[j] = iw.sol[pr.iperm_x[j]];
    };
    // H_L dx for the refinement residual: the KKT's upper-left block (H + dwi + H_L) times dx
    auto hl_mul = [&](const double* v, double* outv) {  // (H + dwi + H_L) v over the stored pairs
      for (int j = 0; j < n; ++j) outv[j] = (H[j] + dwi) * v[j];
      for (int i = 0; i < pr.N; ++i) {
        const auto& pl_ = pr.hpairs[pl::node_type(pr.O, i)];
        const int xo = pr.x_off[i];
        for (size_t q = 0; q < pl_.size(); ++q) {
          const int a = xo + pl_[q].first, b = xo + pl_[q].second;
          const double hv = iw.hv[pr.ik_H_off[i] + q];
          if (a == b) {
            outv[a] += hv * v[a];
          } else {
            outv[a] += hv * v[b];
            outv[b] += hv * v[a];
          }
        }
      }
    };
    std::vector<double> Hdx(n), corr(n);
    if (S.kkt_exact) {
      // iterative refinement on the unregularised KKT [H_K J^T; J -D] [dx; dl] = [-rx; -rhat]
      // (D = 0 on equality rows, 1/Sigma on the others) with the delta_c-regularised factor
      // [H_K J^T; J -1/W] as the solver of each correction (oracle/ip_ref.py kkt_refine="exact")
      std::vector<double> r2(m), ez(m);
      std::fill(iw.dx.begin(), iw.dx.end(), 0.0);
      std::fill(iw.dl.begin(), iw.dl.end(), 0.0);
      std::fill(iw.jdx.begin(), iw.jdx.end(), 0.0);
      for (int t = 0; t <= S.n_refine; ++t) {
        for (int r = 0; r < m; ++r) iw.st[r] = lam[r] + iw.dl[r];
        jt_mul(pr, iw.J.data(), iw.st.data(), iw.res.data());
        hl_mul(iw.dx.data(), Hdx.data());
        for (int j = 0; j < n; ++j) iw.res[j] = -(iw.grad[j] + iw.res[j]) - Hdx[j];
        for (int r = 0; r < m; ++r) {
          const double sig = (hl[r] ? iw.zl[r] / iw.sl[r] : 0.0) + (hu[r] ? iw.zu[r] / iw.su[r] : 0.0);
          const double D = eq[r] ? 0.0 : 1.0 / sig;
          r2[r] = -iw.rhat[r] - iw.jdx[r] + D * iw.dl[r];
        }
        for (int j = 0; j < n; ++j) iw.sol[pr.iperm_x[j]] = iw.res[j];
        for (int r = 0; r < m; ++r) iw.sol[pr.iperm_z[r]] = r2[r];
        ldl_solve(pr.ipk, iw.ldl, iw.sol.data());
        for (int j = 0; j < n; ++j) iw.dx[j] += iw.sol[pr.iperm_x[j]];
        for (int r = 0; r < m; ++r) iw.dl[r] += iw.sol[pr.iperm_z[r]];
        j_mul(pr, iw.J.data(), iw.dx.data(), iw.jdx.data());
      }
    } else {
      for (int r = 0; r < m; ++r) iw.st[r] = iw.W[r] * iw.rhat[r];
      jt_mul(pr, iw.J.data(), iw.st.data(), iw.rhs.data());
      for (int j = 0; j < n; ++j) iw.rhs[j] = -iw.rx[j] - iw.rhs[j];
      kkt_solve(iw.rhs.data(), iw.dx.data());
      for (int t = 0; t < S.n_refine; ++t) {
        j_mul(pr, iw.J.data(), iw.dx.data(), iw.jdx.data());
        for (int r = 0; r < m; ++r) iw.st[r] = lam[r] + iw.W[r] * (iw.jdx[r] + iw.rhat[r]);
        jt_mul(pr, iw.J.data(), iw.st.data(), iw.res.data());
        hl_mul(iw.dx.data(), Hdx.data());
        for (int j = 0; j < n; ++j) iw.res[j] = -(iw.grad[j] + iw.res[j]) - Hdx[j];
        kkt_solve(iw.res.data(), corr.data());
        for (int j = 0; j < n; ++j) iw.dx[j] += corr[j];
      }
    }
    j_mul(pr, iw.J.data(), iw.dx.data(), iw.jdx.data());
    bool finite = true;
    for (int r = 0; r < m; ++r) {
      if (!S.kkt_exact) iw.dl[r] = iw.W[r] * (iw.jdx[r] + iw.rhat[r]);
      const double sig = (hl[r] ? iw.zl[r] / iw.sl[r] : 0.0) + (hu[r] ? iw.zu[r] / iw.su[r] : 0.0);
      iw.ds[r] = eq[r] ? 0.0 : (iw.bs[r] + iw.dl[r]) / sig;
      iw.dzl[r] = hl[r] ? mu / iw.sl[r] - iw.zl[r] - iw.zl[r] / iw.sl[r] * iw.ds[r] : 0.0;
      iw.dzu[r] = hu[r] ? mu / iw.su[r] - iw.zu[r] + iw.zu[r] / iw.su[r] * iw.ds[r] : 0.0;
      finite &= std::isfinite(iw.dl[r]);
    }
    for (int j = 0; j < n; ++j) finite &= std::isfinite(iw.dx[j]);
    if (!finite) { out.status = IP_NONFINITE; break; }
    const double tau = fmax(IP_TAU_MIN, 1.0 - mu);
    const double amax = fmin(ftb(iw.sl, iw.ds, 1.0, tau, hl), ftb(iw.su, iw.ds, -1.0, tau, hu));
    const double az = fmin(ftb(iw.zl, iw.dzl, 1.0, tau, hl), ftb(iw.zu, iw.dzu, 1.0, tau, hu));
    double theta = 0.0;
    for (int r = 0; r < m; ++r) theta += fabs(iw.c[r]);
    const double phi = phi_of(f, iw.sl.data(), iw.su.data());
    double dphi = 0.0, sds = 0.0;
    for (int j = 0; j < n; ++j) dphi += iw.grad[j] * iw.dx[j];
    for (int r = 0; r < m; ++r) sds += (hl[r] ? -mu / iw.sl[r] : 0.0) * iw.ds[r] + (hu[r] ? mu / iw.su[r] : 0.0) * iw.ds[r];
    dphi += sds;
    bool accepted = false, ftype = false;
    double a = amax;
    int t = 0;
    std::vector<double> slt(m), sut(m);
    for (t = 0; t < S.ls_max; ++t) {
      a = amax * pow(0.5, t);
      const double ft = objective(pr, p, x, iw.dx.data(), a, nullptr);
      eval_values<DYN>(pr, p, x, iw.dx.data(), a, iw.gt.data(), iw.lt.data(), iw.ut.data());
      double th_t = 0.0;
      for (int r = 0; r < m; ++r) {
        const double stt = iw.s[r] + a * iw.ds[r];
        iw.st[r] = stt;
        slt[r] = hl[r] ? stt - lbv(r) : 1.0;
        sut[r] = hu[r] ? ubv(r) - stt : 1.0;
        th_t += fabs(cval(iw.gt.data(), iw.st.data(), r));
      }
      const double ph_t = phi_of(ft, slt.data(), sut.data());
      if (ip_debug) {
        double dxm = 0.0;
        for (int j = 0; j < n; ++j) dxm = fmax(dxm, fabs(iw.dx[j]));
        fprintf(stderr, "  it %d trial %d a %.3e theta %.4e -> %.4e  phi %.6e -> %.6e  dphi %.3e amax %.3e az %.3e |dx| %.3e\n",
                k, t, a, theta, th_t, phi, ph_t, dphi, amax, az, dxm);
      }
      if (!(std::isfinite(th_t) && std::isfinite(ph_t)) || th_t > theta_max) continue;
      bool dominated = false;
      for (auto& fp : filt) dominated |= th_t >= fp.first && ph_t >= fp.second;
      if (dominated) continue;
      const bool switching = dphi < 0 && a * pow(-dphi, IP_S_PHI) > IP_DELTA * pow(theta, IP_S_THETA);
      if (theta <= theta_min && switching) {
        if (ph_t <= phi + IP_ETA_PHI * a * dphi) { accepted = ftype = true; break; }
      } else if (th_t <= (1 - IP_GAMMA_THETA) * theta || ph_t <= phi - IP_GAMMA_PHI * theta) {
        accepted = true;
        break;
      }
    }
    out.trials += std::min(t + 1, S.ls_max);
    if (!accepted) { out.status = IP_LS_FAIL; break; }
    if (!ftype) filt.push_back({(1 - IP_GAMMA_THETA) * theta, phi - IP_GAMMA_PHI * theta});
    for (int j = 0; j < n; ++j) x[j] = x[j] + a * iw.dx[j];
    for (int r = 0; r < m; ++r) {
      iw.s[r] = iw.s[r] + a * iw.ds[r];
      lam[r] = lam[r] + a * iw.dl[r];
      double zl = iw.zl[r] + az * iw.dzl[r], zu = iw.zu[r] + az * iw.dzu[r];
      iw.sl[r] = hl[r] ? iw.s[r] - lbv(r) : 1.0;
      iw.su[r] = hu[r] ? ubv(r) - iw.s[r] : 1.0;
      iw.zl[r] = hl[r] ? fmin(fmax(zl, mu / (IP_KAPPA_SIGMA * iw.sl[r])), IP_KAPPA_SIGMA * mu / iw.sl[r]) : 0.0;
      iw.zu[r] = hu[r] ? fmin(fmax(zu, mu / (IP_KAPPA_SIGMA * iw.su[r])), IP_KAPPA_SIGMA * mu / iw.su[r]) : 0.0;
    }
  }
  out.err = err;
  out.f = f;
  for (int r = 0; r < m; ++r) lam_io[r] = lam[r];
  return out;
}

template <int DYN>
void run_problem_ip(const Problem& pr, Work& w, IpWork& iw, const IpSettings& S, const double* P0, const double* X0,
                    const double* XS0, double t0, int steps, double* xs_out, int* stats_out) {
  const PlOcpConst& O = pr.O;
  std::vector<double> p(P0, P0 + pr.np), x(X0, X0 + pr.n), xs(XS0, XS0 + O.nx), Pd(pr.n), lam(pr.m, 0.0);
  hess_diag(pr, p.data(), Pd.data());
  for (int k = 0; k < steps; ++k) {
    for (int j = 0; j < O.nx; ++j) p[O.P.x_init + j] = xs[j];
    pl::gait_schedule(O, pr.S.gait_type, pr.S.gait_period, pr.S.swing_period, t0 + k * p[O.P.dt_min], p.data(),
                      p.data() + O.P.contact, p.data() + O.P.swing);
    if (k > 0) {  // warm start (ocp_whole_body_rnea.py:207-235): forces reset to f_des on stance
      const int fo = pl::u_force_off(O);
      for (int i = 0; i < pr.N; ++i) {
        const int base = pr.x_off[i] + O.ndx + fo;
        for (int c = 0; c < O.nf; ++c) {
          double fd = pl::f_des_comp(pr.M, O, p.data(), c);
          if (c / 3 < 4 && p[O.P.contact + 4 * i + c / 3] == 0.0) fd = 0.0;
          x[base + c] = fd;
        }
      }
    }
    if (!S.mpc_lam) std::fill(lam.begin(), lam.end(), 0.0);
    IpStats s = ip_solve<DYN>(pr, w, iw, S, p.data(), Pd.data(), x.data(), lam.data(), S.mpc_lam && k > 0);
    const double* dx1 = x.data() + pr.x_off[1];
    double qn[PL_MAXQ];
    if (PL_IS_CV(O.dyn)) {
      pl::VecIn<double> acc{dx1 + 6, nullptr, 0.0, -1};
      pl::integrate_q<double>(pr.M, xs.data() + 6, acc, qn);
      for (int j = 0; j < 6; ++j) xs[j] += dx1[j];
      for (int j = 0; j < O.nq; ++j) xs[6 + j] = qn[j];
    } else {
      pl::VecIn<double> acc{dx1, nullptr, 0.0, -1};
      pl::integrate_q<double>(pr.M, xs.data(), acc, qn);
      for (int j = 0; j < O.nq; ++j) xs[j] = qn[j];
      for (int j = 0; j < O.nv; ++j) xs[O.nq + j] += dx1[O.nv + j];
    }
    if (stats_out) {
      stats_out[2 * k] = s.status;
      stats_out[2 * k + 1] = s.iter;
    }
  }
  for (int j = 0; j < O.nx; ++j) xs_out[j] = xs[j];
}

IpSettings ip_settings_from(const double* v) {
  IpSettings S;
  S.tol = v[0]; S.mu_init = v[1]; S.bound_push = v[2]; S.bound_frac = v[3]; S.warm_push = v[4];
  S.delta_w = v[5]; S.delta_c = v[6]; S.max_iter = (int)v[7]; S.ls_max = (int)v[8]; S.n_refine = (int)v[9];
  S.inertia_cap = (int)v[10];
  S.kkt_exact = (int)v[11];
  S.mpc_lam = (int)v[12];
  return S;
}

#define PL_CPU_DISPATCH(DYNV, CALL)                                         \
  switch (DYNV) {                                                           \
    case PL_DYN_RNEA: { constexpr int D_ = PL_DYN_RNEA; CALL; } break;     \
    case PL_DYN_ACC: { constexpr int D_ = PL_DYN_ACC; CALL; } break;       \
    case PL_DYN_ABA: { constexpr int D_ = PL_DYN_ABA; CALL; } break;       \
    case PL_DYN_CA: { constexpr int D_ = PL_DYN_CA; CALL; } break;         \
    case PL_DYN_ACCNB: { constexpr int D_ = PL_DYN_ACCNB; CALL; } break;   \
    case PL_DYN_CVNB: { constexpr int D_ = PL_DYN_CVNB; CALL; } break;     \
    default: { constexpr int D_ = PL_DYN_CV; CALL; } break;                \
  }

}  // namespace

// ---------------------------------------------------------------- C entry points (ctypes)
extern "C" void* cpu_create(const void* model, const void* oc, int N, int n, int m, int nnz, const int* x_off,
                            const int* row_off, const int* nrow, const int* nw, const int* pat_rows,
                            const int* pat_cols, const double* settings, int gait_type, double gait_period) {
  Problem* pr = new Problem();
  memcpy(&pr->M, model, sizeof(PlModel));
  memcpy(&pr->O, oc, sizeof(PlOcpConst));
  Settings& S = pr->S;
  S.rho = settings[0]; S.sigma = settings[1]; S.alpha = settings[2]; S.eps_abs = settings[3];
  S.eps_rel = settings[4]; S.eps_pinf = settings[5]; S.eps_dinf = settings[6];
  S.max_iter = (int)settings[7]; S.check_termination = (int)settings[8]; S.scaling = (int)settings[9];
  S.gait_type = gait_type;
  S.gait_period = gait_period;
  S.swing_period = gait_type == 0 ? 0.5 * gait_period : (gait_type == 1 ? 0.25 * gait_period : gait_period);
  pr->N = N; pr->n = n; pr->m = m; pr->nnz = nnz; pr->np = pr->O.P.np;
  pr->x_off.assign(x_off, x_off + N + 1);
  pr->row_off.assign(row_off, row_off + N + 1);
  pr->nrow.assign(nrow, nrow + N + 1);
  pr->nw.assign(nw, nw + N + 1);
  pr->colnode.assign(n, 0);
  for (int i = 0; i <= N; ++i)
    for (int c = 0; c < nw[i]; ++c) pr->colnode[x_off[i] + c] = i;
  std::vector<int> rownode(m, 0);
  for (int i = 0; i <= N; ++i)
    for (int r = 0; r < nrow[i]; ++r) rownode[row_off[i] + r] = i;
  // A in CSC (rows sorted inside each column)
  std::vector<int> order(nnz);
  for (int e = 0; e < nnz; ++e) order[e] = e;
  std::sort(order.begin(), order.end(), [&](int a, int b) {
    return pat_cols[a] != pat_cols[b] ? pat_cols[a] < pat_cols[b] : pat_rows[a] < pat_rows[b];
  });
  pr->Ap.assign(n + 1, 0);
  pr->Ai.assign(nnz, 0);
  for (int e = 0; e < nnz; ++e) pr->Ap[pat_cols[e] + 1]++;
  for (int j = 0; j < n; ++j) pr->Ap[j + 1] += pr->Ap[j];
  for (int k = 0; k < nnz; ++k) pr->Ai[k] = pat_rows[order[k]];
  // per (node, local column): (local row, CSC slot) of the node's rows
  const int ndx = pr->O.ndx;
  pr->jc_node_base.assign(N + 1, 0);
  int tot = 0;
  for (int i = 0; i < N; ++i) { pr->jc_node_base[i] = tot; tot += nw[i] + ndx; }
  pr->jc_node_base[N] = tot;
  std::vector<std::vector<std::pair<int, int>>> lists(tot);
  for (int j = 0; j < n; ++j)
    for (int k = pr->Ap[j]; k < pr->Ap[j + 1]; ++k) {
      const int r = pr->Ai[k];
      const int i = rownode[r];
      const int lc = (pr->colnode[j] == i) ? j - x_off[i] : nw[i] + (j - x_off[i + 1]);
      lists[pr->jc_node_base[i] + lc].push_back({r - row_off[i], k});
    }
  pr->jc_ptr.assign(tot + 1, 0);
  for (int c = 0; c < tot; ++c) {
    pr->jc_ptr[c + 1] = pr->jc_ptr[c] + (int)lists[c].size();
    for (auto& pr2 : lists[c]) pr->jc_list.push_back(pr2);
  }
  // KKT ordering: node by node, the node's variables then the node's rows
  Kkt& kk = pr->kkt;
  kk.K = n + m;
  pr->perm_x.assign(n, 0);
  pr->perm_z.assign(m, 0);
  int idx = 0;
  for (int i = 0; i <= N; ++i) {
    for (int c = 0; c < nw[i]; ++c) pr->perm_x[x_off[i] + c] = idx++;
    for (int r = 0; r < nrow[i]; ++r) pr->perm_z[row_off[i] + r] = idx++;
  }
  // upper-triangular CSC of the permuted KKT
  std::vector<std::vector<std::pair<int, int>>> cols(kk.K);  // (row, tag)
  for (int j = 0; j < n; ++j) cols[pr->perm_x[j]].push_back({pr->perm_x[j], -1 - j});
  for (int r = 0; r < m; ++r) cols[pr->perm_z[r]].push_back({pr->perm_z[r], -1 - n - r});
  for (int j = 0; j < n; ++j)
    for (int k = pr->Ap[j]; k < pr->Ap[j + 1]; ++k) {
      const int a = pr->perm_x[j], b = pr->perm_z[pr->Ai[k]];
      cols[std::max(a, b)].push_back({std::min(a, b), k});
    }
  kk.Kp.assign(kk.K + 1, 0);
  pr->kdiag_x.assign(n, 0);
  pr->kdiag_z.assign(m, 0);
  pr->kA.assign(nnz, 0);
  for (int c = 0; c < kk.K; ++c) {
    std::sort(cols[c].begin(), cols[c].end());
    for (auto& e : cols[c]) {
      const int slot = (int)kk.Ki.size();
      kk.Ki.push_back(e.first);
      if (e.second >= 0) pr->kA[e.second] = slot;
      else if (-1 - e.second < n) pr->kdiag_x[-1 - e.second] = slot;
      else pr->kdiag_z[-1 - e.second - n] = slot;
    }
    kk.Kp[c + 1] = (int)kk.Ki.size();
  }
  ldl_symbolic(kk);
  return pr;
}

extern "C" void cpu_destroy(void* h) { delete (Problem*)h; }

extern "C" long long cpu_factor_nnz(void* h) { return ((Problem*)h)->kkt.Lp.back(); }

// B problems x `steps` MPC steps on `threads` OpenMP threads (one problem per thread
// at a time).  Returns the wall seconds of the parallel region; xs_out [B][nx],
// stats [B][steps][4] = (OSQP status, ADMM iterations, line-search branch, trials).
extern "C" double cpu_mpc_batch(void* h, int B, const double* P, const double* X, const double* XS, const double* T0,
                                int steps, int threads, double* xs_out, int* stats) {
  const Problem& pr = *(Problem*)h;
  const int nx = pr.O.nx;
  if (threads > 0) omp_set_num_threads(threads);
  const auto t0 = std::chrono::steady_clock::now();
#pragma omp parallel
  {
    Work w;
    w.init(pr);
#pragma omp for schedule(dynamic, 1)
    for (int b = 0; b < B; ++b) {
      const double* Pb = P + (size_t)b * pr.np;
      const double* Xb = X + (size_t)b * pr.n;
      const double* XSb = XS + (size_t)b * nx;
      int* sb = stats ? stats + (size_t)b * steps * 4 : nullptr;
      switch (pr.O.dyn) {
        case PL_DYN_RNEA: run_problem<PL_DYN_RNEA>(pr, w, Pb, Xb, XSb, T0[b], steps, xs_out + (size_t)b * nx, sb); break;
        case PL_DYN_ACC: run_problem<PL_DYN_ACC>(pr, w, Pb, Xb, XSb, T0[b], steps, xs_out + (size_t)b * nx, sb); break;
        case PL_DYN_ABA: run_problem<PL_DYN_ABA>(pr, w, Pb, Xb, XSb, T0[b], steps, xs_out + (size_t)b * nx, sb); break;
        case PL_DYN_CA: run_problem<PL_DYN_CA>(pr, w, Pb, Xb, XSb, T0[b], steps, xs_out + (size_t)b * nx, sb); break;
        case PL_DYN_ACCNB: run_problem<PL_DYN_ACCNB>(pr, w, Pb, Xb, XSb, T0[b], steps, xs_out + (size_t)b * nx, sb); break;
        case PL_DYN_CVNB: run_problem<PL_DYN_CVNB>(pr, w, Pb, Xb, XSb, T0[b], steps, xs_out + (size_t)b * nx, sb); break;
        case PL_DYN_RNEAFD: run_problem<PL_DYN_RNEAFD>(pr, w, Pb, Xb, XSb, T0[b], steps, xs_out + (size_t)b * nx, sb); break;
        default: run_problem<PL_DYN_CV>(pr, w, Pb, Xb, XSb, T0[b], steps, xs_out + (size_t)b * nx, sb); break;
      }
    }
  }
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}

// One SQP iteration of one problem at (x, p) (parity test against the oracle): x is
// updated in place, dx gets the QP step, stats = (status, iter, branch, trials).
extern "C" int cpu_sqp_step(void* h, const double* p, double* x, double* dx, int* stats, double* alpha) {
  const Problem& pr = *(Problem*)h;
  Work w;
  w.init(pr);
  OsqpState st;
  st.x.assign(pr.n, 0.0);
  st.z.assign(pr.m, 0.0);
  st.y.assign(pr.m, 0.0);
  std::vector<double> Pd(pr.n);
  hess_diag(pr, p, Pd.data());
  StepStats s;
  switch (pr.O.dyn) {
    case PL_DYN_RNEA: s = sqp_step<PL_DYN_RNEA>(pr, w, st, p, Pd.data(), x); break;
    case PL_DYN_ACC: s = sqp_step<PL_DYN_ACC>(pr, w, st, p, Pd.data(), x); break;
    case PL_DYN_ABA: s = sqp_step<PL_DYN_ABA>(pr, w, st, p, Pd.data(), x); break;
    case PL_DYN_CA: s = sqp_step<PL_DYN_CA>(pr, w, st, p, Pd.data(), x); break;
    case PL_DYN_ACCNB: s = sqp_step<PL_DYN_ACCNB>(pr, w, st, p, Pd.data(), x); break;
    case PL_DYN_CVNB: s = sqp_step<PL_DYN_CVNB>(pr, w, st, p, Pd.data(), x); break;
    case PL_DYN_RNEAFD: s = sqp_step<PL_DYN_RNEAFD>(pr, w, st, p, Pd.data(), x); break;
    default: s = sqp_step<PL_DYN_CV>(pr, w, st, p, Pd.data(), x); break;
  }
  for (int j = 0; j < pr.n; ++j) dx[j] = w.step[j];
  stats[0] = s.status; stats[1] = s.iter; stats[2] = s.branch; stats[3] = s.trials;
  *alpha = s.alpha;
  return 0;
}

// Interior point: build the Hessian pair lists and the KKT pattern (once per OCP).
extern "C" long long cpu_ip_prepare(void* h) {
  Problem& pr = *(Problem*)h;
  if (pr.O.dyn == PL_DYN_RNEAFD) return -1;  // the Fatrop branch keeps a in u (ocp_whole_body_rnea.py:21)
  if (!pr.ip_ready) PL_CPU_DISPATCH(pr.O.dyn, ip_prepare<D_>(pr));
  return pr.ik_H_off.back();
}

// The Lagrangian Hessian blocks sum_r lam_r d^2 g_r / dw_i^2 at (p, x, lam), as the interior
// point forms them, into H [n][n] (dense, both triangles; tests / debugging).
extern "C" int cpu_ip_lag_hess(void* h, const double* p, const double* x, const double* lam, double* H) {
  Problem& pr = *(Problem*)h;
  if (cpu_ip_prepare(h) < 0) return -1;
  std::vector<double> hv(pr.ik_H_off.back());
  PL_CPU_DISPATCH(pr.O.dyn, lag_hess<D_>(pr, p, x, lam, hv.data()));
  const size_t n = pr.n;
  for (size_t k = 0; k < n * n; ++k) H[k] = 0.0;
  for (int i = 0; i < pr.N; ++i) {
    const auto& pl_ = pr.hpairs[pl::node_type(pr.O, i)];
    for (size_t q = 0; q < pl_.size(); ++q) {
      const size_t a = pr.x_off[i] + pl_[q].first, b = pr.x_off[i] + pl_[q].second;
      H[a * n + b] = H[b * n + a] = hv[pr.ik_H_off[i] + q];
    }
  }
  return 0;
}

// One interior-point solve of one problem from x (in / out); lam [m] in / out (the warm
// start when warm != 0); stats = (status, iterations, line-search trials); err_f = (err, f).
extern "C" int cpu_ip_solve(void* h, const double* p, double* x, double* lam, int warm, const double* settings,
                            int* stats, double* err_f) {
  Problem& pr = *(Problem*)h;
  if (cpu_ip_prepare(h) < 0) return -1;
  const IpSettings S = ip_settings_from(settings);
  Work w;
  w.init(pr);
  IpWork iw;
  iw.init(pr);
  std::vector<double> Pd(pr.n);
  hess_diag(pr, p, Pd.data());
  IpStats s{};
  PL_CPU_DISPATCH(pr.O.dyn, s = ip_solve<D_>(pr, w, iw, S, p, Pd.data(), x, lam, warm != 0));
  stats[0] = s.status; stats[1] = s.iter; stats[2] = s.trials;
  err_f[0] = s.err; err_f[1] = s.f;
  return 0;
}

// B problems x `steps` MPC steps with the interior-point solver (settings mpc_lam: lam_g carried
// across the steps as the Opti branch does, run_mpc.py:115-143, or cold multipliers per solve as
// the reference's default compiled-solver driver does, run_mpc.py:50-111) on `threads` OpenMP
// threads.  Returns
// the wall seconds; xs_out [B][nx], stats [B][steps][2] = (status, iterations).
extern "C" double cpu_ip_mpc_batch(void* h, int B, const double* P, const double* X, const double* XS,
                                   const double* T0, int steps, int threads, const double* settings, double* xs_out,
                                   int* stats) {
  Problem& pr = *(Problem*)h;
  if (cpu_ip_prepare(h) < 0) return -1.0;
  const IpSettings S = ip_settings_from(settings);
  const int nx = pr.O.nx;
  if (threads > 0) omp_set_num_threads(threads);
  const auto t0 = std::chrono::steady_clock::now();
#pragma omp parallel
  {
    Work w;
    w.init(pr);
    IpWork iw;
    iw.init(pr);
#pragma omp for schedule(dynamic, 1)
    for (int b = 0; b < B; ++b) {
      int* sb = stats ? stats + (size_t)b * steps * 2 : nullptr;
      PL_CPU_DISPATCH(pr.O.dyn, run_problem_ip<D_>(pr, w, iw, S, P + (size_t)b * pr.np, X + (size_t)b * pr.n,
                                                   XS + (size_t)b * nx, T0[b], steps, xs_out + (size_t)b * nx, sb));
    }
  }
  return std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
}
