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
  int K;
  std::vector<int> Kp, Ki;
  std::vector<int> kdiag_x, kdiag_z, kA;      // KKT slot of (x_j, x_j), (z_r, z_r), A entry e
  // symbolic LDL^T
  std::vector<int> etree, Lnz, Lp;
};

struct Work {  // per-thread scratch
  std::vector<double> g, lbg, ubg, grad, Ax, A, tan, P, q, l, u, xs_, zs_, ys_, D, E, rho, rinv, Kx, Lx, Dd, Dinv, rhs,
      sol, xt, zt, dx, dy, x_prev, z_prev, Axv, Aty, step, xtrial, buf;
  std::vector<int> Li, yMark, yIdx, elim, nextc;
  void init(const Problem& pr) {
    const int n = pr.n, m = pr.m, K = pr.K;
    for (auto* v : {&g, &lbg, &ubg, &l, &u, &zs_, &ys_, &E, &rho, &rinv, &zt, &dy, &z_prev, &Axv})
      v->assign(m, 0.0);
    for (auto* v : {&grad, &P, &q, &xs_, &D, &xt, &dx, &x_prev, &Aty, &step, &xtrial}) v->assign(n, 0.0);
    Ax.assign(pr.nnz, 0.0);
    A.assign(pr.nnz, 0.0);
    tan.assign(512, 0.0);
    Kx.assign(pr.Ki.size(), 0.0);
    Lx.assign(pr.Lp[K], 0.0);
    Li.assign(pr.Lp[K], 0);
    Dd.assign(K, 0.0);
    Dinv.assign(K, 0.0);
    rhs.assign(K, 0.0);
    sol.assign(K, 0.0);
    buf.assign(K, 0.0);
    yMark.assign(K, 0);
    yIdx.assign(K, 0);
    elim.assign(K, 0);
    nextc.assign(K, 0);
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
void ldl_symbolic(Problem& pr) {
  const int K = pr.K;
  std::vector<int> work(K);
  pr.etree.assign(K, -1);
  pr.Lnz.assign(K, 0);
  for (int j = 0; j < K; ++j) {
    work[j] = j;
    for (int q = pr.Kp[j]; q < pr.Kp[j + 1]; ++q) {
      int i = pr.Ki[q];
      if (i == j) continue;
      while (work[i] != j) {
        if (pr.etree[i] == -1) pr.etree[i] = j;
        pr.Lnz[i]++;
        work[i] = j;
        i = pr.etree[i];
      }
    }
  }
  pr.Lp.assign(K + 1, 0);
  for (int i = 0; i < K; ++i) pr.Lp[i + 1] = pr.Lp[i] + pr.Lnz[i];
}

// Up-looking numeric factorization of the upper-triangular CSC (Kp, Ki, Kx).
bool ldl_numeric(const Problem& pr, Work& w) {
  const int K = pr.K;
  double* y = w.buf.data();
  for (int i = 0; i < K; ++i) { w.yMark[i] = 0; y[i] = 0.0; w.nextc[i] = pr.Lp[i]; }
  for (int k = 0; k < K; ++k) {
    int nnzY = 0;
    w.Dd[k] = 0.0;
    for (int q = pr.Kp[k]; q < pr.Kp[k + 1]; ++q) {
      const int b = pr.Ki[q];
      if (b == k) { w.Dd[k] = w.Kx[q]; continue; }
      y[b] = w.Kx[q];
      int nx = b;
      if (!w.yMark[nx]) {
        w.yMark[nx] = 1;
        w.elim[0] = nx;
        int ne = 1;
        nx = pr.etree[b];
        while (nx != -1 && nx < k) {
          if (w.yMark[nx]) break;
          w.yMark[nx] = 1;
          w.elim[ne++] = nx;
          nx = pr.etree[nx];
        }
        while (ne) w.yIdx[nnzY++] = w.elim[--ne];
      }
    }
    for (int t = nnzY - 1; t >= 0; --t) {
      const int c = w.yIdx[t];
      const int tmp = w.nextc[c];
      const double yc = y[c];
      for (int j = pr.Lp[c]; j < tmp; ++j) y[w.Li[j]] -= w.Lx[j] * yc;
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

void ldl_solve(const Problem& pr, const Work& w, double* x) {
  const int K = pr.K;
  for (int i = 0; i < K; ++i)
    for (int j = pr.Lp[i]; j < pr.Lp[i + 1]; ++j) x[w.Li[j]] -= w.Lx[j] * x[i];
  for (int i = 0; i < K; ++i) x[i] *= w.Dinv[i];
  for (int i = K - 1; i >= 0; --i)
    for (int j = pr.Lp[i]; j < pr.Lp[i + 1]; ++j) x[i] -= w.Lx[j] * x[w.Li[j]];
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
  std::fill(w.Kx.begin(), w.Kx.end(), 0.0);
  for (int j = 0; j < n; ++j) w.Kx[pr.kdiag_x[j]] = P[j] + S.sigma;
  for (int r = 0; r < m; ++r) w.Kx[pr.kdiag_z[r]] = -rinv[r];
  for (int e = 0; e < nnz; ++e) w.Kx[pr.kA[e]] = A[e];
  OsqpInfo info{UNSOLVED, 0, 0.0, 0.0};
  if (!ldl_numeric(pr, w)) {
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
      ldl_solve(pr, w, rhs);
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
  pr->K = n + m;
  pr->perm_x.assign(n, 0);
  pr->perm_z.assign(m, 0);
  int idx = 0;
  for (int i = 0; i <= N; ++i) {
    for (int c = 0; c < nw[i]; ++c) pr->perm_x[x_off[i] + c] = idx++;
    for (int r = 0; r < nrow[i]; ++r) pr->perm_z[row_off[i] + r] = idx++;
  }
  // upper-triangular CSC of the permuted KKT
  std::vector<std::vector<std::pair<int, int>>> cols(pr->K);  // (row, tag)
  for (int j = 0; j < n; ++j) cols[pr->perm_x[j]].push_back({pr->perm_x[j], -1 - j});
  for (int r = 0; r < m; ++r) cols[pr->perm_z[r]].push_back({pr->perm_z[r], -1 - n - r});
  for (int j = 0; j < n; ++j)
    for (int k = pr->Ap[j]; k < pr->Ap[j + 1]; ++k) {
      const int a = pr->perm_x[j], b = pr->perm_z[pr->Ai[k]];
      cols[std::max(a, b)].push_back({std::min(a, b), k});
    }
  pr->Kp.assign(pr->K + 1, 0);
  pr->kdiag_x.assign(n, 0);
  pr->kdiag_z.assign(m, 0);
  pr->kA.assign(nnz, 0);
  for (int c = 0; c < pr->K; ++c) {
    std::sort(cols[c].begin(), cols[c].end());
    for (auto& e : cols[c]) {
      const int slot = (int)pr->Ki.size();
      pr->Ki.push_back(e.first);
      if (e.second >= 0) pr->kA[e.second] = slot;
      else if (-1 - e.second < n) pr->kdiag_x[-1 - e.second] = slot;
      else pr->kdiag_z[-1 - e.second - n] = slot;
    }
    pr->Kp[c + 1] = (int)pr->Ki.size();
  }
  ldl_symbolic(*pr);
  return pr;
}

extern "C" void cpu_destroy(void* h) { delete (Problem*)h; }

extern "C" long long cpu_factor_nnz(void* h) { return ((Problem*)h)->Lp.back(); }

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
