// Interior-point solve: the Fatrop branch of the reference (optimization/ocp.py:248-263
// settings, :360-373 solve; run_mpc.py:34-37 makes it the default), restated as an
// IPOPT-style primal-dual barrier method with a filter line search.  The algorithm
// and every constant follow oracle/ip_ref.py (which documents the choices); in short,
// per iteration:
//
//   eval g, J, grad f at x (k_eval_values / k_eval_jac / k_objective)
//   k_ip_kkt   residuals, scaled NLP error, convergence test, barrier update, and the
//              reduced Newton system (H + J^T W J) dx = -(grad + J^T lam) - J^T W r^
//              written into the OSQP-branch buffers (rho = W, As = J, Ps = H, ...)
//   k_fnode / k_fchain (sigma = delta_w) factor it; k_admm_init + ONE k_admm sweep
//              with alpha = 1 and unbounded rows solves it: xa = dx, za = J dx;
//              n_refine iterative-refinement solves (k_ip_refine) follow
//   k_ip_step  multiplier / slack / bound-multiplier directions, fraction-to-boundary,
//              filter line search (f and the rows at each trial on the first wave,
//              one node per lane), update.
//
// One 256-thread workgroup per problem for the two IP kernels; rows and columns are
// strided over the threads, reductions in LDS.  Problems that have terminated skip
// every kernel that checks info->done / ipinfo->active.
#include <math.h>

#include "eval_common.h"
#include "pinoloco.h"  // PL_PATH_* (pl_ocp_desc.debug_paths)

using pl::VecIn;

void launch_admm_init_zero(PlOcpHandle* h);  // k_qp.hip: k_admm_init with z = y = 0

#define PL_IP_INF 1e30  // bound on the unbounded rows of the Newton solve (OSQP's infinity)

namespace {

constexpr double KAPPA_EPS = 10.0, KAPPA_MU = 0.2, THETA_MU = 1.5;
constexpr double TAU_MIN = 0.99, S_MAX = 100.0, KAPPA_SIGMA = 1e10;
constexpr double GAMMA_THETA = 1e-5, GAMMA_PHI = 1e-8, DELTA = 1.0, S_THETA = 1.1, S_PHI = 2.3, ETA_PHI = 1e-8;
constexpr double W_MIN = 1e-20;
enum { ST_CONVERGED = 1, ST_MAX_ITER = -1, ST_LS_FAIL = -2, ST_NONFINITE = -3 };

struct RowKind {
  bool eq, hl, hu;
};
__device__ __forceinline__ RowKind row_kind(double l, double u) {
  RowKind k;
  k.eq = l == u;
  k.hl = !k.eq && isfinite(l);
  k.hu = !k.eq && isfinite(u);
  return k;
}

// acc + sum over column j's entries of A_e y_row(e) in entry order (the global CSC of
// d.gc_ptr / d.gc_er), the entry words and the operands of 8 entries loaded together (one
// dependent round trip per 8 entries instead of per entry); same operations in the same order
__device__ __forceinline__ double gc_dot(const PlDev& d, int j, const double* A, const double* y, double acc) {
  const int q0 = d.gc_ptr[j], q1 = d.gc_ptr[j + 1];
  for (int qb = q0; qb < q1; qb += 8) {
    int2 er[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) er[u] = d.gc_er[min(qb + u, q1 - 1)];
    double a[8], t[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      a[u] = A[er[u].x];
      t[u] = y[er[u].y];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (qb + u < q1) acc += a[u] * t[u];
  }
  return acc;
}

// red: 256 x K doubles
template <int K>
__device__ void block_reduce(double (&v)[K], const bool (&is_max)[K], double* red) {
#pragma unroll
  for (int k = 0; k < K; ++k) red[k * 256 + threadIdx.x] = v[k];
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        const double a = red[k * 256 + threadIdx.x], b = red[k * 256 + threadIdx.x + s];
        red[k * 256 + threadIdx.x] = is_max[k] ? fmax(a, b) : a + b;
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = red[k * 256];
  __syncthreads();
}

// Row values at a trial point: theta (l1 norm of c) and the barrier sum.
struct TrialEmit {
  const double* s;
  const double* ds;
  double a;
  int r;
  double th, bar;
  __device__ void operator()(double v, double l, double u) {
    const RowKind k = row_kind(l, u);
    if (k.eq) {
      th += fabs(v - l);
    } else {
      const double st = s[r] + a * ds[r];
      th += fabs(v - st);
      if (k.hl) bar += log(st - l);
      if (k.hu) bar += log(u - st);
    }
    ++r;
  }
};

__device__ __forceinline__ double next_mu(double mu, double tol) {
  return fmax(tol / 10.0, fmin(KAPPA_MU * mu, pow(mu, THETA_MU)));
}

}  // namespace

// ---------------------------------------------------------------------------------
// Initial point (warm_start_init_point): slacks pushed into the interior, lam = 0,
// centred bound multipliers; theta_max / theta_min from theta(x0, s0).  Needs g, lbg,
// ubg at d.x (k_eval_values).
// warm: lam = lam0 (the previous solve's lam_g) and the slack-bound multipliers split by the
// sign of lam (z_u - z_l = lam), pushed up to warm_push (oracle/ip_ref.py); cold: lam = 0,
// z = mu / slack
__global__ __launch_bounds__(256) void k_ip_init(PlDev d, int m, PlIpSettings st, int warm) {
  const int b = blockIdx.x;
  __shared__ double red[256];
  if (threadIdx.x == 0 && d.ip_dwi) d.ip_dwi[2 * b + 1] = 0.0;  // no inertia shift used yet in this solve
  const double* g = d.g + (size_t)b * m;
  const double* lbg = d.lbg + (size_t)b * m;
  const double* ubg = d.ubg + (size_t)b * m;
  double* s = d.ip_s + (size_t)b * m;
  double* lam = d.ip_lam + (size_t)b * m;
  double* zl = d.ip_zl + (size_t)b * m;
  double* zu = d.ip_zu + (size_t)b * m;
  const double mu = st.mu_init;
  double th = 0.0;
  for (int r = threadIdx.x; r < m; r += 256) {
    const double l = lbg[r], u = ubg[r];
    const RowKind k = row_kind(l, u);
    double sr = 0.0, zlr = 0.0, zur = 0.0;
    if (k.eq) {
      th += fabs(g[r] - l);
    } else {
      double pl = st.bound_push * fmax(1.0, k.hl ? fabs(l) : 0.0);
      double pu = st.bound_push * fmax(1.0, k.hu ? fabs(u) : 0.0);
      if (k.hl && k.hu) {
        pl = fmin(pl, st.bound_frac * (u - l));
        pu = fmin(pu, st.bound_frac * (u - l));
      }
      sr = g[r];
      if (k.hl) sr = fmax(sr, l + pl);
      if (k.hu) sr = fmin(sr, u - pu);
      if (warm) {
        const double lw = d.ip_lam0[(size_t)b * m + r];
        if (k.hl) zlr = fmax(fmax(-lw, 0.0), st.warm_push);
        if (k.hu) zur = fmax(fmax(lw, 0.0), st.warm_push);
      } else {
        if (k.hl) zlr = mu / (sr - l);
        if (k.hu) zur = mu / (u - sr);
      }
      th += fabs(g[r] - sr);
    }
    s[r] = sr;
    lam[r] = warm ? d.ip_lam0[(size_t)b * m + r] : 0.0;
    zl[r] = zlr;
    zu[r] = zur;
  }
  red[threadIdx.x] = th;
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    if (threadIdx.x < k) red[threadIdx.x] += red[threadIdx.x + k];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    PlIpInfo* ip = d.ipinfo + b;
    const double th0 = red[0];
    ip->mu = mu;
    ip->theta_max = 1e4 * fmax(1.0, th0);
    ip->theta_min = 1e-4 * fmax(1.0, th0);
    ip->err = INFINITY;
    ip->f = 0.0;
    ip->alpha = 0.0;
    ip->alpha_z = 0.0;
    ip->viol_max = 0.0;
    ip->iter = 0;
    ip->status = ST_MAX_ITER;
    ip->nfilt = 0;
    ip->trials = 0;
    ip->ref_solves = 0;
    ip->active = 1;
    for (int q = 0; q < PL_IP_MAXFILT; ++q) ip->alphas[q] = 0.0;
    d.info[b].done = 0;
  }
}

// ---------------------------------------------------------------------------------
// Iteration k: error / termination / barrier update, then the reduced Newton system in
// the buffers the factor and the ADMM sweep read.
__global__ __launch_bounds__(256) void k_ip_kkt(PlDev d, int N, int n, int m, int nnz, int ncpl_max, int k,
                                                PlIpSettings st) {
  const int b = blockIdx.x;
  PlIpInfo* ip = d.ipinfo + b;
  if (!ip->active) return;
  __shared__ double red[256 * 12];
  __shared__ double s_mu;
  __shared__ int s_go;
  const double* g = d.g + (size_t)b * m;
  const double* lbg = d.lbg + (size_t)b * m;
  const double* ubg = d.ubg + (size_t)b * m;
  const double* s = d.ip_s + (size_t)b * m;
  const double* lam = d.ip_lam + (size_t)b * m;
  const double* zl = d.ip_zl + (size_t)b * m;
  const double* zu = d.ip_zu + (size_t)b * m;
  const double* A = d.Araw + (size_t)b * nnz;
  const double* grad = d.grad + (size_t)b * n;
  const double mu = ip->mu;
  // candidate barrier parameters of the monotone update (at most 4 decreases)
  double mus[5];
  mus[0] = mu;
#pragma unroll
  for (int q = 1; q < 5; ++q) mus[q] = next_mu(mus[q - 1], st.tol);
  // v: 0 max|rx|, 1 max|rs|, 2 max|c|, 3 sum|lam|, 4 sum zl + zu, 5 #bounds,
  //    6..10 max complementarity error at mus[0..4], 11 max violation
  double v[12] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  const bool is_max[12] = {true, true, true, false, false, false, true, true, true, true, true, true};
  bool bad = false;
  for (int j = threadIdx.x; j < n; j += 256) {
    const double acc = gc_dot(d, j, A, lam, grad[j]);
    v[0] = fmax(v[0], fabs(acc));
    bad |= !isfinite(acc);
  }
  double comp0 = 0.0;
  for (int r = threadIdx.x; r < m; r += 256) {
    const double l = lbg[r], u = ubg[r];
    const RowKind rk = row_kind(l, u);
    const double c = rk.eq ? g[r] - l : g[r] - s[r];
    v[2] = fmax(v[2], fabs(c));
    v[3] += fabs(lam[r]);
    v[11] = fmax(v[11], fmax(fmax(0.0, l - g[r]), fmax(0.0, g[r] - u)));
    bad |= !isfinite(c);
    if (!rk.eq) {
      v[1] = fmax(v[1], fabs(-lam[r] - zl[r] + zu[r]));
      v[4] += zl[r] + zu[r];
      if (rk.hl) {
        const double cl = (s[r] - l) * zl[r];
        v[5] += 1.0;
        comp0 = fmax(comp0, fabs(cl));
#pragma unroll
        for (int q = 0; q < 5; ++q) v[6 + q] = fmax(v[6 + q], fabs(cl - mus[q]));
      }
      if (rk.hu) {
        const double cu = (u - s[r]) * zu[r];
        v[5] += 1.0;
        comp0 = fmax(comp0, fabs(cu));
#pragma unroll
        for (int q = 0; q < 5; ++q) v[6 + q] = fmax(v[6 + q], fabs(cu - mus[q]));
      }
    }
  }
  block_reduce<12>(v, is_max, red);
  red[threadIdx.x] = comp0;
  red[256 + threadIdx.x] = bad ? 1.0 : 0.0;
  __syncthreads();
  for (int q = 128; q > 0; q >>= 1) {
    if (threadIdx.x < q) {
      red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + q]);
      red[256 + threadIdx.x] = fmax(red[256 + threadIdx.x], red[256 + threadIdx.x + q]);
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    comp0 = red[0];
    const bool nonfinite = red[256] != 0.0;
    const double nb = v[5];
    const double sd = fmax(S_MAX, (v[3] + v[4]) / fmax((double)m + nb, 1.0)) / S_MAX;
    const double sc = fmax(S_MAX, v[4] / fmax(nb, 1.0)) / S_MAX;
    const double base = fmax(fmax(v[0] / sd, v[1] / sd), v[2]);
    const double err = fmax(base, comp0 / sc);
    ip->err = err;
    ip->viol_max = v[11];
    ip->f = d.work[(size_t)b * 8];
    ip->iter = k < 0 ? 0 : k;
    int go = 1;
    if (k < 0) {
      // teacher-forced direction (pl_debug_ip_direction): no termination, mu as given
    } else if (nonfinite || !isfinite(err)) {
      ip->status = ST_NONFINITE;
      go = 0;
    } else if (err <= st.tol) {
      ip->status = ST_CONVERGED;
      go = 0;
    } else if (k == st.max_iter) {
      ip->status = ST_MAX_ITER;
      go = 0;
    }
    double mu_new = mu;
    if (go && k >= 0) {
      for (int q = 0; q < 4; ++q) {
        if (fmax(base, v[6 + q] / sc) > KAPPA_EPS * mus[q]) break;
        if (mus[q + 1] == mus[q]) break;
        mu_new = mus[q + 1];
        ip->nfilt = 0;
      }
      ip->mu = mu_new;
    } else if (!go) {
      ip->active = 0;
      d.info[b].done = 1;
    }
    s_mu = mu_new;
    s_go = go;
  }
  __syncthreads();
  if (!s_go) return;
  const double mun = s_mu;
  // ---- reduced Newton system in the OSQP-branch buffers:
  //   rho = W, As = J, Ps = H (the factor adds sigma = delta_w), qs = rx, xa = 0,
  //   za = -r^, ya = 0 -> k_admm_init's rhs = -rx - J^T W r^; rows unbounded
  double* rho = d.rho + (size_t)b * m;
  double* za = d.za + (size_t)b * m;
  double* ya = d.ya + (size_t)b * m;
  double* ls = d.ls + (size_t)b * m;
  double* us = d.us + (size_t)b * m;
  double* rh = d.ip_rh + (size_t)b * m;
  for (int r = threadIdx.x; r < m; r += 256) {
    const double l = lbg[r], u = ubg[r];
    const RowKind rk = row_kind(l, u);
    double W, rhat;
    if (rk.eq) {
      W = 1.0 / st.delta_c;
      rhat = g[r] - l;
    } else {
      const double sl = rk.hl ? s[r] - l : 1.0, su = rk.hu ? u - s[r] : 1.0;
      const double sig = (rk.hl ? zl[r] / sl : 0.0) + (rk.hu ? zu[r] / su : 0.0);
      W = sig / (1.0 + st.delta_c * sig);
      const double bs = lam[r] + (rk.hl ? mun / sl : 0.0) - (rk.hu ? mun / su : 0.0);
      rhat = (g[r] - s[r]) - bs / sig;
    }
    W = fmax(W, W_MIN);
    rho[r] = W;
    rh[r] = rhat;
    za[r] = -rhat;
    ya[r] = 0.0;
    ls[r] = -PL_IP_INF;
    us[r] = PL_IP_INF;
  }
  double* As = d.As + (size_t)b * nnz;
  for (int e = threadIdx.x; e < nnz; e += 256) As[e] = A[e];
  double* qs = d.qs + (size_t)b * n;
  double* Ps = d.Ps + (size_t)b * n;
  double* xa = d.xa + (size_t)b * n;
  const double* P = d.P + (size_t)b * n;
  for (int j = threadIdx.x; j < n; j += 256) {
    qs[j] = gc_dot(d, j, A, lam, grad[j]);
    Ps[j] = P[j];
    xa[j] = 0.0;
    d.ip_dx[(size_t)b * n + j] = 0.0;
  }
  for (int r = threadIdx.x; r < m; r += 256) d.ip_jdx[(size_t)b * m + r] = 0.0;
  if (threadIdx.x == 0 && d.ip_dwi) {  // inertia correction of this Newton system starts at 0
    d.ip_dwi[2 * b] = 0.0;
    for (int q = 0; q < 4; ++q) d.ip_iflag[4 * b + q] = 0;
  }
  __syncthreads();
  // rho of the coupling rows, contiguous for the ADMM prefetch (as k_qp_finish)
  for (int i = 0; i <= N; ++i) {
    const PlNode nd = d.nodes[i];
    double* rhoc = d.rhoc + (size_t)b * (N + 1) * ncpl_max + (size_t)i * ncpl_max;
    for (int q = threadIdx.x; q < nd.ncpl; q += 256) rhoc[q] = rho[nd.row_off + d.cplrow[nd.cpl_off + q]];
  }
}

// ---------------------------------------------------------------------------------
// Iterative refinement of the Newton step: dx += xa, J dx += za (the last sweep's
// solution), then the x-row residual of the KKT system at the accumulated step,
//   r = -(grad + J^T (lam + dlam)) - (H + delta_w) dx,   dlam = W (J dx + r^),
// becomes the next sweep's right-hand side (qs = -r, za = ya = xa = 0).  With
// W_E = 1 / delta_c = 1e4 one block-inverse solve agrees with the oracle's sparse LU to
// ~1e-12 and the refinement keeps the step at that level as the multipliers grow
// (at W_E = 1e6 the explicit inverses lose ~5 digits and the refinement diverges).
// H_i dx of a node block (r04): one wave per node (nodes w, w + 4, ...), the block's written
// entries (d.hnz, r05: a B2G node writes ~1/5 of its packed-lower block; until r05 every entry
// was read and its row recovered by a square root) in storage order and both halves of every
// entry added into a wave-private LDS vector by ds_add_f64 (fixed lane / instruction order:
// deterministic);
// the per-column gather of the block (strided, uncoalesced) took 2.1 ms per call at the
// headline size, and serves the blocks wider than the LDS vectors (PL_IP_NWMAX).
#define PL_IP_NWMAX 192
__device__ __forceinline__ void ip_lds_add(double* p, double v) {
  typedef __attribute__((address_space(3))) double* LPtr;
  __hip_atomic_fetch_add((LPtr)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}
__device__ __forceinline__ void ip_wsync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

__global__ __launch_bounds__(256) void k_ip_refine(PlDev d, int N, int n, int m, int nnz, double delta_w, int hlag,
                                                   long long hl_stride, int4 hnz_off, int tau_nodes, int iref,
                                                   int gather) {
  const int b = blockIdx.x;
  if (!d.ipinfo[b].active || d.info[b].done) return;  // done: this solve's refinement has converged
  const double* A = d.Araw + (size_t)b * nnz;
  const double* W = d.rho + (size_t)b * m;
  const double* rh = d.ip_rh + (size_t)b * m;
  const double* lam = d.ip_lam + (size_t)b * m;
  const double* grad = d.grad + (size_t)b * n;
  const double* Ps = d.Ps + (size_t)b * n;  // P + the inertia shift (k_ip_kkt, k_ip_inertia)
  double* xa = d.xa + (size_t)b * n;
  double* za = d.za + (size_t)b * m;
  double* ya = d.ya + (size_t)b * m;
  double* qs = d.qs + (size_t)b * n;
  double* dx = d.ip_dx + (size_t)b * n;
  double* jdx = d.ip_jdx + (size_t)b * m;
  double* t = d.ip_dl + (size_t)b * m;  // lam + dlam (scratch; k_ip_step recomputes dlam)
  {  // iref = 0: xa is the first solve's direction; iref >= 1: xa is a refinement correction.
     // A correction larger than the one before it (the refinement diverges: the block inverses'
     // noise floor) is not applied and ends the refinement.  Otherwise it is applied, and the
     // refinement has converged once the correction is below 1e-12 |dx| (IPOPT's refinement
     // stops at a residual ratio of 1e-10) or has stopped contracting (more than 0.9 of the one
     // before: stagnation; a linearly converging refinement with a rate in (0.5, 0.9) keeps
     // going up to n_refine solves).  A stopped problem skips the remaining refinement solves of
     // this Newton system (info->done, which the sweep kernels test; k_ip_step clears it), and
     // its correction buffer is zeroed.  ref_solves counts the solves applied (k_ip_init resets).
    __shared__ double s_c[256], s_d[256];
    __shared__ int s_stop, s_apply;
    double cmax = 0.0, dmax = 0.0;
    for (int j = threadIdx.x; j < n; j += 256) {
      const double c = xa[j];
      cmax = fmax(cmax, fabs(c));
      dmax = fmax(dmax, fabs(dx[j] + c));
    }
    s_c[threadIdx.x] = cmax;
    s_d[threadIdx.x] = dmax;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if (threadIdx.x < w) {
        s_c[threadIdx.x] = fmax(s_c[threadIdx.x], s_c[threadIdx.x + w]);
        s_d[threadIdx.x] = fmax(s_d[threadIdx.x], s_d[threadIdx.x + w]);
      }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      PlIpInfo* ip = d.ipinfo + b;
      const double c = s_c[0];
      const bool grew = iref >= 2 && !(c <= ip->ref_last);
      s_apply = !grew;
      s_stop = grew || (iref >= 1 && (c <= 1e-12 * s_d[0] || (iref >= 2 && c > 0.9 * ip->ref_last)));
      if (!grew) {
        ip->ref_last = c;
        ip->ref_solves += 1;
      }
      if (s_stop) d.info[b].done = 1;
    }
    __syncthreads();
    const bool apply = s_apply, stop = s_stop;
    for (int r = threadIdx.x; r < m; r += 256) {  // J dx follows dx (za = J xa of the last sweep)
      const double jr = apply ? jdx[r] + za[r] : jdx[r];
      jdx[r] = jr;
      t[r] = lam[r] + W[r] * (jr + rh[r]);
      za[r] = 0.0;
      ya[r] = 0.0;
    }
    if (apply)
      for (int j = threadIdx.x; j < n; j += 256) dx[j] += xa[j];
    __syncthreads();
    if (stop) {
      for (int j = threadIdx.x; j < n; j += 256) xa[j] = 0.0;
      return;
    }
  }
  const double* Hb = hlag ? d.Hlag + (size_t)b * hl_stride : nullptr;
  if (Hb) {  // qs = H_i dx_{w_i} per node block (k_lag_hess's packed lower blocks; none on node N)
    __shared__ double hy[4][PL_IP_NWMAX], hx[4][PL_IP_NWMAX];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    double* y = hy[wv];
    double* xv = hx[wv];
    for (int i = wv; i <= N; i += 4) {
      const PlNode nd = d.nodes[i];
      const int nw = nd.nw;
      if (nw > PL_IP_NWMAX || gather) {  // wider blocks than the LDS vectors: the per-column global gather
                                         // (gather: PL_PATH_IP_REFINE_GATHER, its regression test)
        const double* Hi = i < N ? Hb + d.hoff[i] : nullptr;
        for (int c = lane; c < nw; c += 64) {
          double acc = 0.0;
          if (Hi)
            for (int r = 0; r < nw; ++r)
              acc = fma(Hi[r >= c ? r * (r + 1) / 2 + c : c * (c + 1) / 2 + r], dx[nd.x_off + r], acc);
          qs[nd.x_off + c] = acc;
        }
        continue;
      }
      for (int c = lane; c < nw; c += 64) {
        y[c] = 0.0;
        xv[c] = dx[nd.x_off + c];
      }
      ip_wsync();
      if (i < N) {  // the block's written entries only (d.hnz, the node type's list)
        const double* Hi = Hb + d.hoff[i];
        const int t = i == 0 ? 0 : (i < tau_nodes ? 1 : 2);  // rows.h node_type
        const int q0 = t == 0 ? hnz_off.x : (t == 1 ? hnz_off.y : hnz_off.z);
        const int q1 = t == 0 ? hnz_off.y : (t == 1 ? hnz_off.z : hnz_off.w);
        for (int q = q0 + lane; q < q1; q += 64) {
          const int rc = d.hnz[q];
          const int r = rc & 0xffff, c = rc >> 16;
          const double h = Hi[r * (r + 1) / 2 + c];
          ip_lds_add(y + r, h * xv[c]);
          if (c != r) ip_lds_add(y + c, h * xv[r]);
        }
        ip_wsync();
      }
      for (int c = lane; c < nw; c += 64) qs[nd.x_off + c] = y[c];
      ip_wsync();
    }
    __syncthreads();
  }
  for (int j = threadIdx.x; j < n; j += 256) {
    const double dj = dx[j];
    double acc = grad[j] + (Ps[j] + delta_w) * dj;
    if (Hb) acc += qs[j];
    qs[j] = gc_dot(d, j, A, t, acc);  // rhs = -qs = r
  }
  __syncthreads();
  for (int j = threadIdx.x; j < n; j += 256) xa[j] = 0.0;
}

// Inertia correction of the Newton system (IPOPT Algorithm IC, Waechter & Biegler 2006,
// sec. 3.1; Fatrop corrects the same way when its Riccati recursion meets a block that is
// not positive definite).  The reduced matrix H_L + Ps + delta_w I + J^T W J is positive
// definite iff every pivot of the factor's block elimination is (k_fnode / k_fchain report
// a pivot <= 0 in ip_iflag[0]).  Per round: a clean factor resolves the system (and
// records a nonzero shift as the last one); otherwise the shift grows -- first
// 1e-4, or a third of the last one, then x100 while no shift has succeeded in this solve,
// x8 after -- and the problem is refactored (ip_iflag[1]).  After `cap` shifts the system
// is taken as it is.  oracle/ip_ref.py restates the same rule.
__global__ __launch_bounds__(256) void k_ip_inertia(PlDev d, int n, int cap) {
  const int b = blockIdx.x;
  if (!d.ipinfo[b].active) return;
  int* F = d.ip_iflag + 4 * b;
  double* dw = d.ip_dwi + 2 * b;
  __shared__ double s_new;
  __shared__ int s_act;
  if (threadIdx.x == 0) {
    s_act = 0;
    if (F[2]) {
      F[1] = 0;
    } else if (!F[0]) {
      F[2] = 1;
      F[1] = 0;
      if (dw[0] > 0.0) dw[1] = dw[0];
    } else if (F[3] >= cap) {
      F[0] = 0;
      F[1] = 0;
      F[2] = 1;
    } else {
      F[0] = 0;
      const double nd = dw[0] == 0.0 ? (dw[1] == 0.0 ? 1e-4 : fmax(1e-20, dw[1] / 3.0))
                                     : dw[0] * (dw[1] == 0.0 ? 100.0 : 8.0);
      dw[0] = nd;
      F[1] = 1;
      F[3] += 1;
      s_new = nd;
      s_act = 1;
    }
  }
  __syncthreads();
  if (!s_act) return;
  const double* P = d.P + (size_t)b * n;
  double* Ps = d.Ps + (size_t)b * n;
  const double sh = s_new;
  for (int j = threadIdx.x; j < n; j += 256) Ps[j] = P[j] + sh;
}

// ---------------------------------------------------------------------------------
// Directions, fraction-to-boundary, filter line search and update.  dx = d.xa and
// J dx = d.za (the ADMM sweep with alpha = 1 on unbounded rows).
template <int DYN>
__global__ __launch_bounds__(256) void k_ip_step(PlDev d, int N, int n, int m, int np, PlIpSettings st,
                                                 int dir_only) {
  const int b = blockIdx.x;
  PlIpInfo* ip = d.ipinfo + b;
  if (!ip->active) return;
  __shared__ double red[256 * 6];
  __shared__ double s_a, s_az;
  __shared__ int s_acc, s_ftype;
  const PlOcpConst& O = *d.oc;
  const PlModel& M = *d.model;
  const double* g = d.g + (size_t)b * m;
  const double* lbg = d.lbg + (size_t)b * m;
  const double* ubg = d.ubg + (size_t)b * m;
  double* s = d.ip_s + (size_t)b * m;
  double* lam = d.ip_lam + (size_t)b * m;
  double* zl = d.ip_zl + (size_t)b * m;
  double* zu = d.ip_zu + (size_t)b * m;
  const double* rh = d.ip_rh + (size_t)b * m;
  double* jdx = d.ip_jdx + (size_t)b * m;
  const double* rho = d.rho + (size_t)b * m;
  double* dl = d.ip_dl + (size_t)b * m;
  double* ds = d.ip_ds + (size_t)b * m;
  double* x = d.x + (size_t)b * n;
  double* dx = d.ip_dx + (size_t)b * n;
  const double* grad = d.grad + (size_t)b * n;
  const double mu = ip->mu;
  const double tau = fmax(TAU_MIN, 1.0 - mu);
  {  // the last sweep's correction completes the step -- unless the refinement ran all n_refine
     // solves and this correction grew (k_ip_refine's rule); a problem whose refinement stopped
     // has xa = za = 0 here.  info->done (k_ip_refine's stop flag) is cleared for the next system
    const double* xa = d.xa + (size_t)b * n;
    const double* za = d.za + (size_t)b * m;
    __shared__ int s_app;
    double cmax = 0.0;
    for (int j = threadIdx.x; j < n; j += 256) cmax = fmax(cmax, fabs(xa[j]));
    red[threadIdx.x] = cmax;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
      if (threadIdx.x < w) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + w]);
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      const bool pending = !d.info[b].done;
      const bool app = !(pending && st.n_refine >= 2 && !(red[0] <= ip->ref_last));
      if (pending && app) ip->ref_solves += 1;
      s_app = app;
      d.info[b].done = 0;  // set again below on termination
    }
    __syncthreads();
    if (s_app) {
      for (int j = threadIdx.x; j < n; j += 256) dx[j] += xa[j];
      for (int r = threadIdx.x; r < m; r += 256) jdx[r] += za[r];
    }
    __syncthreads();
  }
  // v: 0 alpha_max, 1 alpha_z, 2 theta, 3 barrier sum, 4 dphi, 5 non-finite
  // (the two step bounds are reduced as max of -alpha)
  double v[6] = {-1.0, -1.0, 0.0, 0.0, 0.0, 0.0};
  for (int r = threadIdx.x; r < m; r += 256) {
    const double l = lbg[r], u = ubg[r];
    const RowKind rk = row_kind(l, u);
    const double W = rho[r];
    const double dlr = W * (jdx[r] + rh[r]);
    double dsr = 0.0;
    if (rk.eq) {
      v[2] += fabs(g[r] - l);
    } else {
      const double sl = rk.hl ? s[r] - l : 1.0, su = rk.hu ? u - s[r] : 1.0;
      const double sig = (rk.hl ? zl[r] / sl : 0.0) + (rk.hu ? zu[r] / su : 0.0);
      const double bs = lam[r] + (rk.hl ? mu / sl : 0.0) - (rk.hu ? mu / su : 0.0);
      dsr = (bs + dlr) / sig;
      v[2] += fabs(g[r] - s[r]);
      if (rk.hl) {
        const double dz = mu / sl - zl[r] - zl[r] / sl * dsr;
        if (dsr < 0) v[0] = fmax(v[0], tau * sl / dsr);  // -(-tau sl / ds)
        if (dz < 0) v[1] = fmax(v[1], tau * zl[r] / dz);
        v[3] += log(sl);
        v[4] += -mu / sl * dsr;
      }
      if (rk.hu) {
        const double dz = mu / su - zu[r] + zu[r] / su * dsr;
        if (-dsr < 0) v[0] = fmax(v[0], tau * su / -dsr);
        if (dz < 0) v[1] = fmax(v[1], tau * zu[r] / dz);
        v[3] += log(su);
        v[4] += mu / su * dsr;
      }
    }
    if (!isfinite(dlr) || !isfinite(dsr)) v[5] = 1.0;
    dl[r] = dlr;
    ds[r] = dsr;
  }
  for (int j = threadIdx.x; j < n; j += 256) {
    v[4] += grad[j] * dx[j];
    if (!isfinite(dx[j])) v[5] = 1.0;
  }
  {
    const bool mx[6] = {true, true, false, false, false, true};
    block_reduce<6>(v, mx, red);
  }
  const double amax = fmin(1.0, -v[0]), az = fmin(1.0, -v[1]);
  const double theta = v[2], f0 = d.work[(size_t)b * 8];
  const double phi = f0 - mu * v[3];
  const double dphi = v[4];
  if (dir_only) {  // pl_debug_ip_direction: the direction and the step bounds only
    if (threadIdx.x == 0) {
      ip->alpha = amax;
      ip->alpha_z = az;
    }
    return;
  }
  if (v[5] != 0.0) {
    if (threadIdx.x == 0) {
      ip->status = ST_NONFINITE;
      ip->active = 0;
      d.info[b].done = 1;
    }
    return;
  }
  // ---- trials
  if (threadIdx.x == 0) {
    s_acc = 0;
    s_ftype = 0;
    s_a = 0.0;
  }
  __syncthreads();
  int t = 0;
  __shared__ double kst[PL_KIN_STORE * 64];
  __shared__ double ored[256];
  for (t = 0; t < st.ls_max; ++t) {
    const double a = amax * ldexp(1.0, -t);
    const double ft = objective_wg<false>(d, b, N, n, np, x, dx, a, nullptr, ored);
    TrialEmit e{s, ds, a, 0, 0.0, 0.0};
    if (threadIdx.x < 64) {
      for (int i = threadIdx.x; i < N; i += 64) {
        const PlNode nd = d.nodes[i];
        const PlNode nn = d.nodes[i + 1];
        e.r = nd.row_off;
        VecIn<double> vdx{x + nd.x_off, dx + nd.x_off, a, -1};
        VecIn<double> vu{x + nd.x_off + O.ndx, dx + nd.x_off + O.ndx, a, -1};
        VecIn<double> vdxn{x + nn.x_off, dx + nn.x_off, a, -1};
        pl::node_rows<double, DYN>(M, O, i, d.p + (size_t)b * np, vdx, vu, vdxn, e, kst + threadIdx.x, 64);
      }
    }
    double w[2] = {e.th, e.bar};
    const bool mx2[2] = {false, false};
    block_reduce<2>(w, mx2, red);
    const double th_t = w[0], bar_t = w[1];
    if (threadIdx.x == 0) {
      const double ph_t = ft - mu * bar_t;
      bool ok = isfinite(th_t) && isfinite(ph_t) && th_t <= ip->theta_max;
      if (ok) {
        for (int q = 0; q < ip->nfilt; ++q)
          if (th_t >= ip->filt[2 * q] && ph_t >= ip->filt[2 * q + 1]) { ok = false; break; }
      }
      if (ok) {
        const bool switching = dphi < 0.0 && a * pow(-dphi, S_PHI) > DELTA * pow(theta, S_THETA);
        if (theta <= ip->theta_min && switching) {
          if (ph_t <= phi + ETA_PHI * a * dphi) {
            s_acc = 1;
            s_ftype = 1;
          }
        } else if (th_t <= (1.0 - GAMMA_THETA) * theta || ph_t <= phi - GAMMA_PHI * theta) {
          s_acc = 1;
        }
      }
      if (s_acc) {
        s_a = a;
        ip->f = ft;
      }
    }
    __syncthreads();
    if (s_acc) break;
  }
  const int trials = (t < st.ls_max ? t : st.ls_max - 1) + 1;
  if (!s_acc) {
    if (threadIdx.x == 0) {
      ip->status = ST_LS_FAIL;
      ip->active = 0;
      ip->trials += trials;
      ip->alpha = 0.0;
      ip->alphas[ip->iter] = 0.0;
      d.info[b].done = 1;
    }
    return;
  }
  const double a = s_a;
  if (threadIdx.x == 0) {
    if (!s_ftype && ip->nfilt < PL_IP_MAXFILT) {
      ip->filt[2 * ip->nfilt] = (1.0 - GAMMA_THETA) * theta;
      ip->filt[2 * ip->nfilt + 1] = phi - GAMMA_PHI * theta;
      ip->nfilt++;
    }
    ip->alpha = a;
    ip->alpha_z = az;
    ip->trials += trials;
    ip->alphas[ip->iter] = a;
  }
  for (int j = threadIdx.x; j < n; j += 256) x[j] = x[j] + a * dx[j];
  for (int r = threadIdx.x; r < m; r += 256) {
    const double l = lbg[r], u = ubg[r];
    const RowKind rk = row_kind(l, u);
    lam[r] = lam[r] + a * dl[r];
    if (rk.eq) continue;
    const double sl = rk.hl ? s[r] - l : 1.0, su = rk.hu ? u - s[r] : 1.0;
    const double dsr = ds[r];
    const double sn = s[r] + a * dsr;
    s[r] = sn;
    if (rk.hl) {
      const double dz = mu / sl - zl[r] - zl[r] / sl * dsr;
      const double sln = sn - l;
      const double z = zl[r] + az * dz;
      zl[r] = fmin(fmax(z, mu / (KAPPA_SIGMA * sln)), KAPPA_SIGMA * mu / sln);
    }
    if (rk.hu) {
      const double dz = mu / su - zu[r] + zu[r] / su * dsr;
      const double sun = u - sn;
      const double z = zu[r] + az * dz;
      zu[r] = fmin(fmax(z, mu / (KAPPA_SIGMA * sun)), KAPPA_SIGMA * mu / sun);
    }
  }
}

// ---------------------------------------------------------------------------------
// Per-problem stats into PlProbInfo (pl_stats): status, iterations, last step, f, viol.
__global__ void k_ip_finish(PlDev d, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const PlIpInfo* ip = d.ipinfo + b;
  PlProbInfo* info = d.info + b;
  info->status = ip->status;
  info->iter = ip->iter;
  info->ls_accepted = ip->status != ST_LS_FAIL;
  info->ls_branch = 0;
  info->ls_trials = ip->trials;
  info->ls_alpha = ip->alpha;
  info->viol_max = ip->viol_max;
  info->pri_res = ip->err;
  info->dua_res = ip->mu;
  info->f = ip->f;
}

#define PL_DISPATCH_DYN(dyn, KERNEL, ...)                                          \
  switch (dyn) {                                                                    \
    case PL_DYN_RNEA: hipLaunchKernelGGL(KERNEL<PL_DYN_RNEA>, __VA_ARGS__); break; \
    case PL_DYN_ACC: hipLaunchKernelGGL(KERNEL<PL_DYN_ACC>, __VA_ARGS__); break;   \
    case PL_DYN_CV: hipLaunchKernelGGL(KERNEL<PL_DYN_CV>, __VA_ARGS__); break;     \
    case PL_DYN_CA: hipLaunchKernelGGL(KERNEL<PL_DYN_CA>, __VA_ARGS__); break;     \
    case PL_DYN_ACCNB: hipLaunchKernelGGL(KERNEL<PL_DYN_ACCNB>, __VA_ARGS__); break; \
    case PL_DYN_CVNB: hipLaunchKernelGGL(KERNEL<PL_DYN_CVNB>, __VA_ARGS__); break;   \
    default: hipLaunchKernelGGL(KERNEL<PL_DYN_ABA>, __VA_ARGS__); break;           \
  }

#define PL_IP_INERTIA_CAP 8  // shifts per Newton system (1e-4 x 100^7 = 1e10 from a clean start)

// Factor the Newton system, with the inertia correction when the Lagrangian Hessian is in
// it (the Gauss-Newton system is positive definite by construction).
static void ip_factor(PlOcpHandle* h) {
  const bool exact = h->ip_hess == PL_IP_HESS_EXACT;
  h->fac_hlag = exact ? 1 : 0;
  if (!exact) {
    launch_factor(h);
    return;
  }
  launch_factor_pre(h);
  launch_factor_core(h);
  for (int r = 0; r <= PL_IP_INERTIA_CAP; ++r) {
    hipLaunchKernelGGL(k_ip_inertia, dim3(h->B), dim3(256), 0, h->stream, h->d, h->n, PL_IP_INERTIA_CAP);
    if (r == PL_IP_INERTIA_CAP) break;
    h->fac_only = 1;
    launch_factor_core(h);
    h->fac_only = 0;
  }
  launch_factor_post(h);
  h->fac_hlag = 0;
}

static void ip_refine(PlOcpHandle* h, const PlIpSettings& st, int iref) {
  hipLaunchKernelGGL(k_ip_refine, dim3(h->B), dim3(256), 0, h->stream, h->d, h->N, h->n, h->m, h->nnz, st.delta_w,
                     h->ip_hess == PL_IP_HESS_EXACT ? 1 : 0, h->hl_stride,
                     make_int4(h->hnz_off[0], h->hnz_off[1], h->hnz_off[2], h->hnz_off[3]), h->oc.tau_nodes, iref,
                     (h->debug_paths & PL_PATH_IP_REFINE_GATHER) ? 1 : 0);
}

// One interior-point solve of every problem from d.x (the warm start), enqueued on the
// handle's stream.  Kernels of terminated problems return at once.
void enqueue_ip(PlOcpHandle* h) {
  const PlIpSettings st = h->ip;
  const PlSettings saved = h->set;
  launch_eval_values(h, h->d.x);
  hipLaunchKernelGGL(k_ip_init, dim3(h->B), dim3(256), 0, h->stream, h->d, h->m, st, h->ip_lam_warm);
  h->d.ipskip = h->d.ipinfo;  // from here on the terminated problems skip evaluation and factor
  h->set.sigma = st.delta_w;  // factor: Ps + delta_w on the diagonal
  h->set.alpha = 1.0;         // ADMM sweep: x = x~, z = A x~
  for (int k = 0; k <= st.max_iter; ++k) {
    if (k > 0) launch_eval_values(h, h->d.x);
    launch_objective(h);
    launch_eval_jac(h);
    hipLaunchKernelGGL(k_ip_kkt, dim3(h->B), dim3(256), 0, h->stream, h->d, h->N, h->n, h->m, h->nnz,
                       std::max(h->ncpl_max, 1), k, st);
    if (k == st.max_iter) break;
    if (h->ip_hess == PL_IP_HESS_EXACT) launch_lag_hess(h);
    ip_factor(h);
    launch_admm_init(h);
    launch_admm(h, 1, 0, 0);
    for (int r = 0; r < st.n_refine; ++r) {
      ip_refine(h, st, r);
      launch_admm_init_zero(h);  // k_ip_refine zeroed x, z, y
      launch_admm(h, 1, 0, 0);
    }
    PL_DISPATCH_DYN(h->oc.dyn, k_ip_step, dim3(h->B), dim3(256), 0, h->stream, h->d, h->N, h->n, h->m, h->np, st,
                    0);
  }
  h->set = saved;
  h->d.ipskip = nullptr;
  hipLaunchKernelGGL(k_ip_finish, dim3((h->B + 63) / 64), dim3(64), 0, h->stream, h->d, h->B);
}

// Teacher-forced Newton direction from a given interior-point state (x in d.x; s, lam,
// zl, zu, mu uploaded by pl_debug_ip_direction): eval, KKT, factor, solve + refinement,
// directions and step bounds; no line search, no update.
void enqueue_ip_direction(PlOcpHandle* h) {
  const PlIpSettings st = h->ip;
  const PlSettings saved = h->set;
  h->set.sigma = st.delta_w;
  h->set.alpha = 1.0;
  launch_eval_values(h, h->d.x);
  launch_objective(h);
  launch_eval_jac(h);
  hipLaunchKernelGGL(k_ip_kkt, dim3(h->B), dim3(256), 0, h->stream, h->d, h->N, h->n, h->m, h->nnz,
                     std::max(h->ncpl_max, 1), -1, st);
  if (h->ip_hess == PL_IP_HESS_EXACT) launch_lag_hess(h);
  ip_factor(h);
  launch_admm_init(h);
  launch_admm(h, 1, 0, 0);
  for (int r = 0; r < st.n_refine; ++r) {
    ip_refine(h, st, r);
    launch_admm_init_zero(h);
    launch_admm(h, 1, 0, 0);
  }
  PL_DISPATCH_DYN(h->oc.dyn, k_ip_step, dim3(h->B), dim3(256), 0, h->stream, h->d, h->N, h->n, h->m, h->np, st, 1);
  h->set = saved;
}
