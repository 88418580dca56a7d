// Node evaluation kernels: constraint values, constraint Jacobian (forward-mode
// dual numbers), objective value + gradient, Hessian diagonal.
//
// Replaces the CasADi functions sqp_data / f_data / g_data / hess_data
// (optimization/ocp.py:283-296, 386, 441-452).  One horizon node of one problem
// is the unit of work: values use one thread per (problem, node); the Jacobian
// uses one single-wave workgroup per (problem, node, 64-column chunk) and one
// thread per local column, each thread seeding the tangent of its column and
// writing the column's entries of the fixed sparsity pattern (CSC order inside the node).
#include "dyn.h"
#include "eval_common.h"

using pl::VecIn;

namespace {

struct ValueEmit {
  double* g;
  double* lb;
  double* ub;
  int r;
  __device__ void operator()(double v, double l, double u) {
    g[r] = v;
    lb[r] = l;
    ub[r] = u;
    ++r;
  }
};

struct JacEmit {
  const int* rowidx;  // local rows of this column's entries (sorted)
  double* out;        // entry values of this column
  int ptr, end, r;
  __device__ void operator()(const Dual& v, double, double) {
    if (ptr < end && rowidx[ptr] == r) {
      out[ptr] = v.d;
      ++ptr;
    }
    ++r;
  }
  // a row block holding none of the column's remaining entries is not computed (r06)
  __device__ bool skip_block(int n) {
    if (ptr < end && rowidx[ptr] < r + n) return false;
    r += n;
    return true;
  }
};

__device__ inline void node_inputs(const PlDev& d, const PlNode& nd, const PlNode& nn, const double* x,
                                   const double* step, double alpha, int seed, VecIn<double>* dx, VecIn<double>* u,
                                   VecIn<double>* dxn, int ndx) {
  *dx = VecIn<double>{x + nd.x_off, step ? step + nd.x_off : nullptr, alpha, -1};
  *u = VecIn<double>{x + nd.x_off + ndx, step ? step + nd.x_off + ndx : nullptr, alpha, -1};
  *dxn = VecIn<double>{x + nn.x_off, step ? step + nn.x_off : nullptr, alpha, -1};
}

}  // namespace

// g, lbg, ubg at xsrc for every (problem, node).
template <int DYN>
__global__ __launch_bounds__(64) void k_eval_values(PlDev d, int B, int N, int n, int m, int np, const double* __restrict__ xsrc) {
  const int tid = blockIdx.x * blockDim.x + threadIdx.x;
  if (tid >= B * N) return;
  const int b = tid / N, i = tid - b * N;
  if (ip_skip(d, b)) return;
  const PlOcpConst& O = *d.oc;
  const PlModel& M = *d.model;
  const PlNode nd = d.nodes[i];
  const PlNode nn = d.nodes[i + 1];
  const double* x = xsrc + (size_t)b * n;
  const double* p = d.p + (size_t)b * np;
  VecIn<double> dx, u, dxn;
  node_inputs(d, nd, nn, x, nullptr, 0.0, -1, &dx, &u, &dxn, O.ndx);
  ValueEmit e{d.g + (size_t)b * m + nd.row_off, d.lbg + (size_t)b * m + nd.row_off,
              d.ubg + (size_t)b * m + nd.row_off, 0};
  __shared__ double kst[PL_KIN_STORE * 64];
  pl::node_rows<double, DYN>(M, O, i, p, dx, u, dxn, e, kst + threadIdx.x, 64);
}

// Constraint Jacobian values on the fixed pattern.  One lane = one (node, local column)
// of the work list d.jlist (api.hip build_jac_list): the columns that run the tree pass
// are packed 64 per wave across node boundaries, the cheap ones follow; grid (waves, B).
// Each lane seeds the tangent of its column and writes the column's entries (CSC order
// inside the node).  Single-wave blocks retire independently.
#ifndef PL_JAC_WAVES
#define PL_JAC_WAVES 1
#endif
template <int DYN>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(PL_JAC_WAVES)))
void k_eval_jac(PlDev d, int B, int N, int n, int np, int nnz, int jl_len) {
  const int b = blockIdx.y;
  if (ip_skip(d, b)) return;
  const int q = (int)blockIdx.x * 64 + threadIdx.x;
  // whole_body_rnea / _acc: a tree-pass column of chain c moves only chain c's terms (rows.h,
  // k_hess.hip), so its pass is confined to it (tree_pass only_ch; .y = column | (c + 1) << 16,
  // the list grouped by chain so that a wave walks one chain)
  constexpr bool CH = DYN == PL_DYN_RNEA || DYN == PL_DYN_ACC;
  constexpr int SLOTS = CH ? PL_JAC_SLOTS_CH : PL_JAC_SLOTS;
  const int first = d.jlist[blockIdx.x * 64].x;  // the wave's first node (never padding)
  const bool valid = q < jl_len && d.jlist[min(q, jl_len - 1)].x >= 0;
  const int2 jw = valid ? d.jlist[q] : make_int2(first, 0);
  const int i = jw.x, lc = jw.y & 0xffff, only_ch = CH ? (jw.y >> 16) - 1 : -1;
  const int slot = min(i - first, SLOTS - 1);
  // kinematic outputs: per-lane tangents + one shared value per entry and node of the
  // wave (NodeKin<Dual>; the cheap columns read no stored value)
  __shared__ double kst_tan[PL_KIN_STORE_DUAL * 64];
  __shared__ double kst_val[SLOTS * PL_KIN_STORE_DUAL];
  double* aba_slot = nullptr;
  if constexpr (DYN == PL_DYN_ABA) {
    // the shared primal of each node of the wave (tree-pass columns only): its lanes split
    // the nv + 2 RNEA columns (raw, in kst_tan before node_rows uses it), then the node's
    // first lane factors M and solves for a
    __shared__ double aba_sh[PL_JAC_SLOTS * PL_ABA_SH];
    aba_slot = aba_sh + slot * PL_ABA_SH;
    const int nv = d.oc->nv;
    double* raw = kst_tan + slot * ((PL_KIN_STORE_DUAL * 64) / PL_JAC_SLOTS);
    const bool tree = valid && lc < d.nodes[i].nw;
    int s0 = threadIdx.x, s1 = threadIdx.x;  // this lane's node segment [s0, s1]
    const int wb = (int)blockIdx.x * 64;
    if (tree) {
      while (s0 > 0 && d.jlist[wb + s0 - 1].x == i) --s0;
      while (s1 < 63 && wb + s1 + 1 < jl_len && d.jlist[wb + s1 + 1].x == i) ++s1;
    }
    const double* pb = d.p + (size_t)b * np;
    const double* dxi = d.x + (size_t)b * n + d.nodes[i].x_off;
    if (tree)
      for (int c = threadIdx.x - s0; c < nv + 2; c += s1 - s0 + 1) pl::aba_primal_column(*d.model, *d.oc, pb, dxi, c, raw + c * nv);
    __syncthreads();
    if (tree && threadIdx.x == s0) pl::aba_primal_finish(*d.oc, dxi, raw, aba_slot);
    __syncthreads();
  }
  if (!valid) return;
  const PlNode nd = d.nodes[i];
  const int* cp = d.colptr + nd.colptr_off;
  const int e0 = cp[lc], e1 = cp[lc + 1];
  const PlOcpConst& O = *d.oc;
  const PlModel& M = *d.model;
  const PlNode nn = d.nodes[i + 1];
  const double* x = d.x + (size_t)b * n;
  const double* p = d.p + (size_t)b * np;
  const int ndx = O.ndx;
  VecIn<Dual> dx{x + nd.x_off, nullptr, 0.0, lc};
  VecIn<Dual> u{x + nd.x_off + ndx, nullptr, 0.0, lc - ndx};
  VecIn<Dual> dxn{x + nn.x_off, nullptr, 0.0, lc - nd.nw};
  JacEmit e{d.rowidx + nd.ent_off, d.Araw + (size_t)b * nnz + nd.ent_off, e0, e1, 0};
  pl::node_rows<Dual, DYN>(M, O, i, p, dx, u, dxn, e, reinterpret_cast<Dual*>(kst_tan + threadIdx.x), 64,
                           kst_val + slot * PL_KIN_STORE_DUAL, aba_slot, nullptr, only_ch);
}

namespace {
struct ZeroInD {
  PL_HD double operator[](int) const { return 0.0; }
};
struct UnitIn {  // e_k (k < 0: zero)
  int k;
  PL_HD double operator[](int j) const { return j == k ? 1.0 : 0.0; }
};
}  // namespace

// The RNEA's acceleration and contact-force columns (whole_body_rnea, whole_body_acc): tau is linear in a
// and f, so d tau / d a_k = M(q) e_k and d tau / d f_c = -J_c(q)^T e_c are one primal
// RNEA pass of the zero-gravity model at v = 0 with a = e_k (or f = e_c) instead of a dual
// tree pass (ocp_whole_body_rnea.py:207-235, pin.rnea with the contact forces).  One lane =
// one (node, column) of d.jlin (api_build.hip build_jac_list), grouped by the one chain the
// column moves (a joint acceleration or a foot force: the pass skips the other chains); the
// pass leaves the joint torques in the first nj slots of the lane's store, which node_rows
// then reads as tangents.
template <int DYN>
__global__ __launch_bounds__(64) void k_eval_jac_lin(PlDev d, int B, int n, int np, int nnz, int len) {
  const int b = blockIdx.y;
  if (ip_skip(d, b)) return;
  const int q = (int)blockIdx.x * 64 + threadIdx.x;
  __shared__ double kst[PL_KIN_STORE * 64];
  __shared__ double kval[PL_KIN_STORE];  // the (unused) values of the kinematic outputs
  for (int k = threadIdx.x; k < PL_KIN_STORE; k += 64) kval[k] = 0.0;
  __syncthreads();
  if (q >= len) return;
  const int2 jw = d.jlin[q];
  if (jw.x < 0) return;
  const int i = jw.x, lc = jw.y & 0xffff, only_ch = (jw.y >> 16) - 1;
  const PlOcpConst& O = *d.oc;
  const PlNode nd = d.nodes[i];
  const PlNode nn = d.nodes[i + 1];
  const int ndx = O.ndx;
  const double* x = d.x + (size_t)b * n;
  const double* p = d.p + (size_t)b * np;
  const double* xi = p + O.P.x_init;
  const VecIn<double> dq{x + nd.x_off, nullptr, 0.0, -1};
  double qb[7];
  pl::integrate_ff<double>(xi, dq, qb);
  const pl::RevQ<double, VecIn<double>> qrev{xi, dq};
  pl::NodeKin<double> kp;
  kp.store = kst + threadIdx.x;
  kp.stride = 64;
  const int k = lc - ndx;  // a_k, or force component k - na
  pl::tree_pass<double>(*d.model0, O, qb, qrev, ZeroInD{}, UnitIn{k < O.na ? k : -1}, UnitIn{k - O.na}, true, false,
                        kp, nullptr, std::false_type{}, only_ch);
  double base[6];
  for (int r = 0; r < 6; ++r) base[r] = kp.tau[r];
  const int* cp = d.colptr + nd.colptr_off;
  VecIn<Dual> dx{x + nd.x_off, nullptr, 0.0, lc};
  VecIn<Dual> u{x + nd.x_off + ndx, nullptr, 0.0, lc - ndx};
  VecIn<Dual> dxn{x + nn.x_off, nullptr, 0.0, lc - nd.nw};
  JacEmit e{d.rowidx + nd.ent_off, d.Araw + (size_t)b * nnz + nd.ent_off, cp[lc], cp[lc + 1], 0};
  pl::node_rows<Dual, DYN>(*d.model, O, i, p, dx, u, dxn, e, reinterpret_cast<Dual*>(kst + threadIdx.x), 64, kval,
                           nullptr, base);
}

__global__ __launch_bounds__(256) void k_objective(PlDev d, int N, int n, int np) {
  const int b = blockIdx.x;
  if (ip_skip(d, b)) return;
  __shared__ double red[256];
  double f = objective_wg<true>(d, b, N, n, np, d.x + (size_t)b * n, nullptr, 0.0, d.grad + (size_t)b * n, red);
  if (threadIdx.x == 0) d.work[(size_t)b * 8 + 0] = f;
}

// Constant Hessian diagonal (ocp.py:293-296): 2Q on states, 2R on inputs,
// + 2W on tau_0 (rnea).
__global__ __launch_bounds__(256) void k_hess(PlDev d, int N, int n, int np) {
  const int b = blockIdx.x;
  const PlOcpConst& O = *d.oc;
  const double* p = d.p + (size_t)b * np;
  double* P = d.P + (size_t)b * n;
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    const int i = d.colnode[j];
    const int lc = j - d.nodes[i].x_off;
    double h;
    if (lc < O.ndx) {
      h = 2.0 * p[O.P.Q_diag + lc];
    } else {
      int k = lc - O.ndx;
      h = 2.0 * p[O.P.R_diag + k];
      if (PL_IS_RNEA(O.dyn) && i == 0 && k >= O.na + O.nf) h += 2.0 * p[O.P.W_diag + k - O.na - O.nf];
    }
    P[j] = h;
  }
}

#define PL_DISPATCH_DYN(dyn, KERNEL, ...)                                          \
  switch (dyn) {                                                                    \
    case PL_DYN_RNEA: hipLaunchKernelGGL(KERNEL<PL_DYN_RNEA>, __VA_ARGS__); break; \
    case PL_DYN_ACC: hipLaunchKernelGGL(KERNEL<PL_DYN_ACC>, __VA_ARGS__); break;   \
    case PL_DYN_CV: hipLaunchKernelGGL(KERNEL<PL_DYN_CV>, __VA_ARGS__); break;     \
    case PL_DYN_CA: hipLaunchKernelGGL(KERNEL<PL_DYN_CA>, __VA_ARGS__); break;     \
    case PL_DYN_ACCNB: hipLaunchKernelGGL(KERNEL<PL_DYN_ACCNB>, __VA_ARGS__); break; \
    case PL_DYN_CVNB: hipLaunchKernelGGL(KERNEL<PL_DYN_CVNB>, __VA_ARGS__); break;   \
    case PL_DYN_RNEAFD: hipLaunchKernelGGL(KERNEL<PL_DYN_RNEAFD>, __VA_ARGS__); break; \
    default: hipLaunchKernelGGL(KERNEL<PL_DYN_ABA>, __VA_ARGS__); break;           \
  }

void launch_eval_values(PlOcpHandle* h, const double* xsrc) {
  const int total = h->B * h->N;
  const int bs = 64;
  PL_DISPATCH_DYN(h->oc.dyn, k_eval_values, dim3((total + bs - 1) / bs), dim3(bs), 0, h->stream, h->d, h->B, h->N,
                  h->n, h->m, h->np, xsrc);
}

void launch_eval_jac(PlOcpHandle* h) {
  if (h->jlin_len > 0) {
    const dim3 g((h->jlin_len + 63) / 64, h->B);
    if (h->oc.dyn == PL_DYN_RNEA)
      hipLaunchKernelGGL(k_eval_jac_lin<PL_DYN_RNEA>, g, dim3(64), 0, h->stream, h->d, h->B, h->n, h->np, h->nnz,
                         h->jlin_len);
    else if (h->oc.dyn == PL_DYN_ACC)
      hipLaunchKernelGGL(k_eval_jac_lin<PL_DYN_ACC>, g, dim3(64), 0, h->stream, h->d, h->B, h->n, h->np, h->nnz,
                         h->jlin_len);
    else
      hipLaunchKernelGGL(k_eval_jac_lin<PL_DYN_RNEAFD>, g, dim3(64), 0, h->stream, h->d, h->B, h->n, h->np, h->nnz,
                         h->jlin_len);
  }
  // the cheap columns (after jl_ex) have constant entries: after the first evaluation their
  // waves are not launched (the entries stay in d.Araw; nothing else writes them)
  const int len = (h->jac_cheap_ok && !h->jac_cheap_every) ? h->jl_ex : h->jl_len;
  if (len > 0)
    PL_DISPATCH_DYN(h->oc.dyn, k_eval_jac, dim3((len + 63) / 64, h->B), dim3(64), 0, h->stream, h->d, h->B, h->N,
                    h->n, h->np, h->nnz, h->jl_len);
  h->jac_cheap_ok = 1;
}

void launch_objective(PlOcpHandle* h) {
  hipLaunchKernelGGL(k_objective, dim3(h->B), dim3(256), 0, h->stream, h->d, h->N, h->n, h->np);
}

void launch_hess(PlOcpHandle* h) {
  hipLaunchKernelGGL(k_hess, dim3(h->B), dim3(256), 0, h->stream, h->d, h->N, h->n, h->np);
}

// ---------------------------------------------------------------------------
// Armijo / filter line search (ocp.py:430-480), fused: one workgroup per
// problem evaluates f and the constraint-violation metric at each trial point
// x + a*dx (nodes on threads) and applies the reference's acceptance rules,
// including the quirk that f and g_metric are overwritten by every rejected
// trial (ocp.py:470-471).  Also records the max violation at the returned point
// (ocp.py:412-414).
namespace {
struct ViolEmit {
  double ss, mx;
  __device__ void operator()(double v, double l, double u) {
    double a = fmax(0.0, l - v), c = fmax(0.0, v - u);
    ss += a * a + c * c;
    mx = fmax(mx, fmax(a, c));
  }
};

template <int DYN>
__device__ void violation_at(const PlDev& d, int b, int N, int n, int np, const double* x, const double* step,
                             double alpha, double* kst, double* red, double* metric, double* vmax) {
  const PlOcpConst& O = *d.oc;
  const PlModel& M = *d.model;
  ViolEmit e{0.0, 0.0};
  for (int i = threadIdx.x; threadIdx.x < 64 && i < N; i += 64) {  // nodes on the first wave
    const PlNode nd = d.nodes[i];
    const PlNode nn = d.nodes[i + 1];
    VecIn<double> dx{x + nd.x_off, step ? step + nd.x_off : nullptr, alpha, -1};
    VecIn<double> u{x + nd.x_off + O.ndx, step ? step + nd.x_off + O.ndx : nullptr, alpha, -1};
    VecIn<double> dxn{x + nn.x_off, step ? step + nn.x_off : nullptr, alpha, -1};
    pl::node_rows<double, DYN>(M, O, i, d.p + (size_t)b * np, dx, u, dxn, e, kst + threadIdx.x, 64);
  }
  double s = e.ss, mx = e.mx;
  block_sum_max(s, mx, red);
  *metric = sqrt(s);
  *vmax = mx;
}
}  // namespace

// One wave per problem: the node rows of the trials run on 64 lanes and the ~350 registers
// of the row code fit one wave per SIMD, so a 256-thread workgroup (three idle waves)
// would hold a whole CU per problem.  Every sum keeps its 256-wide order (eval_common.h).
template <int DYN>
__global__ __launch_bounds__(64) void k_line_search(PlDev d, int N, int n, int m, int np) {
  const int b = blockIdx.x;
  // the node rows' store; also the reduction buffer once a pass over the rows is done
  // (one wave, in order), so the workgroup takes 39 KB of LDS and four fit a CU
  __shared__ double kst[PL_KIN_STORE * 64];
  static_assert(PL_KIN_STORE * 64 >= 512, "reduction buffer");
  double* red = kst;
  __shared__ int s_flag;
  double* x = d.x + (size_t)b * n;
  const double* dxs = d.step + (size_t)b * n;
  PlProbInfo* info = d.info + b;
  // NaN step (infeasible QP): every comparison is false -> "didn't converge"
  if (threadIdx.x == 0) s_flag = 0;
  __syncthreads();
  for (int j = threadIdx.x; j < n; j += blockDim.x)
    if (isnan(dxs[j])) s_flag = 1;
  __syncthreads();
  const bool nan_step = s_flag != 0;
  // f, grad_f, g metric at the current x (ocp.py:441-445)
  double f = objective_wg<false>(d, b, N, n, np, x, nullptr, 0.0, nullptr, red);
  double gm, vmax0;
  violation_at<DYN>(d, b, N, n, np, x, nullptr, 0.0, kst, red, &gm, &vmax0);
  double arm = 0.0;
  {
    const double* gr = d.grad + (size_t)b * n;
    for (int vt = threadIdx.x; vt < 256; vt += blockDim.x) {  // 256 virtual threads (eval_common.h)
      double s = 0.0;
      for (int j = vt; j < n; j += 256) s += gr[j] * dxs[j];
      red[vt] = s;
      red[256 + vt] = 0.0;
    }
    block_tree_256(red);
    arm = red[0];
    __syncthreads();
  }
  const double armijo_factor = 1e-4, a_min = 1e-4, a_decay = 0.5, g_max = 1e-3, g_min = 1e-5, gamma = 1e-5;
  double a = 1.0;
  bool accepted = false;
  int branch = 0, trials = 0;
  double new_f = f, new_gm = gm, vmax = vmax0;
  if (nan_step) {
    trials = 14;
  } else {
    while (!accepted && a > a_min) {
      new_f = objective_wg<false>(d, b, N, n, np, x, dxs, a, nullptr, red);
      violation_at<DYN>(d, b, N, n, np, x, dxs, a, kst, red, &new_gm, &vmax);
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
  if (accepted) {
    for (int j = threadIdx.x; j < n; j += blockDim.x) x[j] = x[j] + a_acc * dxs[j];
  }
  if (threadIdx.x == 0) {
    info->ls_accepted = accepted ? 1 : 0;
    info->ls_branch = branch;
    info->ls_trials = trials;
    info->ls_alpha = accepted ? a_acc : 0.0;
    info->viol_max = accepted ? vmax : vmax0;
    info->f = accepted ? new_f : f;
  }
}

void launch_line_search(PlOcpHandle* h) {
  PL_DISPATCH_DYN(h->oc.dyn, k_line_search, dim3(h->B), dim3(64), 0, h->stream, h->d, h->N, h->n, h->m, h->np);
}

// ---------------------------------------------------------------------------
// Device-side MPC loop glue (run_mpc.py:127-143).
// MPC step k, before the solve: parameters (x_init, gait schedule at
// t0 + k dt_min) and warm start (forces <- f_des masked by the new schedule;
// ocp_whole_body_rnea.py:207-235).  k == 0 keeps the initial guess.
__global__ __launch_bounds__(64) void k_mpc_prepare(PlDev d, int k, int N, int n, int np, int nx, int gait_type,
                                                    double period, double swing_period) {
  const int b = blockIdx.x;
  const PlOcpConst& O = *d.oc;
  const PlModel& M = *d.model;
  double* p = d.p + (size_t)b * np;
  for (int j = threadIdx.x; j < nx; j += blockDim.x) p[O.P.x_init + j] = d.xstate[(size_t)b * nx + j];
  if (threadIdx.x == 0) {
    double t = d.t0[b] + k * p[O.P.dt_min];
    pl::gait_schedule(O, gait_type, period, swing_period, t, p, p + O.P.contact, p + O.P.swing);
  }
  __syncthreads();
  if (k == 0) return;
  double* x = d.x + (size_t)b * n;
  const int fo = pl::u_force_off(O);
  for (int idx = threadIdx.x; idx < N * O.nf; idx += blockDim.x) {  // (node, force component) on the lanes
    const int i = idx / O.nf, c = idx - i * O.nf;
    const int base = d.nodes[i].x_off + O.ndx + fo;
    int foot = c / 3;
    double fd = pl::f_des_comp(M, O, p, c);
    if (foot < 4 && p[O.P.contact + 4 * i + foot] == 0.0) fd = 0.0;
    x[base + c] = fd;
  }
}

// After the solve: x_state <- integrate(x_state, DX_prev[1]) (run_mpc.py:142).
__global__ void k_mpc_finish(PlDev d, int B, int n, int nx) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const PlOcpConst& O = *d.oc;
  const PlModel& M = *d.model;
  double* xs = d.xstate + (size_t)b * nx;
  const double* dx1 = d.x + (size_t)b * n + d.nodes[1].x_off;
  double qn[PL_MAXQ];
  if (PL_IS_CV(O.dyn)) {  // x = [h, q]: h + dh, integrate(q, dq) (dynamics_centroidal_vel.py:12-26)
    VecIn<double> acc{dx1 + 6, nullptr, 0.0, -1};
    pl::integrate_q<double>(M, xs + 6, acc, qn);
    for (int k = 0; k < 6; ++k) xs[k] += dx1[k];
    for (int k = 0; k < O.nq; ++k) xs[6 + k] = qn[k];
    return;
  }
  VecIn<double> acc{dx1, nullptr, 0.0, -1};
  pl::integrate_q<double>(M, xs, acc, qn);
  for (int k = 0; k < O.nq; ++k) xs[k] = qn[k];
  for (int k = 0; k < O.nv; ++k) xs[O.nq + k] += dx1[O.nv + k];
}

void launch_mpc_prepare(PlOcpHandle* h, int k) {
  hipLaunchKernelGGL(k_mpc_prepare, dim3(h->B), dim3(64), 0, h->stream, h->d, k, h->N, h->n, h->np, h->nx,
                     h->gait_type, h->gait_period, h->swing_period);
}

void launch_mpc_finish(PlOcpHandle* h) {
  hipLaunchKernelGGL(k_mpc_finish, dim3((h->B + 63) / 64), dim3(64), 0, h->stream, h->d, h->B, h->n, h->nx);
}
