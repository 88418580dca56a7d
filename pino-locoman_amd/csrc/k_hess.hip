// Lagrangian Hessian of the interior-point branch: the curvature of lam^T g that CasADi's
// exact Hessian gives the reference's Fatrop solve (optimization/ocp.py:248-263, Opti with
// expand=True).  The rows of node i depend on w_i = [dx_i, u_i] and linearly on dx_{i+1}
// (the integration rows dx_{i+1} - (dx_i + f dt), rows.h), so
//     H_L = diag(objective Hessian) + sum_i H_i,   H_i = sum_{rows r of node i} lam_r d^2 g_r / dw_i^2
// is block diagonal over the w_i: the same sparsity as the factor's diagonal blocks Kt_ii.
//
// The work list d.hlist holds the (node i, column pair j <= k of w_i) pairs (api.hip
// build_hess_list; pairs with an rnea tau_j column are structurally zero and not listed).  A
// pair's node rows are evaluated in hyper-dual numbers seeded on columns j and k (ad.h HDual)
// and the e1 e2 parts contracted with lam: H_i[k][j] = sum_r lam_r g_r.c, written packed lower
// (k (k + 1) / 2 + j from the node's offset d.hoff[i]), the layout k_fnode assembles Kt_ii in.
#include "dyn.h"
#include "eval_common.h"

using pl::VecIn;

namespace {

struct HessEmit {
  const double* lam;  // the node's rows
  double acc;
  int r;
  __device__ void operator()(const HDual& v, double, double) {
    acc = fma(lam[r], v.c, acc);
    ++r;
  }
};

}  // namespace

// k_lag_hess_pb: one pair per wave and one PROBLEM per lane (grid: pairs x problem groups of
// 64): the seeds are wave-uniform, so the row code's seed tests (tree passes a pair does not
// depend on are skipped) are scalar branches and every lane runs the same path.  (Until r04 a
// kernel with one pair per lane ran beside it, 298 against 254 ms per evaluation at the
// headline: removed.)
template <int DYN>
__global__ __launch_bounds__(64) void k_lag_hess_pb(PlDev d, int B, int N, int n, int m, int np, long long hl_stride) {
  const int b = blockIdx.y * 64 + threadIdx.x;
  if (b >= B || !d.ipinfo[b].active) return;
  const PlOcpConst& O = *d.oc;
  const PlModel& M = *d.model;
  const double* x = d.x + (size_t)b * n;
  const double* p = d.p + (size_t)b * np;
  const double* lam = d.ip_lam + (size_t)b * m;
  double* H = d.Hlag + (size_t)b * hl_stride;
  const int ndx = O.ndx;
  HDual kst[PL_KIN_STORE];
  const int2 w = d.hlist[blockIdx.x];
  const int wx = __builtin_amdgcn_readfirstlane(w.x);
  const int i = wx & 0xffff, only_ch = (wx >> 16) - 1;  // the pair's chain (api.hip set_solver)
  const int jk = __builtin_amdgcn_readfirstlane(w.y);
  const int j = jk & 0xffff, k = jk >> 16;
  const PlNode nd = d.nodes[i];
  const PlNode nn = d.nodes[i + 1];
  VecIn<HDual> dx{x + nd.x_off, nullptr, 0.0, j, k};
  VecIn<HDual> u{x + nd.x_off + ndx, nullptr, 0.0, j - ndx, k - ndx};
  VecIn<HDual> dxn{x + nn.x_off, nullptr, 0.0, j - nd.nw, k - nd.nw};
  HessEmit e{lam + nd.row_off, 0.0, 0};
  pl::node_rows<HDual, DYN>(M, O, i, p, dx, u, dxn, e, kst, 1, nullptr, nullptr, nullptr, only_ch);
  H[d.hoff[i] + k * (k + 1) / 2 + j] = e.acc;
}

// whole_body_rnea (u = [a | f | tau_j]): the rows are linear in a and in the contact forces,
// and only the RNEA rows (base rows and, on the tau nodes, the joint-torque rows; lambda_tau =
// their multipliers as a vector over v) couple them to q, through tau = M(q) a - sum_e J_e(q)^T f_e
// + ... (the DYNV rows are linear in a with constant coefficients, the force rows do not read
// q).  So for a dq column k
//     d^2 L / dq_k da   = d/dq_k [M(q) lambda_tau]        (one RNEA pass at v = 0, a = lambda_tau,
//                                                          f = 0 on the zero-gravity model)
//     d^2 L / dq_k df_e = -d/dq_k [J_e(q) lambda_tau]     (the foot velocities at v = lambda_tau)
// two dual tree passes seeded on dq_k give the whole (dq_k, a) and (dq_k, f_feet) rows of the
// node's block (k_lag_hess_pb would run one hyper-dual pass per pair: ~400 of a B2G node's
// ~1000).  One dq column per wave, one problem per lane.
namespace {
struct ZeroIn {
  PL_HD Dual operator[](int) const { return Dual(0.0, 0.0); }
};
struct LamIn {  // lambda_tau over v: the base rows' multipliers, then the joint-torque rows' (or 0)
  const double* lb;
  const double* lt;
  PL_HD Dual operator[](int k) const { return Dual(k < 6 ? lb[k] : (lt ? lt[k - 6] : 0.0), 0.0); }
};
}  // namespace

__global__ __launch_bounds__(64) void k_lag_hess_lin(PlDev d, int B, int n, int m, int np, long long hl_stride,
                                                     int3 rb_base, int3 rb_tau) {
  const int b = blockIdx.y * 64 + threadIdx.x;
  if (b >= B || !d.ipinfo[b].active) return;
  const PlOcpConst& O = *d.oc;
  const int2 w = d.hlin[blockIdx.x];
  const int i = __builtin_amdgcn_readfirstlane(w.x);
  const int wy = __builtin_amdgcn_readfirstlane(w.y);
  const int k = wy & 0xffff, only_ch = (wy >> 16) - 1;  // dq_k's chain (-1: a base coordinate)
  const PlNode nd = d.nodes[i];
  const double* p = d.p + (size_t)b * np;
  const double* lam = d.ip_lam + (size_t)b * m + nd.row_off;
  double* H = d.Hlag + (size_t)b * hl_stride + d.hoff[i];
  const int type = pl::node_type(O, i);
  const int rbb = type == 0 ? rb_base.x : (type == 1 ? rb_base.y : rb_base.z);
  const int rbt = type == 0 ? rb_tau.x : (type == 1 ? rb_tau.y : rb_tau.z);
  const LamIn lt{lam + rbb, rbt >= 0 ? lam + rbt : nullptr};
  const double* xi = p + O.P.x_init;
  const pl::VecIn<Dual> dq{d.x + (size_t)b * n + nd.x_off, nullptr, 0.0, k};
  Dual qb[7];
  pl::integrate_ff<Dual>(xi, dq, qb);
  const pl::RevQ<Dual, pl::VecIn<Dual>> qrev{xi, dq};
  Dual kst[PL_KIN_STORE];
  pl::NodeKin<Dual> kin;
  kin.vst = reinterpret_cast<double*>(kst);
  kin.dst = kin.vst + 1;
  kin.vstride = kin.dstride = 2;
  const int ndx = O.ndx, nv = O.nv;
  const auto slot = [&](int col) { return (size_t)col * (col + 1) / 2 + k; };  // (k, col) with k < col
  // (dq_k, a_j) = d/dq_k [M(q) lambda_tau]_j
  pl::tree_pass<Dual>(*d.model0, O, qb, qrev, ZeroIn{}, lt, ZeroIn{}, true, false, kin, nullptr, std::false_type{},
                      only_ch);
  for (int j = 0; j < nv; ++j) {
    const double t = j < 6 ? kin.tau[j].d : Dual(kin.tau_j(j - 6)).d;
    H[slot(ndx + j)] = t;
  }
  // (dq_k, f_e) = -d/dq_k [J_e(q) lambda_tau]   (feet)
  pl::tree_pass<Dual>(*d.model, O, qb, qrev, lt, ZeroIn{}, ZeroIn{}, false, true, kin, nullptr, std::false_type{},
                      only_ch);
  const int f0 = ndx + O.na;
  for (int e = 0; e < O.nfeet; ++e)
    for (int c = 0; c < 3; ++c) H[slot(f0 + 3 * e + c)] = -Dual(kin.foot_vel(e, c)).d;
}

#define PL_DISPATCH_DYN(dyn, KERNEL, ...)                                            \
  switch (dyn) {                                                                      \
    case PL_DYN_RNEA: hipLaunchKernelGGL(KERNEL<PL_DYN_RNEA>, __VA_ARGS__); break;   \
    case PL_DYN_ACC: hipLaunchKernelGGL(KERNEL<PL_DYN_ACC>, __VA_ARGS__); break;     \
    case PL_DYN_CV: hipLaunchKernelGGL(KERNEL<PL_DYN_CV>, __VA_ARGS__); break;       \
    case PL_DYN_CA: hipLaunchKernelGGL(KERNEL<PL_DYN_CA>, __VA_ARGS__); break;       \
    case PL_DYN_ACCNB: hipLaunchKernelGGL(KERNEL<PL_DYN_ACCNB>, __VA_ARGS__); break; \
    case PL_DYN_CVNB: hipLaunchKernelGGL(KERNEL<PL_DYN_CVNB>, __VA_ARGS__); break;   \
    default: hipLaunchKernelGGL(KERNEL<PL_DYN_ABA>, __VA_ARGS__); break;             \
  }

void launch_lag_hess(PlOcpHandle* h) {
  const bool prof = h->profile && h->prof_hn < 16;  // pl_mpc_step collects the slots before every step
  if (prof) hipEventRecord(h->prof_hev[h->prof_hn][0], h->stream);
  if (h->hlin_len > 0)
    hipLaunchKernelGGL(k_lag_hess_lin, dim3(h->hlin_len, (h->B + 63) / 64), dim3(64), 0, h->stream, h->d, h->B, h->n,
                       h->m, h->np, h->hl_stride, make_int3(h->hl_rb_base[0], h->hl_rb_base[1], h->hl_rb_base[2]),
                       make_int3(h->hl_rb_tau[0], h->hl_rb_tau[1], h->hl_rb_tau[2]));
  PL_DISPATCH_DYN(h->oc.dyn, k_lag_hess_pb, dim3(h->hl_len, (h->B + 63) / 64), dim3(64), 0, h->stream, h->d, h->B, h->N,
                  h->n, h->m, h->np, h->hl_stride);
  if (prof) {
    hipEventRecord(h->prof_hev[h->prof_hn][1], h->stream);
    h->prof_hn++;
  }
}
