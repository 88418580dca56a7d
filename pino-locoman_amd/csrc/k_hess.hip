// Lagrangian Hessian of the interior-point branch: the curvature of lam^T g that CasADi's
// exact Hessian gives the reference's Fatrop solve (optimization/ocp.py:248-263, Opti with
// expand=True).  The rows of node i depend on w_i = [dx_i, u_i] and linearly on dx_{i+1}
// (the integration rows dx_{i+1} - (dx_i + f dt), rows.h), so
//     H_L = diag(objective Hessian) + sum_i H_i,   H_i = sum_{rows r of node i} lam_r d^2 g_r / dw_i^2
// is block diagonal over the w_i: the same sparsity as the factor's diagonal blocks Kt_ii.
//
// k_lag_hess: one lane per (node i, column pair j <= k of w_i) of the work list d.hlist
// (api.hip build_hess_list; pairs with an rnea tau_j column are structurally zero and not
// listed).  The lane evaluates node i's rows in hyper-dual numbers seeded on columns j and
// k (ad.h HDual) and contracts the e1 e2 parts with lam: H_i[k][j] = sum_r lam_r g_r.c,
// written packed lower (k (k + 1) / 2 + j from the node's offset d.hoff[i]), the layout
// k_fnode assembles Kt_ii in.  Grid (work-list blocks, B); the lanes' kinematic stores
// (NodeKin<HDual>) are private arrays.
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

template <int DYN>
__global__ __launch_bounds__(64) void k_lag_hess(PlDev d, int N, int n, int m, int np, int hl_len, long long hl_stride) {
  const int b = blockIdx.y;
  if (!d.ipinfo[b].active) return;
  const PlOcpConst& O = *d.oc;
  const PlModel& M = *d.model;
  const double* x = d.x + (size_t)b * n;
  const double* p = d.p + (size_t)b * np;
  const double* lam = d.ip_lam + (size_t)b * m;
  double* H = d.Hlag + (size_t)b * hl_stride;
  const int ndx = O.ndx;
  HDual kst[PL_KIN_STORE];
  for (int q = blockIdx.x * 64 + threadIdx.x; q < hl_len; q += gridDim.x * 64) {
    const int2 w = d.hlist[q];
    const int i = w.x, j = w.y & 0xffff, k = w.y >> 16;
    const PlNode nd = d.nodes[i];
    const PlNode nn = d.nodes[i + 1];
    VecIn<HDual> dx{x + nd.x_off, nullptr, 0.0, j, k};
    VecIn<HDual> u{x + nd.x_off + ndx, nullptr, 0.0, j - ndx, k - ndx};
    VecIn<HDual> dxn{x + nn.x_off, nullptr, 0.0, j - nd.nw, k - nd.nw};
    HessEmit e{lam + nd.row_off, 0.0, 0};
    pl::node_rows<HDual, DYN>(M, O, i, p, dx, u, dxn, e, kst, 1);
    H[d.hoff[i] + k * (k + 1) / 2 + j] = e.acc;
  }
}

// The same Hessian with one pair per wave and one PROBLEM per lane (grid: pairs x problem
// groups of 64): the seeds are wave-uniform, so the row code's seed tests (tree passes a pair
// does not depend on are skipped) are scalar branches and every lane runs the same path.
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
  const int i = __builtin_amdgcn_readfirstlane(w.x);
  const int jk = __builtin_amdgcn_readfirstlane(w.y);
  const int j = jk & 0xffff, k = jk >> 16;
  const PlNode nd = d.nodes[i];
  const PlNode nn = d.nodes[i + 1];
  VecIn<HDual> dx{x + nd.x_off, nullptr, 0.0, j, k};
  VecIn<HDual> u{x + nd.x_off + ndx, nullptr, 0.0, j - ndx, k - ndx};
  VecIn<HDual> dxn{x + nn.x_off, nullptr, 0.0, j - nd.nw, k - nd.nw};
  HessEmit e{lam + nd.row_off, 0.0, 0};
  pl::node_rows<HDual, DYN>(M, O, i, p, dx, u, dxn, e, kst, 1);
  H[d.hoff[i] + k * (k + 1) / 2 + j] = e.acc;
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
  const bool prof = h->profile && h->prof_hn < 16;
  if (prof) hipEventRecord(h->prof_hev[h->prof_hn][0], h->stream);
  if (h->hess_pb) {
    PL_DISPATCH_DYN(h->oc.dyn, k_lag_hess_pb, dim3(h->hl_len, (h->B + 63) / 64), dim3(64), 0, h->stream, h->d, h->B, h->N,
                    h->n, h->m, h->np, h->hl_stride);
  } else {
    const int blocks = std::min((h->hl_len + 63) / 64, std::max(1, 2048 / std::max(h->B, 1)));
    PL_DISPATCH_DYN(h->oc.dyn, k_lag_hess, dim3(blocks, h->B), dim3(64), 0, h->stream, h->d, h->N, h->n, h->m, h->np,
                    h->hl_len, h->hl_stride);
  }
  if (prof) {
    hipEventRecord(h->prof_hev[h->prof_hn][1], h->stream);
    h->prof_hn++;
  }
}
