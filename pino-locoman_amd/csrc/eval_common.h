// Device helpers shared by the evaluation kernels (k_eval.hip) and the interior-point
// kernels (k_ip.hip): objective value / gradient over one problem and block reductions.
#pragma once
#include "state.h"
#include "targets.h"

// Objective f and gradient at d.x (ocp.py:80-101; ocp_whole_body_rnea.py:108-136).
// One workgroup per problem.  f is written to work[b * 8 + 0].
template <bool kGrad>
__device__ inline double objective_wg(const PlDev& d, int b, int N, int n, int np, const double* x, const double* step,
                               double alpha, double* grad, double* red) {  // red: >= 256 doubles of LDS
  const PlOcpConst& O = *d.oc;
  const PlModel& M = *d.model;
  const double* p = d.p + (size_t)b * np;
  __shared__ double dxd[2 * PL_MAXV];
  if (threadIdx.x == 0) pl::compute_dx_des(M, O, p, dxd);
  __syncthreads();
  const int ndx = O.ndx;
  const double* Q = p + O.P.Q_diag;
  const double* R = p + O.P.R_diag;
  // 256 virtual threads (partial vt sums j = vt, vt + 256, ...) and a 256-wide tree, for
  // any blockDim <= 256: the same summation order, hence the same bits, in every kernel
  for (int vt = threadIdx.x; vt < 256; vt += blockDim.x) {
  double acc = 0.0;
  for (int j = vt; j < n; j += 256) {
    const int i = d.colnode[j];
    const int lc = j - d.nodes[i].x_off;
    const double xj = step ? x[j] + alpha * step[j] : x[j];
    double gj;
    if (lc < ndx) {
      double e = xj - dxd[lc];
      acc += e * (Q[lc] * e);
      gj = 2.0 * Q[lc] * e;
    } else {
      int k = lc - ndx;
      double e = xj - pl::u_des(M, O, p, k);
      acc += e * (R[k] * e);
      gj = 2.0 * R[k] * e;
      if (PL_IS_RNEA(O.dyn) && i == 0 && k >= O.na + O.nf) {
        int t = k - O.na - O.nf;
        double W = p[O.P.W_diag + t];
        double et = xj - p[O.P.tau_prev + t];
        acc += et * (W * et);
        gj += 2.0 * W * et;
      }
    }
    if (kGrad) grad[j] = gj;
  }
  red[vt] = acc;
  }
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    for (int u = threadIdx.x; u < s; u += blockDim.x) red[u] += red[u + s];
    __syncthreads();
  }
  double f = red[0];
  __syncthreads();
  return f;
}


// Sum of red[0..256) into red[0] and max of red[256..512) into red[256] over a fixed
// 256-wide tree, whatever blockDim (<= 256) does the work.
__device__ inline void block_tree_256(double* red) {
  __syncthreads();
  for (int k = 128; k > 0; k >>= 1) {
    for (int u = threadIdx.x; u < k; u += blockDim.x) {
      red[u] += red[u + k];
      red[256 + u] = fmax(red[256 + u], red[256 + u + k]);
    }
    __syncthreads();
  }
}

__device__ inline void block_sum_max(double& s, double& mx, double* red) {
  // 256 partials (threads past blockDim contribute 0: the sums and the non-negative
  // maxima reduced here keep their 256-thread bits for any blockDim <= 256)
  red[threadIdx.x] = s;
  red[256 + threadIdx.x] = mx;
  for (int u = blockDim.x + threadIdx.x; u < 256; u += blockDim.x) {
    red[u] = 0.0;
    red[256 + u] = 0.0;
  }
  block_tree_256(red);
  s = red[0];
  mx = red[256];
  __syncthreads();
}

