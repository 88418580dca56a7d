// Device helpers shared by the evaluation kernels (k_eval.hip) and the interior-point
// kernels (k_ip.hip): objective value / gradient over one problem and block reductions.
#pragma once
#include "state.h"
#include "targets.h"

// Objective f and gradient at d.x (ocp.py:80-101; ocp_whole_body_rnea.py:108-136).
// One workgroup per problem.  f is written to work[b * 8 + 0].
template <bool kGrad>
__device__ inline double objective_wg(const PlDev& d, int b, int N, int n, int np, const double* x, const double* step,
                               double alpha, double* grad) {
  const PlOcpConst& O = *d.oc;
  const PlModel& M = *d.model;
  const double* p = d.p + (size_t)b * np;
  __shared__ double dxd[2 * PL_MAXV];
  __shared__ double red[256];
  if (threadIdx.x == 0) pl::compute_dx_des(M, O, p, dxd);
  __syncthreads();
  const int ndx = O.ndx;
  const double* Q = p + O.P.Q_diag;
  const double* R = p + O.P.R_diag;
  double acc = 0.0;
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
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
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  double f = red[0];
  __syncthreads();
  return f;
}


__device__ inline void block_sum_max(double& s, double& mx, double* red) {
  red[threadIdx.x] = s;
  red[256 + threadIdx.x] = mx;
  __syncthreads();
  for (int k = blockDim.x / 2; k > 0; k >>= 1) {
    if (threadIdx.x < k) {
      red[threadIdx.x] += red[threadIdx.x + k];
      red[256 + threadIdx.x] = fmax(red[256 + threadIdx.x], red[256 + threadIdx.x + k]);
    }
    __syncthreads();
  }
  s = red[0];
  mx = red[256];
  __syncthreads();
}

