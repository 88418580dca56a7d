// QP kernels: OSQP-0.6-equivalent scaling, KKT factorisation and ADMM.
//
// Replaces osqp.update(q, Ax, l, u) + osqp.solve() (optimization/ocp.py:391-401;
// OSQP settings ocp.py:267-273).  The KKT system OSQP factors with QDLDL,
//     [P + sigma I, A^T; A, -diag(rho)^-1],
// is solved here in its reduced SPD form K = P + sigma I + A^T diag(rho) A, which
// is block tridiagonal over the horizon (rows of node i touch w_i = [dx_i, u_i]
// and dx_{i+1}).  The factorisation keeps, per node, the EXPLICIT inverse
// S_i = Ktilde_ii^-1 of the Schur-complemented diagonal block (symmetric, lower
// 8x8 tiles only), so each ADMM iteration is two block sweeps that read S_i once
// each:
//     forward : bt_i = rhs_i - K_{i,i-1} w_{i-1},    w_i = S_i bt_i
//     backward: x_i  = S_i (bt_i - K_{i+1,i}^T x_{i+1})
// with the off-diagonal products applied directly from the (sparse) scaled A.
// z~ = A x~ and the z / y / rhs updates of the rows of node i are fused into the
// backward sweep, so A is read once per iteration.
//
// Layout of a node's factor block: work unit u = (lower tile t, half h) covers the
// 8x4 sub-block rows 0..7, cols 4h..4h+3 of tile t; element pair k (0..15) of
// unit u lives at s_off + (k * nunit + u) * 2 -> every 16-byte load instruction of
// a wave is one contiguous 1 KiB segment.
#include <algorithm>

#include "state.h"

#define PL_OSQP_INFTY 1e30
#define PL_MIN_SCALING 1e-4
#define PL_MAX_SCALING 1e4
#define PL_RHO_MIN 1e-6
#define PL_RHO_TOL 1e-4
#define PL_RHO_EQ_OVER_INEQ 1e3
#define PL_DIV_TOL 1e-30

enum {
  PL_ST_SOLVED = 1,
  PL_ST_SOLVED_INACCURATE = 2,
  PL_ST_MAX_ITER = -2,
  PL_ST_PRIMAL_INF = -3,
  PL_ST_PRIMAL_INF_INACC = 3,
  PL_ST_DUAL_INF = -4,
  PL_ST_DUAL_INF_INACC = 4,
  PL_ST_NON_CVX = -7,
  PL_ST_UNSOLVED = -10
};

namespace {

__device__ __forceinline__ double limit_scaling(double v) {
  v = v < PL_MIN_SCALING ? 1.0 : v;
  return v > PL_MAX_SCALING ? PL_MAX_SCALING : v;
}


// block reductions over 256 threads
__device__ double block_max(double v, double* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + s]);
    __syncthreads();
  }
  double r = red[0];
  __syncthreads();
  return r;
}
// max of K values per thread in one reduction (red: K x RS doubles, RS >= blockDim.x)
template <int K, int RS>
__device__ void block_max_k(double (&v)[K], double* red) {
#pragma unroll
  for (int k = 0; k < K; ++k) red[k * RS + threadIdx.x] = v[k];
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
#pragma unroll
      for (int k = 0; k < K; ++k) red[k * RS + threadIdx.x] = fmax(red[k * RS + threadIdx.x], red[k * RS + threadIdx.x + s]);
    }
    __syncthreads();
  }
#pragma unroll
  for (int k = 0; k < K; ++k) v[k] = red[k * RS];
  __syncthreads();
}
__device__ double block_sum(double v, double* red) {
  red[threadIdx.x] = v;
  __syncthreads();
  for (int s = blockDim.x / 2; s > 0; s >>= 1) {
    if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  double r = red[0];
  __syncthreads();
  return r;
}

}  // namespace

// ---------------------------------------------------------------------------
// OSQP data update + Ruiz equilibration (osqp_update_lin_cost / _bounds / _A and
// scale_data, OSQP 0.6 src/scaling.c).  D, E and the cost scale c are kept
// cumulatively against the raw data, so each pass needs
//   Dt_j = max(c D_j^2 |P_jj|, D_j max_r |A_rj| E_r),   Et_r = E_r max_j |A_rj| D_j.
// The norms of a pass run over a (problem x node) grid: the workgroup of node i
// owns its columns w_i (entries of node i plus node i-1's entries on dx_i) and
// its rows; the update of D, E and c is one workgroup per problem.
__global__ __launch_bounds__(256) void k_ruiz_init(PlDev d, int n, int m) {
  const int b = blockIdx.x;
  double* D = d.D + (size_t)b * n;
  double* E = d.E + (size_t)b * m;
  for (int j = threadIdx.x; j < n; j += blockDim.x) D[j] = 1.0;
  for (int r = threadIdx.x; r < m; r += blockDim.x) E[r] = 1.0;
  if (threadIdx.x == 0) d.cs[b] = 1.0;
}

// Norms of one pass for node i, from its A slice, D / E slices and its ADMM program
// staged in LDS (balanced chunk maxima, as the ADMM gathers):
//   Dt_j = max(c D_j^2 |P_jj|, D_j max over node i's entries of column j)  for j in w_i
//   Dx_j = max over node i's entries of column j                        for j in dx_{i+1}
//   Et_r = E_r max_j |A_rj| D_j                                         for the rows of node i
// k_ruiz_update folds D_j Dx_j into Dt_j (max is exact in any order).
__global__ __launch_bounds__(256) void k_ruiz_norms(PlDev d, int N, int n, int m, int nnz, int ndx, int nent_max,
                                                    int ncol_max, int nrow_max, int chunk_max) {
  extern __shared__ double lds[];
  const int b = blockIdx.x / (N + 1), i = blockIdx.x - b * (N + 1);
  typedef const __attribute__((address_space(4))) PlAdmmNode* CNode;
  CNode an = (CNode)d.anodes;
  const int nw = an[i].nw, nrow = an[i].nrow, nent = an[i].nent, ncol = an[i].ncol;
  const int x_off = an[i].x_off, row_off = an[i].row_off, ent_off = an[i].ent_off;
  const int prog = an[i].prog, plen = an[i].prog_len;
  double* As = lds;
  double* Dl = As + nent_max;
  double* El = Dl + ncol_max;
  double* cm = El + nrow_max;
  // the node program is read in place (L2-resident, shared by the batch): staging it
  // per (problem, node) block cost more L2 traffic than the A values themselves
  const uint16_t* __restrict__ P = d.aprog + prog;
  const double* A = d.Araw + (size_t)b * nnz + ent_off;
  const double* Pd = d.P + (size_t)b * n;
  const double* D = d.D + (size_t)b * n;
  const double* E = d.E + (size_t)b * m;
  double* Dt = d.dxs + (size_t)b * n;  // scratch
  double* Dx = d.aty + (size_t)b * n;  // scratch: dx_{i+1} column maxima of node i
  double* Et = d.dys + (size_t)b * m;  // scratch
  const double c = d.cs[b];
  const int tid = threadIdx.x;
  for (int k = tid; k < nent; k += 256) As[k] = A[k];
  for (int k = tid; k < ncol; k += 256) Dl[k] = D[x_off + k];  // w_i then dx_{i+1}: contiguous
  for (int k = tid; k < nrow; k += 256) El[k] = E[row_off + k];
  (void)plen;
  __syncthreads();
  // ---- columns
  const int cchn = an[i].cchn;
  {
    const uint8_t* colr = reinterpret_cast<const uint8_t*>(P + an[i].colr);
    const uint32_t* cch = reinterpret_cast<const uint32_t*>(P + an[i].cch);
    for (int ch = tid; ch < cchn; ch += 256) {
      const uint32_t w = cch[ch];
      const int e0 = w & 0xffff, e1 = (int)(w >> 16);
      double mx = 0.0;
      for (int e = e0; e < e1; ++e) mx = fmax(mx, fabs(As[e]) * El[colr[e]]);
      cm[ch] = mx;
    }
  }
  __syncthreads();
  for (int lc = tid; lc < nw; lc += 256) {
    double mx = 0.0;
    if (ncol) {
      const int k0 = P[an[i].cchptr + lc], k1 = P[an[i].cchptr + lc + 1];
      for (int k = k0; k < k1; ++k) mx = fmax(mx, cm[k]);
    }
    const int j = x_off + lc;
    const double dj = D[j];
    Dt[j] = fmax(c * dj * dj * fabs(Pd[j]), dj * mx);
    if (lc >= ndx || i == 0) Dx[j] = 0.0;  // no predecessor entries on these columns
  }
  for (int lc = nw + tid; lc < ncol; lc += 256) {  // dx_{i+1}: node i's share
    const int k0 = P[an[i].cchptr + lc], k1 = P[an[i].cchptr + lc + 1];
    double mx = 0.0;
    for (int k = k0; k < k1; ++k) mx = fmax(mx, cm[k]);
    Dx[x_off + lc] = mx;
  }
  __syncthreads();
  // ---- rows
  const int rchn = an[i].rchn;
  {
    const uint16_t* rowe = P + an[i].rowe;
    const uint8_t* rowc = reinterpret_cast<const uint8_t*>(P + an[i].rowc);
    const uint32_t* rch = reinterpret_cast<const uint32_t*>(P + an[i].rch);
    for (int ch = tid; ch < rchn; ch += 256) {
      const uint32_t w = rch[ch];
      const int q0 = w & 0xffff, q1 = (int)(w >> 16);
      double mx = 0.0;
      for (int q = q0; q < q1; ++q) mx = fmax(mx, fabs(As[rowe[q]]) * Dl[rowc[q]]);
      cm[ch] = mx;
    }
  }
  __syncthreads();
  for (int lr = tid; lr < nrow; lr += 256) {
    const int k0 = P[an[i].rchptr + lr], k1 = P[an[i].rchptr + lr + 1];
    double mx = 0.0;
    for (int k = k0; k < k1; ++k) mx = fmax(mx, cm[k]);
    Et[row_off + lr] = El[lr] * mx;
  }
}

// All passes of the equilibration in one launch, one 1024-thread workgroup per problem
// (the same D, E and c bit for bit as k_ruiz_norms + k_ruiz_update: maxima are exact in
// any order, D_j max(a, b) = max(D_j a, D_j b) under monotone rounding, and the cost sum
// keeps k_ruiz_update's 256-thread order).  D and E live in LDS for the whole launch; a
// pass reads the problem's A twice (column maxima with the old E, then row maxima with the
// old D) in entry order, coalesced, into one LDS buffer of maxima (ds_max_u64 on the bit
// patterns of the non-negative products; NaN products are skipped as fmax does).  With
// one workgroup per CU the A slices of the resident problems (~0.36 MB each at the
// headline size) stay in the Infinity Cache across the passes, so HBM sees A about once.
namespace {
__device__ __forceinline__ void lds_max_bits(unsigned long long* p, double v) {
  if (v == v) __hip_atomic_fetch_max(p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_WORKGROUP);
}
constexpr int RUIZ_NT = 1024, RUIZ_PER = 8;  // n, m <= RUIZ_NT x RUIZ_PER
constexpr int RUIZ_U = 16;                   // entries per thread with loads in flight together

// f(coordinates, |A_e|) over the problem's entries, RUIZ_U loads per thread issued together
template <class F>
__device__ __forceinline__ void ruiz_sweep(const double* A, const uint32_t* erc, int nnz, F f) {
  const int tid = threadIdx.x;
  for (int e0 = 0; e0 < nnz; e0 += RUIZ_U * RUIZ_NT) {
    uint32_t w[RUIZ_U];
    double a[RUIZ_U];
#pragma unroll
    for (int u = 0; u < RUIZ_U; ++u) {
      const int e = min(e0 + u * RUIZ_NT + tid, nnz - 1);
      w[u] = erc[e];
      a[u] = A[e];
    }
#pragma unroll
    for (int u = 0; u < RUIZ_U; ++u)
      if (e0 + u * RUIZ_NT + tid < nnz) f(w[u], fabs(a[u]));
  }
}
}  // namespace

__global__ __launch_bounds__(RUIZ_NT) void k_ruiz_fused(PlDev d, int n, int m, int nnz, int passes) {
  extern __shared__ double lds[];
  __shared__ double red[256];
  __shared__ double c_sh;
  const int b = blockIdx.x, tid = threadIdx.x;
  double* Dl = lds;
  double* El = Dl + ((n + 1) & ~1);
  unsigned long long* mx = reinterpret_cast<unsigned long long*>(El + ((m + 1) & ~1));
  const double* A = d.Araw + (size_t)b * nnz;
  const double* P = d.P + (size_t)b * n;
  const double* q = d.grad + (size_t)b * n;
  const uint32_t* __restrict__ erc = d.erc;
  for (int j = tid; j < n; j += RUIZ_NT) Dl[j] = 1.0;
  for (int r = tid; r < m; r += RUIZ_NT) El[r] = 1.0;
  double c = 1.0;
  double Pa[RUIZ_PER];
#pragma unroll
  for (int k = 0; k < RUIZ_PER; ++k) {
    const int j = tid + RUIZ_NT * k;
    Pa[k] = j < n ? fabs(P[j]) : 0.0;
  }
  for (int pass = 0; pass < passes; ++pass) {
    // ---- column maxima max_r |A_rj| E_r -> Dt_j
    for (int j = tid; j < n; j += RUIZ_NT) mx[j] = 0ull;
    __syncthreads();
    ruiz_sweep(A, erc, nnz, [&](uint32_t w, double a) __attribute__((always_inline)) {
      lds_max_bits(mx + (w & 0xffff), a * El[w >> 16]);
    });
    __syncthreads();
    double dt[RUIZ_PER];
#pragma unroll
    for (int k = 0; k < RUIZ_PER; ++k) {
      const int j = tid + RUIZ_NT * k;
      dt[k] = 0.0;
      if (j < n) {
        const double dj = Dl[j];
        dt[k] = fmax(c * dj * dj * Pa[k], dj * __longlong_as_double((long long)mx[j]));
      }
    }
    __syncthreads();
    // ---- row maxima max_j |A_rj| D_j -> Et_r
    for (int r = tid; r < m; r += RUIZ_NT) mx[r] = 0ull;
    __syncthreads();
    ruiz_sweep(A, erc, nnz, [&](uint32_t w, double a) __attribute__((always_inline)) {
      lds_max_bits(mx + (w >> 16), a * Dl[w & 0xffff]);
    });
    __syncthreads();
#pragma unroll
    for (int k = 0; k < RUIZ_PER; ++k) {
      const int r = tid + RUIZ_NT * k;
      if (r < m) El[r] *= 1.0 / sqrt(limit_scaling(El[r] * __longlong_as_double((long long)mx[r])));
      const int j = tid + RUIZ_NT * k;
      if (j < n) Dl[j] = Dl[j] * (1.0 / sqrt(limit_scaling(dt[k])));
    }
    __syncthreads();
    // ---- cost normalisation (k_ruiz_update's order: 256 strided partial sums, then a tree)
    double sum = 0.0, qmax = 0.0;
    if (tid < 256) {
      for (int j = tid; j < n; j += 256) {
        const double dj = Dl[j];
        sum += c * dj * dj * fabs(P[j]);
        qmax = fmax(qmax, fabs(c * dj * q[j]));
      }
      red[tid] = sum;
    }
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (tid < s) red[tid] += red[tid + s];
      __syncthreads();
    }
    sum = red[0];
    __syncthreads();
    if (tid < 256) red[tid] = qmax;
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (tid < s) red[tid] = fmax(red[tid], red[tid + s]);
      __syncthreads();
    }
    if (tid == 0) {
      double ct = fmax(sum / (double)n, limit_scaling(red[0]));
      ct = limit_scaling(ct);
      c_sh = c * (1.0 / ct);
    }
    __syncthreads();
    c = c_sh;
  }
  double* D = d.D + (size_t)b * n;
  double* E = d.E + (size_t)b * m;
  for (int j = tid; j < n; j += RUIZ_NT) D[j] = Dl[j];
  for (int r = tid; r < m; r += RUIZ_NT) E[r] = El[r];
  if (tid == 0) d.cs[b] = c;
}

size_t ruiz_fused_lds(const PlOcpHandle* h) {
  return (size_t)(((h->n + 1) & ~1) + ((h->m + 1) & ~1) + std::max(h->n, h->m)) * 8;
}

bool ruiz_fused_supported(const PlOcpHandle* h) {
  return h->d.erc && h->n <= RUIZ_NT * RUIZ_PER && h->m <= RUIZ_NT * RUIZ_PER &&
         ruiz_fused_lds(h) <= 156 * 1024;
}

__global__ __launch_bounds__(256) void k_ruiz_update(PlDev d, int n, int m) {
  const int b = blockIdx.x;
  __shared__ double red[256];
  const double* P = d.P + (size_t)b * n;
  const double* q = d.grad + (size_t)b * n;
  double* D = d.D + (size_t)b * n;
  double* E = d.E + (size_t)b * m;
  const double* Dt = d.dxs + (size_t)b * n;
  const double* Dx = d.aty + (size_t)b * n;
  const double* Et = d.dys + (size_t)b * m;
  const double c = d.cs[b];
  double sum = 0.0, qmax = 0.0;
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    const double dt = fmax(Dt[j], D[j] * Dx[j]);  // + node i-1's entries on dx_i
    const double dj = D[j] * (1.0 / sqrt(limit_scaling(dt)));
    D[j] = dj;
    sum += c * dj * dj * fabs(P[j]);
    qmax = fmax(qmax, fabs(c * dj * q[j]));
  }
  for (int r = threadIdx.x; r < m; r += blockDim.x) E[r] *= 1.0 / sqrt(limit_scaling(Et[r]));
  // cost normalisation: c_temp = max(mean |P_jj|, ||q||_inf) on the scaled data
  sum = block_sum(sum, red);
  qmax = block_max(qmax, red);
  if (threadIdx.x == 0) {
    double ct = fmax(sum / (double)n, limit_scaling(qmax));
    ct = limit_scaling(ct);
    d.cs[b] = c * (1.0 / ct);
  }
}

// Scaled problem data of node i: As, qs, Ps (columns), ls, us, rho (rows), and
// rho of the coupling rows for the ADMM prefetch.
__global__ __launch_bounds__(256) void k_qp_finish(PlDev d, int N, int n, int m, int nnz, int ncpl_max, PlSettings st) {
  const int b = blockIdx.x / (N + 1), i = blockIdx.x - b * (N + 1);
  const PlNode nd = d.nodes[i];
  const double* A = d.Araw + (size_t)b * nnz;
  const double* P = d.P + (size_t)b * n;
  const double* q = d.grad + (size_t)b * n;
  const double* D = d.D + (size_t)b * n;
  const double* E = d.E + (size_t)b * m;
  const double c = d.cs[b];
  double* qs = d.qs + (size_t)b * n;
  double* Ps = d.Ps + (size_t)b * n;
  for (int lc = threadIdx.x; lc < nd.nw; lc += blockDim.x) {
    const int j = nd.x_off + lc;
    qs[j] = c * D[j] * q[j];
    Ps[j] = c * D[j] * D[j] * P[j];
  }
  if (i == N) return;
  const PlNode nn = d.nodes[i + 1];
  double* As = d.As + (size_t)b * nnz;
  for (int e = threadIdx.x; e < nd.nent; e += blockDim.x) {
    const int r = nd.row_off + d.rowidx[nd.ent_off + e];
    const int lc = d.entcol[nd.ent_off + e];
    const int j = lc < nd.nw ? nd.x_off + lc : nn.x_off + (lc - nd.nw);
    As[nd.ent_off + e] = E[r] * A[nd.ent_off + e] * D[j];
  }
  const double* g = d.g + (size_t)b * m;
  const double* lbg = d.lbg + (size_t)b * m;
  const double* ubg = d.ubg + (size_t)b * m;
  double* ls = d.ls + (size_t)b * m;
  double* us = d.us + (size_t)b * m;
  double* rho = d.rho + (size_t)b * m;
  __shared__ double rho_s[256];
  for (int lr = threadIdx.x; lr < nd.nrow; lr += blockDim.x) {
    const int r = nd.row_off + lr;
    double l = fmax(lbg[r] - g[r], -PL_OSQP_INFTY);
    double u = fmin(ubg[r] - g[r], PL_OSQP_INFTY);
    double lsr = E[r] * l, usr = E[r] * u;
    ls[r] = lsr;
    us[r] = usr;
    double rr;
    if (lsr < -PL_OSQP_INFTY * PL_MIN_SCALING && usr > PL_OSQP_INFTY * PL_MIN_SCALING) rr = PL_RHO_MIN;
    else if (usr - lsr < PL_RHO_TOL) rr = PL_RHO_EQ_OVER_INEQ * st.rho;
    else rr = st.rho;
    rho[r] = rr;
    if (lr < 256) rho_s[lr] = rr;
  }
  __syncthreads();
  // rho of the node's coupling rows, contiguous for the ADMM prefetch
  double* rhoc = d.rhoc + (size_t)b * (N + 1) * ncpl_max + (size_t)i * ncpl_max;
  for (int s = threadIdx.x; s < nd.ncpl; s += blockDim.x) {
    const int lr = d.cplrow[nd.cpl_off + s];
    rhoc[s] = lr < 256 ? rho_s[lr] : rho[nd.row_off + lr];
  }
}

void launch_qp_setup(PlOcpHandle* h) {
  const dim3 nodes_grid(h->B * (h->N + 1));
  if (h->ruiz_fused && ruiz_fused_supported(h)) {
    static bool fattr = false;
    if (!fattr) {
      hipFuncSetAttribute((const void*)k_ruiz_fused, hipFuncAttributeMaxDynamicSharedMemorySize, 156 * 1024);  // + static
      fattr = true;
    }
    hipLaunchKernelGGL(k_ruiz_fused, dim3(h->B), dim3(RUIZ_NT), ruiz_fused_lds(h), h->stream, h->d, h->n, h->m, h->nnz,
                       h->set.scaling);
    hipLaunchKernelGGL(k_qp_finish, nodes_grid, dim3(256), 0, h->stream, h->d, h->N, h->n, h->m, h->nnz,
                       std::max(h->ncpl_max, 1), h->set);
    return;
  }
  hipLaunchKernelGGL(k_ruiz_init, dim3(h->B), dim3(256), 0, h->stream, h->d, h->n, h->m);
  const int nent_max = (std::max(h->nent_max, 1) + 1) & ~1, ncol_max = (std::max(h->ncol_max, h->nw_max) + 1) & ~1;
  const int nrow_max = (std::max(h->nrow_max, 1) + 1) & ~1, chunk_max = (std::max(h->chunk_max, 1) + 1) & ~1;
  const size_t lds = (size_t)(nent_max + ncol_max + nrow_max + chunk_max) * 8;
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)k_ruiz_norms, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  for (int pass = 0; pass < h->set.scaling; ++pass) {
    hipLaunchKernelGGL(k_ruiz_norms, nodes_grid, dim3(256), lds, h->stream, h->d, h->N, h->n, h->m, h->nnz,
                       h->ndx, nent_max, ncol_max, nrow_max, chunk_max);
    hipLaunchKernelGGL(k_ruiz_update, dim3(h->B), dim3(256), 0, h->stream, h->d, h->n, h->m);
  }
  hipLaunchKernelGGL(k_qp_finish, nodes_grid, dim3(256), 0, h->stream, h->d, h->N, h->n, h->m, h->nnz,
                     std::max(h->ncpl_max, 1), h->set);
}

// rhs = sigma x - q + A^T (rho z - y)   (before the first iteration of a solve)
// zero (the interior point's refinement sweeps): z = y = 0, so A^T (rho z - y) adds nothing
// and the gathers are skipped (rhs = sigma x - q, the same value up to the sign of a zero)
__global__ __launch_bounds__(256) void k_admm_init(PlDev d, int N, int n, int m, int nnz, double sigma, int zero) {
  const int b = blockIdx.x;
  if (d.info[b].done) return;
  const double* As = d.As + (size_t)b * nnz;
  const double* za = d.za + (size_t)b * m;
  const double* ya = d.ya + (size_t)b * m;
  const double* rho = d.rho + (size_t)b * m;
  const double* xa = d.xa + (size_t)b * n;
  const double* qs = d.qs + (size_t)b * n;
  double* rhs = d.rhs + (size_t)b * n;
  // gathers in chunks of CK entries (index words, then the operands, then the FMAs in
  // entry order: the same arithmetic as one entry at a time, see k_check_part)
  constexpr int CK = 8;
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    double acc = sigma * xa[j] - qs[j];
    if (zero) {
      rhs[j] = acc;
      continue;
    }
    const int q0 = d.gc_ptr[j], q1 = d.gc_ptr[j + 1];
    for (int q = q0; q < q1; q += CK) {
      int2 er[CK];
      double av[CK], rv[CK], zv[CK], yv[CK];
#pragma unroll
      for (int k = 0; k < CK; ++k) er[k] = d.gc_er[min(q + k, q1 - 1)];
#pragma unroll
      for (int k = 0; k < CK; ++k) {
        av[k] = As[er[k].x];
        rv[k] = rho[er[k].y];
        zv[k] = za[er[k].y];
        yv[k] = ya[er[k].y];
      }
#pragma unroll
      for (int k = 0; k < CK; ++k)
        if (q + k < q1) acc += av[k] * (rv[k] * zv[k] - yv[k]);
    }
    rhs[j] = acc;
  }
}

void launch_admm_init(PlOcpHandle* h) {
  hipLaunchKernelGGL(k_admm_init, dim3(h->B), dim3(256), 0, h->stream, h->d, h->N, h->n, h->m, h->nnz,
                     h->set.sigma, 0);
}
// (k_ip.hip) the refinement sweeps: x = z = y = 0
void launch_admm_init_zero(PlOcpHandle* h) {
  hipLaunchKernelGGL(k_admm_init, dim3(h->B), dim3(256), 0, h->stream, h->d, h->N, h->n, h->m, h->nnz,
                     h->set.sigma, 1);
}

// ---------------------------------------------------------------------------
// Termination (OSQP 0.6 update_info + check_termination, incl. infeasibility
// certificates and the x10 "approximate" check at max_iter).
// Residual norms per (problem, node), one 64-lane block each, partial maxima to d.chk:
//   chk[b][i][0..2] = max |E^-1 (A x - z)|, |E^-1 z|, |E^-1 A x|   over node i's rows
//   chk[b][i][3..6] = max |D^-1 (P x + q + A^T y)|, |D^-1 q|, |D^-1 A^T y|, |D^-1 P x|
//                     over node i's columns w_i
// A x and A^T y stream the node's entries in storage order (coalesced 8-byte loads of As
// and of the packed local coordinates d.erl) into LDS accumulators with ds_add_f64: x of
// w_i and dx_{i+1} is staged in LDS, y is read from its row.  Entries are node-major and
// column-major inside a node, and one wave adds the lanes of an instruction and its
// instructions in a fixed order, so every row sums its entries in column order and every
// column its own node's rows first, then node i-1's coupling rows on dx_i: a fixed order per
// problem (bit-identical in any batch).  The previous row / column gathers over the global
// CSR / CSC were latency chains: 0.68 ms per check at B2G rnea N=50, B = 1024.
__device__ __forceinline__ void chk_lds_add(double* p, double v) {
  typedef __attribute__((address_space(3))) double* LPtr;
  __hip_atomic_fetch_add((LPtr)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
}

__global__ __launch_bounds__(64) void k_check_part(PlDev d, int N, int n, int m, int nnz, int ndx) {
  extern __shared__ double lds[];
  const int b = blockIdx.x / (N + 1), i = blockIdx.x - b * (N + 1);
  if (d.info[b].done) return;
  const PlNode nd = d.nodes[i];
  const int tid = threadIdx.x;
  const int nrow = nd.nrow, nw = nd.nw, ncol = nd.ncol;
  const int nx = max(ncol, nw);
  const double* __restrict__ As = d.As + (size_t)b * nnz;
  const double* __restrict__ xa = d.xa + (size_t)b * n;
  const double* __restrict__ ya = d.ya + (size_t)b * m;
  const uint32_t* __restrict__ erl = d.erl;
  double* xl = lds;                      // x of w_i, dx_{i+1}
  double* ax = xl + ((nx + 1) & ~1);     // A x over the node's rows
  double* aty = ax + ((nrow + 1) & ~1);  // A^T y over w_i
  for (int c = tid; c < nx; c += 64) xl[c] = xa[nd.x_off + c];
  for (int r = tid; r < nrow; r += 64) ax[r] = 0.0;
  for (int c = tid; c < nw; c += 64) aty[c] = 0.0;
  __syncthreads();
  {
    const double* __restrict__ Ai = As + nd.ent_off;
    const uint32_t* __restrict__ Li = erl + nd.ent_off;
    const double* __restrict__ yi = ya + nd.row_off;
    for (int e = tid; e < nd.nent; e += 64) {
      const uint32_t w = Li[e];
      const int r = (int)(w >> 16), c = (int)(w & 0xffff);
      const double a = Ai[e];
      const double yr = yi[r];
      chk_lds_add(ax + r, a * xl[c]);
      if (c < nw) chk_lds_add(aty + c, a * yr);
    }
  }
  if (i > 0) {  // node i-1's coupling rows on dx_i: the tail of its column-major entries
    const PlNode pn = d.nodes[i - 1];
    const int e0 = d.colptr[pn.colptr_off + pn.nw];
    const double* __restrict__ Ap = As + pn.ent_off;
    const uint32_t* __restrict__ Lp = erl + pn.ent_off;
    const double* __restrict__ yp = ya + pn.row_off;
    for (int e = e0 + tid; e < pn.nent; e += 64) {
      const uint32_t w = Lp[e];
      chk_lds_add(aty + ((int)(w & 0xffff) - pn.nw), Ap[e] * yp[w >> 16]);
    }
  }
  __syncthreads();
  double v[7] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  {
    const double* za = d.za + (size_t)b * m + nd.row_off;
    const double* E = d.E + (size_t)b * m + nd.row_off;
    for (int r = tid; r < nrow; r += 64) {
      const double ei = 1.0 / E[r], zr = za[r], axr = ax[r];
      v[0] = fmax(v[0], fabs(ei * (axr - zr)));
      v[1] = fmax(v[1], fabs(ei * zr));
      v[2] = fmax(v[2], fabs(ei * axr));
    }
  }
  {
    const double* qs = d.qs + (size_t)b * n + nd.x_off;
    const double* Ps = d.Ps + (size_t)b * n + nd.x_off;
    const double* D = d.D + (size_t)b * n + nd.x_off;
    for (int lc = tid; lc < nw; lc += 64) {
      const double di = 1.0 / D[lc], qc = qs[lc];
      const double px = Ps[lc] * xl[lc];
      const double atyc = aty[lc];
      v[3] = fmax(v[3], fabs(di * (px + qc + atyc)));
      v[4] = fmax(v[4], fabs(di * qc));
      v[5] = fmax(v[5], fabs(di * atyc));
      v[6] = fmax(v[6], fabs(di * px));
    }
  }
  // one wave: butterfly maxima across the 64 lanes (max is order-free, so exact)
#pragma unroll
  for (int s = 32; s > 0; s >>= 1)
#pragma unroll
    for (int k = 0; k < 7; ++k) v[k] = fmax(v[k], __shfl_xor(v[k], s, 64));
  double* out = d.chk + ((size_t)b * (N + 1) + i) * 8;
#pragma unroll
  for (int k = 0; k < 7; ++k)
    if (tid == k) out[k] = v[k];
}

// Termination (OSQP 0.6 update_info + check_termination, incl. infeasibility
// certificates and the x10 "approximate" check at max_iter), from the node partials.
constexpr int CHECK_NT = 256;
__global__ __launch_bounds__(CHECK_NT) void k_check(PlDev d, int N, int n, int m, int nnz, PlSettings st,
                                                     int final_check) {
  const int b = blockIdx.x;
  PlProbInfo* info = d.info + b;
  if (info->done) return;
  __shared__ double red[7 * CHECK_NT];
  const double* As = d.As + (size_t)b * nnz;
  const double* xa = d.xa + (size_t)b * n;
  const double* qs = d.qs + (size_t)b * n;
  const double* Ps = d.Ps + (size_t)b * n;
  const double* D = d.D + (size_t)b * n;
  const double* E = d.E + (size_t)b * m;
  const double* ls = d.ls + (size_t)b * m;
  const double* us = d.us + (size_t)b * m;
  const double* dxs = d.dxs + (size_t)b * n;
  const double* dys = d.dys + (size_t)b * m;
  const int* __restrict__ gr_ptr = d.gr_ptr;
  const int2* __restrict__ gr_ec = d.gr_ec;
  const int* __restrict__ gc_ptr = d.gc_ptr;
  const int2* __restrict__ gc_er = d.gc_er;
  const double c = d.cs[b], cinv = 1.0 / c;
  double pv[7] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
  for (int i = threadIdx.x; i <= N; i += blockDim.x) {
    const double* ck = d.chk + ((size_t)b * (N + 1) + i) * 8;
#pragma unroll
    for (int k = 0; k < 7; ++k) pv[k] = fmax(pv[k], ck[k]);
  }
  block_max_k<7, CHECK_NT>(pv, red);
  const double pri = pv[0], nz = pv[1], nax = pv[2];
  const double dua = cinv * pv[3], nq = pv[4], naty = pv[5], npx = pv[6];
  __shared__ int s_status;
  for (int pass = 0; pass < (final_check ? 2 : 1); ++pass) {
    const bool approx = (pass == 1);
    const double mul = approx ? 10.0 : 1.0;
    const double eps_abs = st.eps_abs * mul, eps_rel = st.eps_rel * mul;
    const double eps_pinf = st.eps_prim_inf * mul, eps_dinf = st.eps_dual_inf * mul;
    int status = PL_ST_UNSOLVED;
    if (pri > PL_OSQP_INFTY || dua > PL_OSQP_INFTY) {
      status = PL_ST_NON_CVX;
    } else {
      const double eps_pri = eps_abs + eps_rel * fmax(nz, nax);
      const double eps_dua = eps_abs + eps_rel * cinv * fmax(nq, fmax(naty, npx));
      const bool prim_ok = pri < eps_pri;
      const bool dual_ok = dua < eps_dua;
      bool prim_inf = false, dual_inf = false;
      if (!prim_ok) {
        // project delta_y onto the polar of the recession cone, ||E dy||
        double ndy = 0.0, ineq = 0.0;
        for (int r = threadIdx.x; r < m; r += blockDim.x) {
          double dy = dys[r];
          const bool uinf = us[r] > PL_OSQP_INFTY * PL_MIN_SCALING, linf = ls[r] < -PL_OSQP_INFTY * PL_MIN_SCALING;
          if (uinf && linf) dy = 0.0;
          else if (uinf) dy = fmin(dy, 0.0);
          else if (linf) dy = fmax(dy, 0.0);
          ndy = fmax(ndy, fabs(E[r] * dy));
          ineq += us[r] * fmax(dy, 0.0) + ls[r] * fmin(dy, 0.0);
        }
        ndy = block_max(ndy, red);
        ineq = block_sum(ineq, red);
        if (ndy > PL_DIV_TOL && ineq < eps_pinf * ndy) {
          double natdy = 0.0;
          for (int j = threadIdx.x; j < n; j += blockDim.x) {
            double s = 0.0;
            for (int q = gc_ptr[j]; q < gc_ptr[j + 1]; ++q) {
              const int e = gc_er[q].x, r = gc_er[q].y;
              double dy = dys[r];
              const bool uinf = us[r] > PL_OSQP_INFTY * PL_MIN_SCALING, linf = ls[r] < -PL_OSQP_INFTY * PL_MIN_SCALING;
              if (uinf && linf) dy = 0.0;
              else if (uinf) dy = fmin(dy, 0.0);
              else if (linf) dy = fmax(dy, 0.0);
              s += As[e] * dy;
            }
            natdy = fmax(natdy, fabs(s / D[j]));
          }
          natdy = block_max(natdy, red);
          prim_inf = natdy < eps_pinf * ndy;
        }
      }
      if (!dual_ok) {
        double ndx_ = 0.0, qdx = 0.0, npdx = 0.0;
        for (int j = threadIdx.x; j < n; j += blockDim.x) {
          ndx_ = fmax(ndx_, fabs(D[j] * dxs[j]));
          qdx += qs[j] * dxs[j];
          npdx = fmax(npdx, fabs(Ps[j] * dxs[j] / D[j]));
        }
        ndx_ = block_max(ndx_, red);
        qdx = block_sum(qdx, red);
        npdx = block_max(npdx, red);
        if (ndx_ > PL_DIV_TOL && qdx < c * eps_dinf * ndx_ && npdx < c * eps_dinf * ndx_) {
          int bad = 0;
          for (int r = threadIdx.x; r < m; r += blockDim.x) {
            double adx = 0.0;
            for (int q = gr_ptr[r]; q < gr_ptr[r + 1]; ++q) adx += As[gr_ec[q].x] * dxs[gr_ec[q].y];
            adx /= E[r];
            if ((us[r] < PL_OSQP_INFTY * PL_MIN_SCALING && adx > eps_dinf * ndx_) ||
                (ls[r] > -PL_OSQP_INFTY * PL_MIN_SCALING && adx < -eps_dinf * ndx_))
              bad = 1;
          }
          dual_inf = block_max((double)bad, red) == 0.0;
        }
      }
      if (prim_ok && dual_ok) status = approx ? PL_ST_SOLVED_INACCURATE : PL_ST_SOLVED;
      else if (prim_inf) status = approx ? PL_ST_PRIMAL_INF_INACC : PL_ST_PRIMAL_INF;
      else if (dual_inf) status = approx ? PL_ST_DUAL_INF_INACC : PL_ST_DUAL_INF;
    }
    if (threadIdx.x == 0) {
      info->pri_res = pri;
      info->dua_res = dua;
      if (status != PL_ST_UNSOLVED) {
        info->status = status;
        info->done = 1;
      } else if (approx) {
        info->status = PL_ST_MAX_ITER;
        info->done = 1;
      }
      s_status = info->done;
    }
    __syncthreads();
    if (s_status) break;
  }
}

void launch_check(PlOcpHandle* h, int it, int final_check) {
  (void)it;
  {
    const int lds = ((std::max(h->ncol_max, h->nw_max) + 1) & ~1) + ((h->nrow_max + 1) & ~1) + ((h->nw_max + 1) & ~1);
    hipLaunchKernelGGL(k_check_part, dim3(h->B * (h->N + 1)), dim3(64), lds * 8, h->stream, h->d, h->N, h->n, h->m,
                       h->nnz, h->ndx);
  }
  hipLaunchKernelGGL(k_check, dim3(h->B), dim3(CHECK_NT), 0, h->stream, h->d, h->N, h->n, h->m, h->nnz, h->set,
                     final_check);
}

// Unscaled solution dx = D x (store_solution); NaN + cold start on infeasibility.
__global__ __launch_bounds__(256) void k_unscale(PlDev d, int n, int m) {
  const int b = blockIdx.x;
  const PlProbInfo info = d.info[b];
  const bool bad = info.status == PL_ST_PRIMAL_INF || info.status == PL_ST_PRIMAL_INF_INACC ||
                   info.status == PL_ST_DUAL_INF || info.status == PL_ST_DUAL_INF_INACC || info.status == PL_ST_NON_CVX;
  double* step = d.step + (size_t)b * n;
  double* xa = d.xa + (size_t)b * n;
  const double* D = d.D + (size_t)b * n;
  for (int j = threadIdx.x; j < n; j += blockDim.x) {
    step[j] = bad ? __builtin_nan("") : D[j] * xa[j];
    if (bad) xa[j] = 0.0;
  }
  if (bad) {
    for (int r = threadIdx.x; r < m; r += blockDim.x) {
      d.za[(size_t)b * m + r] = 0.0;
      d.ya[(size_t)b * m + r] = 0.0;
    }
  }
}

void launch_unscale(PlOcpHandle* h) {
  hipLaunchKernelGGL(k_unscale, dim3(h->B), dim3(256), 0, h->stream, h->d, h->n, h->m);
}

__global__ void k_reset_info(PlDev d, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  PlProbInfo& I = d.info[b];
  I.status = PL_ST_UNSOLVED;
  I.iter = 0;
  I.done = 0;
}

__global__ void k_reset_prof(PlDev d, int B) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b < B) d.info[b].iter_prof = 0;
}

void launch_reset_prof(PlOcpHandle* h) {
  hipLaunchKernelGGL(k_reset_prof, dim3((h->B + 63) / 64), dim3(64), 0, h->stream, h->d, h->B);
}

void launch_reset_info(PlOcpHandle* h) {
  hipLaunchKernelGGL(k_reset_info, dim3((h->B + 63) / 64), dim3(64), 0, h->stream, h->d, h->B);
}

// Cold start of the ADMM iterates (OSQP setup state: x = z = y = 0).
__global__ void k_zero(double* p, size_t len) {
  for (size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x; t < len; t += (size_t)gridDim.x * blockDim.x) p[t] = 0.0;
}

void launch_reset_iterates(PlOcpHandle* h) {
  hipLaunchKernelGGL(k_zero, dim3(1024), dim3(256), 0, h->stream, h->d.xa, (size_t)h->B * h->n);
  hipLaunchKernelGGL(k_zero, dim3(1024), dim3(256), 0, h->stream, h->d.za, (size_t)h->B * h->m);
  hipLaunchKernelGGL(k_zero, dim3(1024), dim3(256), 0, h->stream, h->d.ya, (size_t)h->B * h->m);
}
