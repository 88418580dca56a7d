// Block factorisation of the reduced KKT system (the numeric refactorisation
// osqp.update(Ax=...) triggers, optimization/ocp.py:391-395; OSQP factors the
// quasi-definite KKT with QDLDL, here its reduced SPD form is factored).
//
//   K = P + sigma I + A^T diag(rho) A   is block tridiagonal over w_i = [dx_i, u_i].
//   For i = 0..N:
//     Kt_ii = diag(P + sigma) + sum_{rows r of node i} rho_r a_r a_r^T |_{w_i}
//             + E_i  on the dx_i block,   E_i = D_i - Kc_{i-1} S_{i-1} Kc_{i-1}^T
//     S_i   = Kt_ii^{-1}                        (Gauss-Jordan, symmetrised)
//     Kc_i  = K_{i+1,i} = sum_{coupling rows s} rho_s x_s w_s^T   (ndx x nw)
//     D_{i+1} = sum_{coupling rows s} rho_s x_s x_s^T            (ndx x ndx)
//   where a coupling row s of node i has its dx_{i+1} part x_s and w_i part w_s.
// S_i is stored in the tiled layout the ADMM sweeps stream (k_admm.hip).
//
// One 256-thread workgroup per problem.  Everything a node needs is staged in
// LDS first (its scaled A values, rho, and the CSR row program), so no phase
// walks a dependent chain of HBM loads; Kc, the packed lower S and U = Kc S stay
// in LDS, and the dense products are register-blocked (7x7 for the assembly and
// Gauss-Jordan, 3x7 for U, 3x3 for the Schur complement).
#include <algorithm>

#include "state.h"

namespace {

constexpr int NT = 256;
constexpr int FB = 7;    // Gauss-Jordan / assembly register block (16 x 16 blocks of 7 -> 112)
constexpr int FG = 16;
constexpr int FCH = 16;  // rows per assembly chunk
constexpr int GJ_LDS = 2 * 49 + 2 * 16 * 49 + 2 * 16 * 49;  // block Gauss-Jordan buffers (doubles)

struct FactorMap {
  int sl;        // packed lower S / chunk buffer / U / Gauss-Jordan panels (doubles)
  int ent, row;  // A values and rho of one node
  int flen;      // u16 row program
  __host__ __device__ size_t total(int ndx, int nw_max) const {
    // + 17 words of optional phase timing at the end (8-byte aligned)
    return ((size_t)sl + (size_t)ndx * ndx + (size_t)ndx * nw_max + ent + row + FCH + 17) * sizeof(double) +
           ((2 * (size_t)flen + 7) & ~(size_t)7);
  }
};

__device__ __forceinline__ int lidx(int r, int c) {  // packed lower, r >= c
  return r * (r + 1) / 2 + c;
}
__device__ __forceinline__ double sym_at(const double* Sl, int r, int c) {
  return r >= c ? Sl[lidx(r, c)] : Sl[lidx(c, r)];
}

}  // namespace

template <bool TIMING>
__global__ __launch_bounds__(256) void k_factor(PlDev d, int N, int n, int m, int nnz, int ndx, int S_stride, int nw_max,
                                                FactorMap fm, double sigma) {
  // optional phase timing (s_memtime, thread 0) into d.dbg[b][16 + k]
  extern __shared__ double lds[];
  unsigned long long* tacc = reinterpret_cast<unsigned long long*>(lds) + (fm.total(ndx, nw_max) / 8 - 17);
  if constexpr (TIMING) {
    if (threadIdx.x < 17) tacc[threadIdx.x] = 0;
  }
  auto T = [&](int slot) {
    if constexpr (TIMING) {
      if (threadIdx.x == 0) {
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        if (slot >= 0) tacc[slot] += now - tacc[16];
        tacc[16] = now;
      }
    }
  };
  typedef const __attribute__((address_space(4))) PlAdmmNode* CNode;
  CNode an = (CNode)d.anodes;
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int ty = tid / FG, tx = tid % FG;
  double* Sl = lds;                  // packed lower S_i | chunk buffer | U (ndx x nw)
  double* Cb = Sl + fm.sl;           // E_i (ndx x ndx), then D_{i+1}, then E_{i+1}
  double* Kc = Cb + ndx * ndx;       // ndx x nw
  double* asb = Kc + ndx * nw_max;   // node's A values
  double* rwb = asb + fm.ent;        // node's rho
  double* rw = rwb + fm.row;         // FCH
  uint16_t* pg = reinterpret_cast<uint16_t*>(rw + FCH);

  const double* __restrict__ As = d.As + (size_t)b * nnz;
  const double* __restrict__ rho = d.rho + (size_t)b * m;
  const double* __restrict__ Ps = d.Ps + (size_t)b * n;
  double* Sg = d.S + (size_t)b * S_stride;

  for (int k = tid; k < ndx * ndx; k += NT) Cb[k] = 0.0;

  for (int i = 0; i <= N; ++i) {
    const int nw = an[i].nw, nrow = an[i].nrow, ncpl = an[i].ncpl, nent = an[i].nent, ncol = an[i].ncol;
    const int ent_off = an[i].ent_off, row_off = an[i].row_off, x_off = an[i].x_off;
    const int prog = an[i].fprog, flen = an[i].flen, p_rowptr = an[i].f_rowptr, p_cplr = an[i].f_cplr,
              p_rowp = an[i].f_rowp;
    const int ntile = an[i].ntile, nunit = an[i].nunit, ntl = an[i].ntl, s_off = an[i].s_off;
    __syncthreads();
    T(-1);
    // ---- stage the node's A values, rho and row program
    for (int k = tid; k < nent; k += NT) asb[k] = As[ent_off + k];
    for (int k = tid; k < nrow; k += NT) rwb[k] = rho[row_off + k];
    {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(d.fprog + prog);
      uint32_t* dst = reinterpret_cast<uint32_t*>(pg);
      for (int k = tid; k < (flen >> 1); k += NT) dst[k] = src[k];
    }
    const uint32_t* rowp = reinterpret_cast<const uint32_t*>(pg + p_rowp);
    // dense chunk buf[s][c - c0] (c in [c0, c0 + W)) of rows rows(s), rho in rw[s]
    auto fill = [&](int s0, int nr, bool cpl_rows, int c0, int W) {
      __syncthreads();
      for (int t = tid; t < FCH * W; t += NT) Sl[t] = 0.0;
      __syncthreads();
      for (int s = tid / 16; s < nr; s += NT / 16) {
        const int lr = cpl_rows ? pg[p_cplr + s0 + s] : s0 + s;
        const int q0 = pg[p_rowptr + lr], q1 = pg[p_rowptr + lr + 1];
        for (int q = q0 + (tid & 15); q < q1; q += 16) {
          const uint32_t w = rowp[q];
          const int c = (int)(w >> 16) - c0;
          if (c >= 0 && c < W) Sl[s * W + c] = asb[w & 0xffff];
        }
        if ((tid & 15) == 0) rw[s] = rwb[lr];
      }
      __syncthreads();
    };

    T(0);
    __syncthreads();
    T(1);
    // ---- Kt_ii: diagonal (identity on the padding), E_i on the dx block
    double Kr[FB][FB];
#pragma unroll
    for (int rr = 0; rr < FB; ++rr)
#pragma unroll
      for (int cc = 0; cc < FB; ++cc) {
        const int gi = FB * ty + rr, gj = FB * tx + cc;
        double v = 0.0;
        if (gi == gj) v = (gi < nw) ? Ps[x_off + gi] + sigma : 1.0;
        if (gi < ndx && gj < ndx) v += Cb[gi * ndx + gj];
        Kr[rr][cc] = v;
      }
    __syncthreads();  // E_i consumed: the buffer now carries D_{i+1}
    // coupling lists (state.h): rho_s A of the coupling rows of node i
    const uint32_t* f_cw = reinterpret_cast<const uint32_t*>(pg + an[i].f_cwp);
    const uint32_t* f_xc = reinterpret_cast<const uint32_t*>(pg + an[i].f_xcp);
    const uint32_t* f_cx = reinterpret_cast<const uint32_t*>(pg + an[i].f_cxp);
    const int p_cwptr = an[i].f_cwptr, p_xcptr = an[i].f_xcptr, p_cxptr = an[i].f_cxptr;
    if (i < N) {
      // D_{i+1}[a][b] = sum_s rho_s x_{s,a} x_{s,b} over the coupling rows s with an entry in column a
      for (int k = tid; k < ndx * ndx; k += NT) {
        const int ra = k / ndx, cb = k - ra * ndx;
        double acc = 0.0;
        for (int q = pg[p_xcptr + ra]; q < pg[p_xcptr + ra + 1]; ++q) {
          const uint32_t w = f_xc[q];
          const int sidx = (int)(w >> 16);
          for (int q2 = pg[p_cxptr + sidx]; q2 < pg[p_cxptr + sidx + 1]; ++q2) {
            const uint32_t w2 = f_cx[q2];
            if ((int)(w2 >> 16) == cb) acc += rwb[pg[p_cplr + sidx]] * asb[w & 0xffff] * asb[w2 & 0xffff];
          }
        }
        Cb[k] = acc;
      }
    }
    T(2);
    // ---- rows of node i on the w_i columns
    for (int r0 = 0; r0 < nrow; r0 += FCH) {
      const int nr = min(FCH, nrow - r0);
      fill(r0, nr, false, 0, nw);
      // rows past nr are zero in the chunk buffer, so pairs of rows need no tail
      for (int s = 0; s < nr; s += 2) {
        const double* a0 = Sl + s * nw;
        const double* a1 = a0 + nw;
        const double w0 = rw[s], w1 = (s + 1 < nr) ? rw[s + 1] : 0.0;
        double ar0[FB], ac0[FB], ar1[FB], ac1[FB];
#pragma unroll
        for (int k = 0; k < FB; ++k) {
          const int gi = FB * ty + k, gj = FB * tx + k;
          ar0[k] = gi < nw ? w0 * a0[gi] : 0.0;
          ac0[k] = gj < nw ? a0[gj] : 0.0;
          ar1[k] = gi < nw ? w1 * a1[gi] : 0.0;
          ac1[k] = gj < nw ? a1[gj] : 0.0;
        }
#pragma unroll
        for (int rr = 0; rr < FB; ++rr)
#pragma unroll
          for (int cc = 0; cc < FB; ++cc) Kr[rr][cc] += ar0[rr] * ac0[cc] + ar1[rr] * ac1[cc];
      }
    }
    T(3);
    __syncthreads();  // chunk buffer consumed: the Gauss-Jordan panels reuse it
    // ---- in-place block Gauss-Jordan inversion over the 7x7 register blocks
    // (SPD, no pivoting).  Pivot block K, B = A_KK:
    //   A_KK <- B^-1,  A_Kj <- B^-1 A_Kj,  A_iK <- -A_iK B^-1,  A_ij <- A_ij - A_iK B^-1 A_Kj.
    // Two barriers per block; the panels live in the (free) Sl region.
    {
      const int nb = (nw + FB - 1) / FB;
      double* Bi = Sl;                  // [2][49]  B^-1
      double* CP = Bi + 2 * 49;         // [2][16][49] old column panel A_iK
      double* RP = CP + 2 * 16 * 49;    // [16][49] old row panel A_Kj (read by its owner only)
      double* NRP = RP + 16 * 49;       // [16][49] new row panel B^-1 A_Kj
      for (int K = 0; K < nb; ++K) {
        double* bi = Bi + (K & 1) * 49;
        double* cp = CP + (K & 1) * 16 * 49;
        if (ty == K && tx == K) {  // invert the pivot block in registers (scalar GJ, 7x7)
          double Bm[FB][FB];
#pragma unroll
          for (int r = 0; r < FB; ++r)
#pragma unroll
            for (int c = 0; c < FB; ++c) Bm[r][c] = Kr[r][c];
#pragma unroll
          for (int k = 0; k < FB; ++k) {
            const double pinv = 1.0 / Bm[k][k];
#pragma unroll
            for (int r = 0; r < FB; ++r)
#pragma unroll
              for (int c = 0; c < FB; ++c) {
                if (r == k || c == k) continue;
                Bm[r][c] -= Bm[r][k] * (Bm[k][c] * pinv);
              }
#pragma unroll
            for (int c = 0; c < FB; ++c)
              if (c != k) Bm[k][c] *= pinv;
#pragma unroll
            for (int r = 0; r < FB; ++r)
              if (r != k) Bm[r][k] *= -pinv;
            Bm[k][k] = pinv;
          }
#pragma unroll
          for (int r = 0; r < FB; ++r)
#pragma unroll
            for (int c = 0; c < FB; ++c) bi[r * FB + c] = Bm[r][c];
        } else if (ty == K) {  // old row panel (owner only)
#pragma unroll
          for (int r = 0; r < FB; ++r)
#pragma unroll
            for (int c = 0; c < FB; ++c) RP[tx * 49 + r * FB + c] = Kr[r][c];
        } else if (tx == K) {  // old column panel (read by every row block)
#pragma unroll
          for (int r = 0; r < FB; ++r)
#pragma unroll
            for (int c = 0; c < FB; ++c) cp[ty * 49 + r * FB + c] = Kr[r][c];
        }
        __syncthreads();
        if (ty == K && tx != K) {  // A_Kj <- B^-1 A_Kj
#pragma unroll
          for (int r = 0; r < FB; ++r) {
            double br[FB];
#pragma unroll
            for (int k = 0; k < FB; ++k) br[k] = bi[r * FB + k];
#pragma unroll
            for (int c = 0; c < FB; ++c) {
              double acc = 0.0;
#pragma unroll
              for (int k = 0; k < FB; ++k) acc += br[k] * RP[tx * 49 + k * FB + c];
              Kr[r][c] = acc;
              NRP[tx * 49 + r * FB + c] = acc;
            }
          }
        }
        __syncthreads();
        if (ty == K && tx == K) {
#pragma unroll
          for (int r = 0; r < FB; ++r)
#pragma unroll
            for (int c = 0; c < FB; ++c) Kr[r][c] = bi[r * FB + c];
        } else if (tx == K) {  // A_iK <- -A_iK B^-1
#pragma unroll
          for (int r = 0; r < FB; ++r) {
            double ar[FB];
#pragma unroll
            for (int k = 0; k < FB; ++k) ar[k] = Kr[r][k];
#pragma unroll
            for (int c = 0; c < FB; ++c) {
              double acc = 0.0;
#pragma unroll
              for (int k = 0; k < FB; ++k) acc += ar[k] * bi[k * FB + c];
              Kr[r][c] = -acc;
            }
          }
        } else if (ty != K) {  // A_ij <- A_ij - A_iK (B^-1 A_Kj)
#pragma unroll
          for (int k = 0; k < FB; ++k) {
            double cv[FB], rv[FB];
#pragma unroll
            for (int q = 0; q < FB; ++q) {
              cv[q] = cp[ty * 49 + q * FB + k];
              rv[q] = NRP[tx * 49 + k * FB + q];
            }
#pragma unroll
            for (int rr = 0; rr < FB; ++rr)
#pragma unroll
              for (int cc = 0; cc < FB; ++cc) Kr[rr][cc] -= cv[rr] * rv[cc];
          }
        }
      }
    }
    __syncthreads();
    T(4);
    // ---- symmetrise into the packed lower Sl: GJ without pivoting leaves S_i
    // slightly non-symmetric (~eps cond); the sweeps and the next Schur
    // complement must see the same matrix, and (S + S^T) / 2 is the more accurate.
#pragma unroll
    for (int rr = 0; rr < FB; ++rr)
#pragma unroll
      for (int cc = 0; cc < FB; ++cc) {
        const int gi = FB * ty + rr, gj = FB * tx + cc;
        if (gi < nw && gj <= gi) Sl[lidx(gi, gj)] = Kr[rr][cc];
      }
    __syncthreads();
#pragma unroll
    for (int rr = 0; rr < FB; ++rr)
#pragma unroll
      for (int cc = 0; cc < FB; ++cc) {
        const int gi = FB * ty + rr, gj = FB * tx + cc;
        if (gj < nw && gi < gj) {
          double* p = Sl + lidx(gj, gi);
          *p = 0.5 * (*p + Kr[rr][cc]);
        }
      }
    __syncthreads();
    T(5);
    // ---- store S_i in the ADMM lane-tile layout (state.h): 4x4 tile t = K l + k of
    // lane l, pair j at s_off + ((k * 8 + j) * 64 + l) * 2 (coalesced over o)
    {
      double* Sn = Sg + s_off;
      const int total = nunit * 64 * 16;
      for (int o = tid; o < total; o += NT) {
        const int slot = o & 1, l = (o >> 1) & 63, j = (o >> 7) & 7, k = o >> 10;
        const int t = nunit * l + k;
        double val = 0.0;
        if (t < ntl) {
          int I = (int)((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
          while (I * (I + 1) / 2 > t) --I;
          while ((I + 1) * (I + 2) / 2 <= t) ++I;
          const int J = t - I * (I + 1) / 2;
          const int gi = 4 * I + (j >> 1), gj = 4 * J + 2 * (j & 1) + slot;
          if (gi < nw && gj < nw) val = sym_at(Sl, gi, gj);
        }
        Sn[o] = val;
      }
    }
    (void)ntile;
    T(6);
    if (i == N) break;
    // ---- U = Kc S (ndx x nw), Kc = sum_s rho_s x_s w_s^T from the coupling lists:
    // U[a][j] = sum_{(e, s) in xc(a)} rho_s A_e sum_{(e', p) in cw(s)} A_e' S[p][j]
    for (int k = tid; k < ndx * nw; k += NT) {
      const int ra = k / nw, j = k - ra * nw;
      double acc = 0.0;
      for (int q = pg[p_xcptr + ra]; q < pg[p_xcptr + ra + 1]; ++q) {
        const uint32_t w = f_xc[q];
        const int sidx = (int)(w >> 16);
        double t = 0.0;
        for (int q2 = pg[p_cwptr + sidx]; q2 < pg[p_cwptr + sidx + 1]; ++q2) {
          const uint32_t w2 = f_cw[q2];
          t += asb[w2 & 0xffff] * sym_at(Sl, (int)(w2 >> 16), j);
        }
        acc += rwb[pg[p_cplr + sidx]] * asb[w & 0xffff] * t;
      }
      Kc[k] = acc;  // the (now unused) Kc buffer holds U
    }
    T(7);
    __syncthreads();
    // ---- E_{i+1} = D_{i+1} - U Kc^T:  (U Kc^T)[a][b] = sum_{(e, s) in xc(b)} rho_s A_e (U w_s)[a]
    for (int k = tid; k < ndx * ndx; k += NT) {
      const int ra = k / ndx, cb = k - ra * ndx;
      double acc = 0.0;
      for (int q = pg[p_xcptr + cb]; q < pg[p_xcptr + cb + 1]; ++q) {
        const uint32_t w = f_xc[q];
        const int sidx = (int)(w >> 16);
        double t = 0.0;
        for (int q2 = pg[p_cwptr + sidx]; q2 < pg[p_cwptr + sidx + 1]; ++q2) {
          const uint32_t w2 = f_cw[q2];
          t += asb[w2 & 0xffff] * Kc[ra * nw + (int)(w2 >> 16)];
        }
        acc += rwb[pg[p_cplr + sidx]] * asb[w & 0xffff] * t;
      }
      Cb[k] -= acc;
    }
    T(8);
  }
  if constexpr (TIMING) {
    if (threadIdx.x == 0 && d.dbg)
      for (int k = 0; k < 9; ++k) d.dbg[(size_t)b * 16 + 16 * (size_t)gridDim.x + k] = (double)tacc[k];
  }
}

size_t factor_lds_bytes(const PlOcpHandle* h) {
  const int nwm = h->nw_max;
  FactorMap fm{std::max(std::max(std::max(nwm * (nwm + 1) / 2, h->ndx * nwm), FCH * h->ncol_max), GJ_LDS),
               std::max(h->nent_max, 1),
               std::max(h->nrow_max, 1), h->flen_max};
  return fm.total(h->ndx, nwm);
}

void launch_factor(PlOcpHandle* h) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)k_factor<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)k_factor<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const int nwm = h->nw_max;
  FactorMap fm{std::max(std::max(std::max(nwm * (nwm + 1) / 2, h->ndx * nwm), FCH * h->ncol_max), GJ_LDS),
               std::max(h->nent_max, 1),
               std::max(h->nrow_max, 1), h->flen_max};
  if (h->d.dbg)
    hipLaunchKernelGGL(k_factor<true>, dim3(h->B), dim3(256), fm.total(h->ndx, nwm), h->stream, h->d, h->N, h->n,
                       h->m, h->nnz, h->ndx, h->S_stride, nwm, fm, h->set.sigma);
  else
    hipLaunchKernelGGL(k_factor<false>, dim3(h->B), dim3(256), fm.total(h->ndx, nwm), h->stream, h->d, h->N, h->n,
                       h->m, h->nnz, h->ndx, h->S_stride, nwm, fm, h->set.sigma);
}
