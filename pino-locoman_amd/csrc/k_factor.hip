// Block factorisation of the reduced KKT system (the numeric refactorisation
// osqp.update(Ax=...) triggers, optimization/ocp.py:391-395; OSQP factors the
// quasi-definite KKT with QDLDL, here its reduced SPD form is factored).
//
//   K = P + sigma I + A^T diag(rho) A   is block tridiagonal over w_i = [dx_i, u_i].
//   The ADMM sweeps (k_admm.hip) need, per node, S_i = (Kt_ii + E_i)^-1 where
//     Kt_ii = diag(P + sigma) + sum_{rows r of node i} rho_r a_r a_r^T |_{w_i}
//     E_i   = D_i - Kc_{i-1} S_{i-1} Kc_{i-1}^T  on the dx_i block (0 for i = 0),
//     Kc_i  = K_{i+1,i},  D_{i+1} = sum_{coupling rows s} rho_s x_s x_s^T.
//
// Only E_i chains the nodes, and it touches the dx block alone.  Writing
//   Kt_ii = [[A, B], [B^T, C]]  (A: dx x dx, C: u x u),
// the Schur complement on the u block gives
//   S_xx = (A' + E_i)^-1,  A' = A - B C^-1 B^T,  G = C^-1 B^T,
//   S_ux = -G S_xx,        S_uu = C^-1 + G S_xx G^T,
// so everything but an X x X inverse (X = ndx) is independent of the chain:
//
//   k_fnode  one 256-thread workgroup per (problem, node), all in parallel: assembles
//            Kt_ii in LDS from host-balanced slot-owner streams, sweeps the u pivots of
//            [C | B^T] in registers (wave 0: the C columns, wave 1: the B^T columns),
//            and writes A', G, C^-1 to the factor scratch d.FS;
//   k_fchain one 256-thread workgroup per problem, sequential over the nodes: sweeps
//            A' + E_i (wave 0, one column per lane), forms S_ux / S_uu / E_{i+1} with
//            all four waves, and stores S_i in the lane-tile layout the ADMM streams.
//
// Sweep operator (symmetric Gauss-Jordan): pivot k with p = M_kk:
//   M_rj -= M_rk M_kj / p,  M_rk = M_rk / p,  M_kj = M_kj / p,  M_kk = -1 / p,
// which keeps M symmetric, so the pivot column is the pivot row: every lane
// publishes its row-k entry and reads the column back as a broadcast.
// Sweeping a set of pivots turns their block into -inverse, the off-block into
// inverse x off-block and the rest into the Schur complement.
#include <algorithm>
#include <type_traits>

#include "state.h"

namespace {

constexpr int NT = PL_FAC_NT;

__device__ __forceinline__ int lidx(int r, int c) { return r * (r + 1) / 2 + c; }  // packed lower, r >= c
__device__ __forceinline__ int sidx(int r, int c) { return r >= c ? lidx(r, c) : lidx(c, r); }

__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// compile-time loop: f(std::integral_constant<int, k>) for k in [K0, K1), so register
// arrays indexed by k stay in registers
template <int K0, int K1, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (K0 < K1) {
    f(std::integral_constant<int, K0>{});
    static_for<K0 + 1, K1>(f);
  }
}

// 1 / p for the SPD pivots (normal numbers): v_rcp_f64 and two Newton steps
__device__ __forceinline__ double rcp_nr(double p) {
  double r = __builtin_amdgcn_rcp(p);
  r = fma(r, fma(-p, r, 1.0), r);
  r = fma(r, fma(-p, r, 1.0), r);
  return r;
}

typedef double f64x4 __attribute__((ext_vector_type(4)));

// v_mfma_f64_16x16x4_f64 (tools/native/mfma_f64_check.hip pins the layout): lane l
// supplies A[l & 15][l >> 4] and B[l >> 4][l & 15]; D register r of lane l is
// D[(l >> 4) + 4 r][l & 15].
__device__ __forceinline__ f64x4 mfma4(double a, double b, f64x4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// Blocked sweep of the first 4 nblocks pivots of a symmetric matrix whose columns are
// held one per lane (R rows in registers), four pivots P = [k, k + 4) per block:
//   Q = M_PP^-1;  non-pivot column j: t = Q M_Pj, M_rj -= M_rP t, M_Pj = t;
//   pivot column j = k + q: M_rj = (M_rP Q)_q, M_Pj = -Q_:q.
// After all pivots the swept block holds -M^-1 (Schur complements / G elsewhere).
// The loop is rolled (small code: the instruction cache holds it) and the register
// column rotates by four rows per block, so the current pivot rows are always
// col[0..3]: at block B, col[r] holds row (r + 4 B) mod R.  The publishing wave
// writes its pivot-row entries (M_{k+p, l} = M_{l, k+p} by symmetry) twice, at lane l
// and lane l + R, so row (r + k) needs no modulo.  pb: 2 x [2 R_pub][4] doubles.
// kSync: 0 = one wave (wave-scope fence), 1 = workgroup barrier (publisher and
// readers are different waves; every wave of the group must call).
// kTrack: pmin <- min(pmin, every pivot) (the positive-definiteness test of the
// interior-point inertia correction; pivots are wave-uniform)
template <int R, int kSync, int kBatch, bool kTrack = false>
__device__ __forceinline__ void sweep_rot(double (&col)[R], double* pb, int pbstride, int l, int nblocks,
                                          bool publish, bool active, bool pivcols, double* pmin = nullptr) {
#pragma unroll 1
  for (int B = 0; B < nblocks; ++B) {
    const int k = 4 * B;
    double* pk = pb + (B & 1) * pbstride;
    if (publish && l < R) {  // lanes past R hold no row of the swept block
      const double2 v0 = make_double2(col[0], col[1]), v1 = make_double2(col[2], col[3]);
      double2* pw = reinterpret_cast<double2*>(pk + 4 * l);
      pw[0] = v0;
      pw[1] = v1;
      double2* pw2 = reinterpret_cast<double2*>(pk + 4 * (l + R));
      pw2[0] = v0;
      pw2[1] = v1;
    }
    if constexpr (kSync == 0) wsync();
    else __syncthreads();
    if (active) {
      const double2* pr = reinterpret_cast<const double2*>(pk + 4 * k);  // row k + r at pr[2 r]
      double m[4][4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const double2 a = pr[2 * p], b = pr[2 * p + 1];
        m[p][0] = a.x; m[p][1] = a.y; m[p][2] = b.x; m[p][3] = b.y;
      }
      // m <- -M_PP^-1 (4-pivot sweep, wave-uniform values)
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        if constexpr (kTrack) *pmin = fmin(*pmin, m[p][p]) + (m[p][p] == m[p][p] ? 0.0 : -1.0);  // NaN: fails
        const double pinv = rcp_nr(m[p][p]);
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
          for (int c = 0; c < 4; ++c)
            if (r != p && c != p) m[r][c] = fma(-m[r][p] * pinv, m[p][c], m[r][c]);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (r != p) { m[r][p] *= pinv; m[p][r] *= pinv; }
        m[p][p] = -pinv;
      }
      // branch-free: e_s = [q == s] on pivot lanes (0 elsewhere), pv = [pivot lane]
      const int q = l - k;
      const bool piv = pivcols && (unsigned)q < 4u;
      const double pv = piv ? 1.0 : 0.0;
      double e[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) e[p] = (piv && q == p) ? 1.0 : 0.0;
      double t[4], nb[4];
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const double qf = -(m[p][0] * col[0] + m[p][1] * col[1] + m[p][2] * col[2] + m[p][3] * col[3]);
        const double qcol = m[p][0] * e[0] + m[p][1] * e[1] + m[p][2] * e[2] + m[p][3] * e[3];  // -Q_pq
        nb[p] = fma(1.0 - pv, qf, qcol);
        t[p] = nb[p] + e[p];
      }
      // rank-4 update of the other rows, rotated into place: col[r - 4] <- row r, the
      // broadcast reads issued kBatch rows at a time (registers vs. latency), two-deep chains
#pragma unroll
      for (int r0 = 4; r0 < R; r0 += kBatch) {
        double2 ra[kBatch], rb[kBatch];
#pragma unroll
        for (int j = 0; j < kBatch; ++j)
          if (r0 + j < R) {
            ra[j] = pr[2 * (r0 + j)];
            rb[j] = pr[2 * (r0 + j) + 1];
          }
#pragma unroll
        for (int j = 0; j < kBatch; ++j)
          if (r0 + j < R) {
            const double h0 = fma(ra[j].y, t[1], ra[j].x * t[0]);
            const double h1 = fma(rb[j].y, t[3], rb[j].x * t[2]);
            col[r0 + j - 4] = col[r0 + j] - (h0 + h1);
          }
        if (kBatch < R) __builtin_amdgcn_sched_barrier(0);
      }
#pragma unroll
      for (int p = 0; p < 4; ++p) col[R - 4 + p] = nb[p];
    }
  }
}

typedef const __attribute__((address_space(4))) PlFacNode* CFac;
typedef const __attribute__((address_space(4))) uint32_t* CU32;
typedef const __attribute__((address_space(4))) double* CF64;

}  // namespace

// ---------------------------------------------------------------------------------
// Stage 1: per (problem, node).  X = ndx, UM >= nu (register columns of the sweep).
// HL: the interior point's exact-Hessian system -- Kt_ii += H_i (d.Hlag), pivots <= 0
// reported in d.ip_iflag, and (fac_only) only the problems flagged for a refactor
template <int X, int UM, bool HL>
__global__ __launch_bounds__(NT) void k_fnode(PlDev d, int n, int m, int nnz, int i0, int ni, long long fs_stride,
                                              double sigma, long long hl_stride, int fac_only) {
  const int task = blockIdx.x;
  const int b = task / ni;
  const int i = i0 + (task - b * ni);
  if constexpr (HL) {
    if (fac_only && !d.ip_iflag[4 * b + 1]) return;
  }
  const int tid = threadIdx.x, l = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform
  CFac fn = (CFac)d.fnodes + i;
  const int nw = fn->nw, U = fn->nu, nent = fn->nent;
  const int nK = (nw * (nw + 1) / 2 + 1) & ~1;
  extern __shared__ double lds[];
  double* K = lds;         // packed lower Kt_ii
  double* Ar = K + nK;     // rho-scaled A values (nent + 1, the last one zero), during the assembly
  double* Av = Ar + nent + 1;
  double* pb = K + nK;     // pivot block rows [2][512] during the sweep
  double* Gs = K + nK;     // after the sweep: G (U x X), row-major

  const double* __restrict__ As = d.As + (size_t)b * nnz + fn->ent_off;
  const double* __restrict__ rho = d.rho + (size_t)b * m + fn->row_off;
  const int* __restrict__ rid = d.rowidx + fn->ent_off;
  for (int e = tid; e <= nent; e += NT) {
    const double a = e < nent ? As[e] : 0.0;
    Av[e] = a;
    Ar[e] = e < nent ? rho[rid[e]] * a : 0.0;
  }
  for (int k = tid; k < nK; k += NT) K[k] = 0.0;
  __syncthreads();
  // ---- assembly: each thread owns a set of slots; its stream walks their triples
  {
    const uint32_t* __restrict__ st = d.kasm + fn->asm_off;
    const uint16_t* __restrict__ fl = d.kfl + fn->fl_off;
    const int L = fn->asm_len;
    double acc = 0.0;
    int f = 0;
    for (int t = 0; t < L; ++t) {
      const uint32_t q = st[(size_t)t * NT + tid];
      acc = fma(Ar[q & 0x7fff], Av[q >> 16], acc);
      if (q & 0x8000u) {
        K[fl[f * NT + tid]] = acc;
        acc = 0.0;
        ++f;
      }
    }
  }
  __syncthreads();
  {
    const double* __restrict__ Ps = d.Ps + (size_t)b * n + fn->x_off;
    for (int c = tid; c < nw; c += NT) K[lidx(c, c)] += Ps[c] + sigma;
  }
  if constexpr (HL) {
    __syncthreads();
    const double* __restrict__ Hb = d.Hlag + (size_t)b * hl_stride + d.hoff[i];
    for (int k = tid; k < nw * (nw + 1) / 2; k += NT) K[k] += Hb[k];
  }
  __syncthreads();
  double* FS = d.FS + (size_t)b * fs_stride + fn->fs_off;
  double* Ag = FS;
  double* Gg = Ag + X * X;
  double* Cg = Gg + U * X;
  if (U > 0) {
    // ---- sweep the u pivots of [C | B^T]: wave 0 holds column l of C, wave 1 column l of B^T
    double col[UM];
    if (w == 0) {
#pragma unroll
      for (int r = 0; r < UM; ++r) {  // clamped unconditional loads, then select (no per-element branches)
        const double v = K[sidx(X + min(r, U - 1), X + min(l, U - 1))];
        // arithmetic masks, not selects: a select lets the compiler sink each load
        // into its own branch (one serialised round trip per element)
        col[r] = fma(v, (r < U && l < U) ? 1.0 : 0.0, (r == l && l >= U) ? 1.0 : 0.0);
      }
    } else if (w == 1) {
#pragma unroll
      for (int r = 0; r < UM; ++r) {
        const double v = K[lidx(X + min(r, U - 1), min(l, X - 1))];
        col[r] = v * ((r < U && l < X) ? 1.0 : 0.0);
      }
    }
    // pivots k >= U meet an identity pad (wave 0) and zero rows (wave 1): no-ops;
    // the rotation is back to the identity once all UM / 4 blocks are swept
    double pmin = 1.0;
    sweep_rot<UM, 1, 8, HL>(col, pb, 8 * 64, l, UM / 4, w == 0, w < 2, w == 0, &pmin);
    if constexpr (HL) {
      if (w == 0 && l == 0 && !(pmin > 0.0)) d.ip_iflag[4 * b] = 1;
    }
    if (w == 0 && l < U) {
#pragma unroll
      for (int r = 0; r < UM; ++r)
        if (r < U) Cg[r * U + l] = -col[r];
    } else if (w == 1 && l < X) {
#pragma unroll
      for (int r = 0; r < UM; ++r)
        if (r < U) {
          Gg[r * X + l] = col[r];
          Gs[r * X + l] = col[r];
        }
    }
    __syncthreads();
  }
  // ---- A' = A - B G (X x X) on the f64 MFMA: lower 16 x 16 tiles (mt >= nt), K = U in
  // steps of 4; written to both triangles
  {
    constexpr int NX = (X + 15) / 16;
    constexpr int NTL = NX * (NX + 1) / 2;
    const int ku = (U + 3) / 4;
    for (int tt = w; tt < NTL; tt += 4) {
      int mt = 0;
      while ((mt + 1) * (mt + 2) / 2 <= tt) ++mt;
      const int nt = tt - mt * (mt + 1) / 2;
      const int ar = 16 * mt + (l & 15), bcol = 16 * nt + (l & 15);
      f64x4 acc = {0.0, 0.0, 0.0, 0.0};
      for (int kk = 0; kk < ku; ++kk) {
        const int u = 4 * kk + (l >> 4);
        const int uc = min(u, U - 1);
        const double av0 = K[lidx(X + uc, min(ar, X - 1))];
        const double bv0 = Gs[uc * X + min(bcol, X - 1)];
        const double av = av0 * ((u < U && ar < X) ? 1.0 : 0.0);
        const double bv = bv0 * ((u < U && bcol < X) ? 1.0 : 0.0);
        acc = mfma4(av, bv, acc);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = 16 * mt + (l >> 4) + 4 * r;
        if (row < X && bcol < X && bcol <= row) {
          const double v = K[lidx(row, bcol)] - acc[r];
          Ag[row * X + bcol] = v;
          Ag[bcol * X + row] = v;
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------------
// Stage 2: the Schur chain of one problem (one 256-thread workgroup).
//
// Store S_i in the ADMM lane-tile layout (state.h): 4x4 tile t = K l + k of lane l,
// pair j at s_off + ((k * 8 + j) * 64 + l) * 2 (coalesced over o).  Threads [t0, t0 + nt).
__device__ __forceinline__ void store_tiles(const PlDev& d, CFac fn, const double* Sl, double* Sg, int t0, int nt,
                                            int tid) {
  double* Sn = Sg + fn->s_off;
  const int nunit = fn->nunit, ntl = fn->ntl, nw = fn->nw;
  const int total = nunit * 64 * 16;
  for (int o = tid - t0; o < total; o += nt) {
    const int slot = o & 1, ln = (o >> 1) & 63, j = (o >> 7) & 7, k = o >> 10;
    const int t = nunit * ln + k;
    double val = 0.0;
    if (t < ntl) {
      int I = (int)((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
      I -= (I * (I + 1) / 2 > t);
      I += ((I + 1) * (I + 2) / 2 <= t);
      const int J = t - I * (I + 1) / 2;
      const int gi = 4 * I + (j >> 1), gj = 4 * J + 2 * (j & 1) + slot;
      if (gi < nw && gj < nw) val = Sl[sidx(gi, gj)];
    }
    Sn[o] = val;
  }
}

template <int X, bool HL>
__global__ __launch_bounds__(NT) void k_fchain(PlDev d, int N, int m, int nnz, int S_stride, long long fs_stride,
                                               int nwm, int ny, int ncw, int fac_only, int gc, int ncm, int nxcm) {
  const int b = blockIdx.x;
  if constexpr (HL) {
    if (fac_only && !d.ip_iflag[4 * b + 1]) return;
  }
  const int tid = threadIdx.x, l = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform
  extern __shared__ double lds[];
  const int nS = (nwm * (nwm + 1) / 2 + 1) & ~1;
  constexpr int nE = (X * (X + 1) / 2 + 1) & ~1;
  double* Sl = lds;       // packed lower S_i
  double* Yb = Sl + nS;   // transpose buffer [X][X + 1], then Y [npc][X]
  double* pb = Yb;        // pivot block rows [2][128][4] during the sweep (Yb is free then; ny >= 1024)
  double* Eb = Yb + ny;   // E_i, packed lower
  double* Acw = Eb + nE;  // A values of the coupling rows' w parts (ncw)
  double* cv = Acw + ncw;   // rho_a A_{e_a} (X)
  double* ev = cv + X;      // A_{e_a} (X)
  // optional phase timing (thread 0, s_memtime): 8 accumulators + last stamp in LDS
  unsigned long long* tacc = reinterpret_cast<unsigned long long*>(ev + X);
  // general coupling (gc): Z [ncm][ncm], staged dx_{i+1} values of the coupling rows, their rho
  double* Zb = ev + X + 10;
  double* Axc = Zb + ncm * ncm;
  double* rcl = Axc + nxcm;
  const bool TIMING = d.dbg != nullptr;  // optional phase timing (PL_ADMM_TIMING=1)
  if (TIMING && tid < 9) tacc[tid] = 0;
  auto T = [&](int slot) {
    if (TIMING) {
      if (tid == 0) {
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        if (slot >= 0) tacc[slot] += now - tacc[8];
        tacc[8] = now;
      }
    }
  };
  for (int k = tid; k < nE; k += NT) Eb[k] = 0.0;
  double* Sg = d.S + (size_t)b * S_stride;
  const double* __restrict__ FSb = d.FS + (size_t)b * fs_stride;
  for (int i = 0; i <= N; ++i) {
    CFac fn = (CFac)d.fnodes + i;
    const int U = fn->nu;
    const double* __restrict__ Ag = FSb + fn->fs_off;
    CF64 Gg = (CF64)(Ag + X * X);
    const double* __restrict__ Cg = Ag + X * X + U * X;
    CU32 cp = (CU32)d.kcpl + fn->cp_off;
    CU32 crow = cp;
    CU32 cent = cp + X;
    CU32 cwptr = cp + 2 * X;
    CU32 pcl = cp + 3 * X + 1;
    const int npc = fn->npc;
    CU32 cwl = pcl + npc;
    // general coupling program (api.hip build_factor_prog): crow[nc] | cwptr[nc + 1] | pcl[npc] |
    // cw[ncw] | xcptr[X + 1] | xc[nxc]
    const int nc = gc ? fn->nc : 0;
    CU32 gcwptr = cp + nc;
    CU32 gpcl = gcwptr + nc + 1;
    CU32 gcwl = gpcl + npc;
    CU32 gxcptr = gcwl + (gc && i < N ? (int)gcwptr[nc] : 0);
    CU32 gxcl = gxcptr + X + 1;
    const double* __restrict__ Asb = d.As + (size_t)b * nnz + fn->ent_off;
    const double* __restrict__ rhob = d.rho + (size_t)b * m + fn->row_off;
    __syncthreads();
    T(-1);
    if (w == 0) {
      // ---- S_xx = (A' + E_i)^-1, one column per lane.  The sweep runs on XS = X rounded up
      // to 4 pivots: rows / columns X..XS-1 are an identity pad (their pivots are no-ops),
      // e.g. X = 30 for B2G centroidal_vel (6 + nv).
      constexpr int XS = (X + 3) & ~3;
      double col[XS];
#pragma unroll
      for (int r = 0; r < XS; ++r)
      {
        // lanes >= XS duplicate column XS - 1: never pivots, never published, never stored
        const int lc = min(l, XS - 1);
        const int rc = min(r, X - 1), cc = min(lc, X - 1);
        const double v = Ag[rc * X + cc] + Eb[sidx(rc, cc)];
        col[r] = (r < X && lc < X) ? v : (r == lc ? 1.0 : 0.0);
      }
      unsigned long long ts0 = 0;
      if (TIMING) ts0 = __builtin_amdgcn_s_memtime();
      double pmin = 1.0;
      sweep_rot<XS, 0, XS, HL>(col, pb, 8 * 64, l, XS / 4, true, true, true, &pmin);
      if constexpr (HL) {
        if (l == 0 && !(pmin > 0.0)) d.ip_iflag[4 * b] = 1;
      }
      if (TIMING) {
        const unsigned long long ts1 = __builtin_amdgcn_s_memtime();
        if (l == 0) tacc[5] += ts1 - ts0;
      }
      // symmetrise -col (sweep round-off) through the transpose buffer
      constexpr int XP = X + 1;
      if (l < X) {
#pragma unroll
        for (int r = 0; r < X; ++r) Yb[r * XP + l] = -col[r];
      }
      __syncthreads();  // (a) the other waves are done with Sl (tile store of S_{i-1})
      if (l < X)
        for (int r = l; r < X; ++r) Sl[lidx(r, l)] = 0.5 * (Yb[r * XP + l] + Yb[l * XP + r]);
    } else {
      // ---- waves 1-3, while wave 0 sweeps: store S_{i-1}, stage node i's coupling values
      unsigned long long ts0 = 0;
      if (TIMING) ts0 = __builtin_amdgcn_s_memtime();
      if (i > 0) store_tiles(d, (CFac)d.fnodes + (i - 1), Sl, Sg, 64, NT - 64, tid);
      if (i < N && gc) {
        const int ncwi = (int)gcwptr[nc], nxci = (int)gxcptr[X];
        for (int q = tid - 64; q < ncwi; q += NT - 64) Acw[q] = Asb[gcwl[q] & 0xffff];
        for (int q = tid - 64; q < nxci; q += NT - 64) Axc[q] = Asb[gxcl[q] & 0xffff];
        for (int q = tid - 64; q < nc; q += NT - 64) rcl[q] = rhob[crow[q]];
      } else if (i < N) {
        const int ncwi = (int)cwptr[X];
        for (int q = tid - 64; q < ncwi; q += NT - 64) Acw[q] = Asb[cwl[q] & 0xffff];
        for (int a = tid - 64; a < X; a += NT - 64) {
          const double ea = Asb[cent[a]];
          ev[a] = ea;
          cv[a] = rhob[crow[a]] * ea;
        }
      }
      if (TIMING) {
        const unsigned long long ts1 = __builtin_amdgcn_s_memtime();
        if (tid == 64) tacc[7] += ts1 - ts0;
      }
      __syncthreads();  // (a)
    }
    __syncthreads();
    T(0);
    // ---- S_ux = -G S_xx (U x X) and S_uu = C^-1 - G S_ux^T (U x U, lower) on the f64
    // MFMA: wave w owns the 16-row tile mt = w of both; K = X in steps of 4.
    {
      constexpr int KX = (X + 3) / 4;  // K = X in steps of 4 (a partial last step is masked)
      constexpr int NX = (X + 15) / 16;
      const int mt = w;
      const bool act = 16 * mt < U;
      const int arow = 16 * mt + (l & 15);
      double ga[KX];  // G[16 mt + (l & 15)][4 kk + (l >> 4)]
#pragma unroll
      for (int kk = 0; kk < KX; ++kk) {
        const int kc = 4 * kk + (l >> 4);
        const double v = Ag[X * X + min(arow, max(U - 1, 0)) * X + min(kc, X - 1)];
        ga[kk] = v * ((act && arow < U && kc < X) ? 1.0 : 0.0);
      }
      if (act) {
#pragma unroll
        for (int nt = 0; nt < NX; ++nt) {
          f64x4 acc = {0.0, 0.0, 0.0, 0.0};
          const int bc = 16 * nt + (l & 15);
#pragma unroll
          for (int kk = 0; kk < KX; ++kk) {
            const int kc = 4 * kk + (l >> 4);
            const double bv0 = Sl[sidx(min(kc, X - 1), min(bc, X - 1))];
            const double bv = bv0 * ((bc < X && kc < X) ? 1.0 : 0.0);
            acc = mfma4(ga[kk], bv, acc);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * mt + (l >> 4) + 4 * r;
            if (row < U && bc < X) Sl[lidx(X + row, bc)] = -acc[r];
          }
        }
      }
      __syncthreads();
      T(1);
      if (act) {
        for (int nt = 0; nt <= mt; ++nt) {
          f64x4 acc = {0.0, 0.0, 0.0, 0.0};
          const int bu = 16 * nt + (l & 15);
          double ci[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * mt + (l >> 4) + 4 * r;
            const double v = Cg[min(row, U - 1) * U + min(bu, U - 1)];
            ci[r] = v * ((row < U && bu <= row) ? 1.0 : 0.0);
          }
#pragma unroll
          for (int kk = 0; kk < KX; ++kk) {
            const int kc = 4 * kk + (l >> 4);
            const double bv0 = Sl[lidx(X + min(bu, U - 1), min(kc, X - 1))];
            const double bv = bv0 * ((bu < U && kc < X) ? 1.0 : 0.0);
            acc = mfma4(ga[kk], bv, acc);
          }
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int row = 16 * mt + (l >> 4) + 4 * r;
            if (row < U && bu <= row) Sl[lidx(X + row, X + bu)] = ci[r] - acc[r];
          }
        }
      }
    }
    __syncthreads();
    T(2);
    if (i == N) break;
    if (gc) {
      // ---- general coupling: E_{i+1} = Wc^T Z Wc with Z = R - R Vc S Vc^T R over the nc
      // coupling rows (Vc: their w_i parts, Wc: their dx_{i+1} parts)
      // Y[pc][s] = (S Vc_s^T)[pcl[pc]]
      if (l < nc) {
        const int q0 = (int)gcwptr[l], q1 = (int)gcwptr[l + 1];
        for (int pc = w; pc < npc; pc += 4) {
          const int p = (int)gpcl[pc];
          double acc = 0.0;
          for (int q = q0; q < q1; ++q) acc = fma(Acw[q], Sl[sidx(p, (gcwl[q] >> 16) & 0xff)], acc);
          Yb[pc * nc + l] = acc;
        }
      }
      __syncthreads();
      T(3);
      // Z[s][t] = rho_s d_st - rho_s rho_t Vc_s . Y[:, t]  (lower, mirrored)
      if (l < nc) {
        const double rt = rcl[l];
        for (int s2 = w; s2 < nc; s2 += 4) {
          if (l > s2) continue;
          double acc = 0.0;
          for (int q = (int)gcwptr[s2]; q < (int)gcwptr[s2 + 1]; ++q)
            acc = fma(Acw[q], Yb[(gcwl[q] >> 24) * nc + l], acc);
          const double rs = rcl[s2];
          const double z = (s2 == l ? rs : 0.0) - rs * rt * acc;
          Zb[s2 * nc + l] = z;
          Zb[l * nc + s2] = z;
        }
      }
      __syncthreads();
      // T[s][b] = sum_t Z[s][t] Wc[t][b]  (into the Y buffer)
      if (l < X) {
        const int q0 = (int)gxcptr[l], q1 = (int)gxcptr[l + 1];
        for (int s2 = w; s2 < nc; s2 += 4) {
          double acc = 0.0;
          for (int q = q0; q < q1; ++q) acc = fma(Axc[q], Zb[s2 * nc + (gxcl[q] >> 16)], acc);
          Yb[s2 * X + l] = acc;
        }
      }
      __syncthreads();
      // E[a][b] = sum_s Wc[s][a] T[s][b]  (lower)
      if (l < X) {
        for (int a = w; a < X; a += 4) {
          if (l > a) continue;
          double acc = 0.0;
          for (int q = (int)gxcptr[a]; q < (int)gxcptr[a + 1]; ++q)
            acc = fma(Axc[q], Yb[(gxcl[q] >> 16) * X + l], acc);
          Eb[lidx(a, l)] = acc;
        }
      }
      T(4);
      continue;
    }
    // ---- E_{i+1} = D - Kc S Kc^T, Kc row a = rho_a A_{e_a} w_{s_a}^T (one coupling row per column)
    // Y[pc][bb] = (S w_{s_bb})[pcl[pc]]: thread (w, l) -> bb = l, pc = w (mod 4)
    if (l < X) {
      const int q0 = (int)cwptr[l], q1 = (int)cwptr[l + 1];
      constexpr int CR = 4;  // list entries held in registers (longer lists: LDS loop)
      double av[CR];
      int qc[CR];
#pragma unroll
      for (int j = 0; j < CR; ++j) {
        const bool ok = q0 + j < q1;
        av[j] = ok ? Acw[q0 + j] : 0.0;
        qc[j] = ok ? (int)((cwl[q0 + j] >> 16) & 0xff) : 0;
      }
      for (int pc = w; pc < npc; pc += 4) {
        const int p = (int)pcl[pc];
        double acc = 0.0;
#pragma unroll
        for (int j = 0; j < CR; ++j) acc = fma(av[j], Sl[sidx(p, qc[j])], acc);
        for (int q = q0 + CR; q < q1; ++q) acc = fma(Acw[q], Sl[sidx(p, (cwl[q] >> 16) & 0xff)], acc);
        Yb[pc * X + l] = acc;
      }
    }
    __syncthreads();
    T(3);
    if (l < X) {
      const double cb = cv[l];
      for (int a = w; a < X; a += 4) {  // lower triangle (l <= a) only: E is symmetric
        if (l > a) continue;
        const double ca = cv[a];
        double acc = 0.0;
        for (int q = (int)cwptr[a]; q < (int)cwptr[a + 1]; ++q)
          acc = fma(Acw[q], Yb[(cwl[q] >> 24) * X + l], acc);
        Eb[lidx(a, l)] = (a == l ? ca * ev[a] : 0.0) - ca * cb * acc;
      }
    }
    T(4);
  }
  store_tiles(d, (CFac)d.fnodes + N, Sl, Sg, 0, NT, tid);
  T(6);
  if (TIMING) {
    if (tid == 0)
      for (int k = 0; k < 8; ++k) d.dbg[(size_t)b * 16 + 16 * (size_t)gridDim.x + k] = (double)tacc[k];
  }
}

namespace {

template <int X, int UM, bool HL>
void launch_fnode(PlOcpHandle* h, int g) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)k_fnode<X, UM, HL>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((k_fnode<X, UM, HL>), dim3(h->B * h->fg_n[g]), dim3(NT), h->fg_lds[g], h->stream, h->d, h->n,
                     h->m, h->nnz, h->fg_i0[g], h->fg_n[g], h->fs_stride, h->set.sigma, h->hl_stride, h->fac_only);
}

template <int X, bool HL>
void launch_fchain(PlOcpHandle* h) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)k_fchain<X, HL>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((k_fchain<X, HL>), dim3(h->B), dim3(NT), h->fchain_lds, h->stream, h->d, h->N, h->m, h->nnz,
                     h->S_stride, h->fs_stride, h->nw_max, h->fchain_ny, h->fchain_ncw, h->fac_only, h->fac_gc,
                     h->fchain_nc, h->fchain_nxc);
}

template <int X, bool HL>
void launch_factor_xh(PlOcpHandle* h) {
  for (int g = 0; g < h->nfgroup; ++g) {
    if (h->fg_um[g] <= 40) launch_fnode<X, 40, HL>(h, g);
    else launch_fnode<X, 64, HL>(h, g);
  }
  launch_fchain<X, HL>(h);
}

template <int X>
void launch_factor_x(PlOcpHandle* h) {
  if (h->fac_hlag) launch_factor_xh<X, true>(h);
  else launch_factor_xh<X, false>(h);
}

}  // namespace

// ndx values of the shipped models: 36 (Go2 / B2 whole body), 48 (B2G whole body),
// 24 (Go2 / B2 centroidal_vel: 6 + nv), 30 (B2G centroidal_vel, swept with a 2-row identity
// pad); the handle refuses others.
bool factor_supports_ndx(int ndx) { return ndx == 24 || ndx == 30 || ndx == 36 || ndx == 48; }

void launch_factor_pre(PlOcpHandle* h) {
  launch_acpl(h);  // the sweep's compact coupling A values (k_admm.hip) for this As
}

void launch_factor_core(PlOcpHandle* h) {
  switch (h->ndx) {
    case 24: launch_factor_x<24>(h); break;
    case 30: launch_factor_x<30>(h); break;
    case 36: launch_factor_x<36>(h); break;
    case 48: launch_factor_x<48>(h); break;
    default: break;
  }
}

void launch_factor_post(PlOcpHandle* h) {
  if (h->admm_rc) launch_fred(h);  // chain blocks of the reduced-chain ADMM (k_admm_rc.hip)
}

void launch_factor(PlOcpHandle* h) {
  launch_factor_pre(h);
  launch_factor_core(h);
  launch_factor_post(h);
}
