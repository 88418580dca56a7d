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

// Workgroup barrier that orders LDS only (lgkmcnt + s_barrier): __syncthreads() would also
// wait for every outstanding global store.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
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

// Blocked symmetric sweep, four pivots P = [k, k + 4) per block, M_PP = L D L^T:
//   Q = M_PP^-1;  non-pivot column j: t = M_PP^-1 M_Pj (substitution), M_rj -= M_rP t, M_Pj = t;
//   pivot column j = k + q: M_rj = (M_rP Q)_q, M_Pj = -Q_:q.
// After all pivots the swept block holds -M^-1 (Schur complements / G elsewhere).
// Columns are held one per lane.  The loop over the pivot blocks is rolled (small code:
// the instruction cache holds it; the fully unrolled 48-step sweep was ~60 KB of code and
// ran 4x slower).  Until r03 one wave held all rows of its columns with the register column
// rotating four rows per block (sweep_rot); the rows are now dealt to several waves.
// The rows of every column are dealt to NW waves in blocks of four
// (block B -> wave B % NW of the column set, local block B / NW): a wave holds NB local
// blocks = 4 NB rows of column l (lane), col[4 j + q] = row 4 (ws + NW j) + q, ws = the
// wave's index within its column set.  Per pivot block the owner wave of each column set
// publishes its four pivot rows at its columns (pkC: the set holding the pivot columns,
// whose entries at column r are also M_{r,P} by symmetry; pkO: this wave's set), one
// barrier, then every wave updates its own rows from the broadcast pivot rows.  Each
// element sees the same operations in the same order as in the one-wave rotated sweep, with
// 1 / NW of the rows per wave.  No rotation: col[] ends in natural order.  Rows past R (waves with fewer
// blocks) are padding and never used.  Every wave of the workgroup must call.
//   isC: this wave belongs to the set holding the pivot columns (identity on its pivot lanes)
//   ncol: lanes carrying a column of this wave's set (the others duplicate column ncol - 1)
//   side(B): independent work interleaved with pivot block B (k_fchain: slices of the
//   previous node's tile store); the barriers order LDS only, so its global stores drain
//   in the background
template <int NB, int R, int NW, bool kTrack = false, class Side>
__device__ __forceinline__ void sweep_split(double (&col)[4 * NB], double* pbC, double* pbO, int pbstride, int l,
                                            int ws, bool isC, int ncol, double* pmin, Side&& side) {
  constexpr int nblocks = R / 4;
  // outer loop unrolled over the local block index (so the owner's pivot rows are
  // compile-time register indices), inner loop rolled over the owner wave
#pragma unroll
  for (int lb = 0; lb < NB; ++lb)
#pragma unroll 1
  for (int ow = 0; ow < NW; ++ow) {
    const int B = NW * lb + ow;
    if (B >= nblocks) break;
    const int k = 4 * B;
    double* pkC = pbC + (B & 1) * pbstride;
    double* pkO = pbO + (B & 1) * pbstride;
    if (ws == ow && l < ncol) {
      double2* pw = reinterpret_cast<double2*>(pkO + 4 * l);
      pw[0] = make_double2(col[4 * lb], col[4 * lb + 1]);
      pw[1] = make_double2(col[4 * lb + 2], col[4 * lb + 3]);
    }
    lds_barrier();
    side(B);
    const double2* pr = reinterpret_cast<const double2*>(pkC + 4 * k);
    double m[4][4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const double2 a = pr[2 * p], b = pr[2 * p + 1];
      m[p][0] = a.x; m[p][1] = a.y; m[p][2] = b.x; m[p][3] = b.y;
    }
    // LDL^T of the pivot block (wave-uniform, no pivoting: the block is SPD).  A non-pivot column
    // takes t = M_PP^-1 M_Pj by substitution and the pivot columns take Q = M_PP^-1 from the same
    // factors.  Until r05 Q came from a Gauss-Jordan of the 4x4 block and t = Q M_Pj: on
    // ill-conditioned pivot blocks (the u block of a stance node, cond(C) ~ 5e5) the explicit
    // inverse applied to the pivot rows lost ~20x the accuracy of the substitution (C^-1 1e-10 ..
    // 3e-10 against 1e-11 in long double, profiles/r05/factor_stages_*), which 100 ADMM
    // iterations carried into the QP step as up to 1.5e-7 (all-stance fixture).  Substitution for
    // t with the Gauss-Jordan Q kept for the pivot columns was worse still (an inconsistent
    // update, 7e-7 on go2_rnea_fd_n20); both from the LDL^T: every fixture's step <= 1e-9 of the
    // KKT oracle but one (3.4e-9, profiles/r05/parity_sweep*.json).
    double Lm[4][4], dinv[4], dd[4];
    {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        double s = m[j][j];
#pragma unroll
        for (int k2 = 0; k2 < j; ++k2) s = fma(-Lm[j][k2] * dd[k2], Lm[j][k2], s);
        dd[j] = s;
        dinv[j] = rcp_nr(s);
#pragma unroll
        for (int i2 = j + 1; i2 < 4; ++i2) {
          double t2 = m[i2][j];
#pragma unroll
          for (int k2 = 0; k2 < j; ++k2) t2 = fma(-Lm[i2][k2] * dd[k2], Lm[j][k2], t2);
          Lm[i2][j] = t2 * dinv[j];
        }
      }
    }
    // the pivots d are the Gauss-Jordan pivots: the interior point's inertia check (<= 0 or NaN)
    if constexpr (kTrack) {
#pragma unroll
      for (int p = 0; p < 4; ++p) *pmin = fmin(*pmin, dd[p]) + (dd[p] == dd[p] ? 0.0 : -1.0);
    }
    // Q = L^-T D^-1 L^-1 (the pivot columns), m = -Q
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      double y[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        double a = r == c ? 1.0 : 0.0;
#pragma unroll
        for (int k2 = 0; k2 < r; ++k2) a = fma(-Lm[r][k2], y[k2], a);
        y[r] = a;
      }
      double z[4];
#pragma unroll
      for (int r = 3; r >= 0; --r) {
        double a = y[r] * dinv[r];
#pragma unroll
        for (int k2 = 3; k2 > r; --k2) a = fma(-Lm[k2][r], z[k2], a);
        z[r] = a;
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) m[r][c] = -z[r];
    }
    // this lane's column of the pivot rows
    const int lc = min(l, ncol - 1);
    const double2 o0 = reinterpret_cast<const double2*>(pkO + 4 * lc)[0];
    const double2 o1 = reinterpret_cast<const double2*>(pkO + 4 * lc)[1];
    const double own[4] = {o0.x, o0.y, o1.x, o1.y};
    const int q = l - k;
    const bool piv = isC && (unsigned)q < 4u;
    const double pv = piv ? 1.0 : 0.0;
    double e[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) e[p] = (piv && q == p) ? 1.0 : 0.0;
    // t = M_PP^-1 own: forward substitution, 1 / d, back substitution
    double ts[4];
    {
      const double y0 = own[0];
      const double y1 = fma(-Lm[1][0], y0, own[1]);
      const double y2 = fma(-Lm[2][1], y1, fma(-Lm[2][0], y0, own[2]));
      const double y3 = fma(-Lm[3][2], y2, fma(-Lm[3][1], y1, fma(-Lm[3][0], y0, own[3])));
      ts[3] = y3 * dinv[3];
      ts[2] = fma(-Lm[3][2], ts[3], y2 * dinv[2]);
      ts[1] = fma(-Lm[3][1], ts[3], fma(-Lm[2][1], ts[2], y1 * dinv[1]));
      ts[0] = fma(-Lm[3][0], ts[3], fma(-Lm[2][0], ts[2], fma(-Lm[1][0], ts[1], y0 * dinv[0])));
    }
    double t[4], nb[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const double qcol = m[p][0] * e[0] + m[p][1] * e[1] + m[p][2] * e[2] + m[p][3] * e[3];
      nb[p] = fma(1.0 - pv, ts[p], qcol);
      t[p] = nb[p] + e[p];
    }
    const bool own_blk = ws == ow;
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int g0 = 4 * (ws + NW * j);  // first row of local block j
      if (own_blk && lb == j) {
#pragma unroll
        for (int p = 0; p < 4; ++p) col[4 * j + p] = nb[p];
      } else if (g0 < R) {
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const double2 ra = reinterpret_cast<const double2*>(pkC + 4 * (g0 + p))[0];
          const double2 rb = reinterpret_cast<const double2*>(pkC + 4 * (g0 + p))[1];
          const double h0 = fma(ra.y, t[1], ra.x * t[0]);
          const double h1 = fma(rb.y, t[3], rb.x * t[2]);
          col[4 * j + p] = col[4 * j + p] - (h0 + h1);
        }
      }
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
  if (ip_skip(d, b)) return;
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

  // optional phase timing (PL_ADMM_TIMING=1): thread 0's s_memtime per phase, added into
  // d.dbg[32 B + 8 b + k] (k: 0 staging, 1 assembly, 2 diagonal / H, 3 u sweep, 4 C / G
  // store, 5 A' MFMA) by global f64 atomics
  const bool TIMING = d.dbg != nullptr;
  unsigned long long tl = TIMING ? __builtin_amdgcn_s_memtime() : 0ull;
  auto T = [&](int slot) {
    if (TIMING && tid == 0) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      atomicAdd(d.dbg + (size_t)32 * gridDim.x / ni + (size_t)8 * b + slot, (double)(now - tl));
      tl = now;
    }
  };
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
  T(0);
  // ---- assembly: each thread owns a set of slots; its stream walks their triples
  {
    // the stream words are prefetched PF steps ahead (double-buffered registers), the slot
    // indices two flags ahead, and a chunk's LDS operands are read before its slot stores: the
    // one-word-per-step loop waited an L2 round trip per product (40 k of a B2G node's 70 k
    // cycles, r04); same FMA order
    const uint32_t* __restrict__ st = d.kasm + fn->asm_off;
    const uint16_t* __restrict__ fl = d.kfl + fn->fl_off;
    const int L = fn->asm_len, FL = fn->fl_len;
    constexpr int PF = 8;
    double acc = 0.0;
    int f = 0;
    if (L > 0) {
      int fcur = fl[tid], fnext = fl[(size_t)min(1, FL - 1) * NT + tid];
      uint32_t qa[PF];
#pragma unroll
      for (int u = 0; u < PF; ++u) qa[u] = st[(size_t)min(u, L - 1) * NT + tid];
      for (int t0 = 0; t0 < L; t0 += PF) {
        uint32_t qn[PF];
#pragma unroll
        for (int u = 0; u < PF; ++u) qn[u] = st[(size_t)min(t0 + PF + u, L - 1) * NT + tid];
        // the chunk's operands first: the slot stores below may alias Ar / Av for the compiler,
        // which would otherwise issue each load after the previous iteration's store
        double ar[PF], av[PF];
#pragma unroll
        for (int u = 0; u < PF; ++u) {
          ar[u] = Ar[qa[u] & 0x7fff];
          av[u] = Av[qa[u] >> 16];
        }
#pragma unroll
        for (int u = 0; u < PF; ++u) {
          const uint32_t q = qa[u];
          if (t0 + u < L) {
            acc = fma(ar[u], av[u], acc);
            if (q & 0x8000u) {
              K[fcur] = acc;
              acc = 0.0;
              ++f;
              fcur = fnext;
              fnext = fl[(size_t)min(f + 1, FL - 1) * NT + tid];
            }
          }
        }
#pragma unroll
        for (int u = 0; u < PF; ++u) qa[u] = qn[u];
      }
    }
  }
  __syncthreads();
  T(1);
  {
    const double* __restrict__ Ps = d.Ps + (size_t)b * n + fn->x_off;
    for (int c = tid; c < nw; c += NT) K[lidx(c, c)] += Ps[c] + sigma;
  }
  if constexpr (HL) {
    // + H_i: a thread's entries of the packed block loaded together (one round trip per 16,
    // not per entry: 20 k of a B2G node's cycles, r05)
    __syncthreads();
    const double* __restrict__ Hb = d.Hlag + (size_t)b * hl_stride + d.hoff[i];
    const int ne = nw * (nw + 1) / 2;
    constexpr int HB = 16;
    for (int k0 = 0; k0 < ne; k0 += NT * HB) {
      double hv[HB];
#pragma unroll
      for (int u = 0; u < HB; ++u) hv[u] = Hb[min(k0 + u * NT + tid, ne - 1)];
#pragma unroll
      for (int u = 0; u < HB; ++u)
        if (k0 + u * NT + tid < ne) K[k0 + u * NT + tid] += hv[u];
    }
  }
  __syncthreads();
  T(2);
  double* FS = d.FS + (size_t)b * fs_stride + fn->fs_off;
  double* Ag = FS;
  double* Gg = Ag + X * X;
  double* Cg = Gg + U * X;
  if (U > 0) {
    // ---- sweep the u pivots of [C | B^T]: waves 0, 2 hold column l of C, waves 1, 3 column
    // l of B^T, the rows of each column split between the two waves of its set (sweep_split)
    constexpr int NBU = (UM / 4 + 1) / 2;
    const int set = w & 1, ws = w >> 1;
    double col[4 * NBU];
#pragma unroll
    for (int j = 0; j < NBU; ++j)
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int r = 4 * (ws + 2 * j) + p;
        // clamped unconditional loads, arithmetic masks (no per-element branches)
        if (set == 0) {
          const double v = K[sidx(X + min(r, U - 1), X + min(l, U - 1))];
          col[4 * j + p] = fma(v, (r < U && l < U) ? 1.0 : 0.0, (r == l && l >= U) ? 1.0 : 0.0);
        } else {
          const double v = K[lidx(X + min(r, U - 1), min(l, X - 1))];
          col[4 * j + p] = v * ((r < U && l < X) ? 1.0 : 0.0);
        }
      }
    // pivots k >= U meet an identity pad (C) and zero rows (B^T): no-ops
    double pmin = 1.0;
    sweep_split<NBU, UM, 2, HL>(col, pb, pb + 2 * 256 * set, 256, l, ws, set == 0, set == 0 ? UM : 64, &pmin,
                                [](int) {});
    if constexpr (HL) {
      if (w == 0 && l == 0 && !(pmin > 0.0)) d.ip_iflag[4 * b] = 1;
    }
    __syncthreads();  // every wave is done with the pivot buffers (they share Gs' region)
    T(3);
#pragma unroll
    for (int j = 0; j < NBU; ++j)
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const int r = 4 * (ws + 2 * j) + p;
        if (r < U) {
          if (set == 0 && l < U) Cg[r * U + l] = -col[4 * j + p];
          if (set == 1 && l < X) {
            Gg[r * X + l] = col[4 * j + p];
            Gs[r * X + l] = col[4 * j + p];
          }
        }
      }
    __syncthreads();
    T(4);
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
  if (TIMING) {
    __syncthreads();
    T(5);
  }
}

// ---------------------------------------------------------------------------------
// Stage 2: the Schur chain of one problem (one 256-thread workgroup).
//
// Store S_i in the ADMM lane-tile layout (state.h): 4x4 tile t = K l + k of lane l,
// pair j at s_off + ((k * 8 + j) * 64 + l) * 2 (coalesced over o).  Threads [t0, t0 + nt).
__device__ __forceinline__ void store_tiles_range(CFac fn, const double* Sl, double* Sg, int o0, int o1, int nt) {
  double* Sn = Sg + fn->s_off;
  const int nunit = fn->nunit, ntl = fn->ntl, nw = fn->nw;
  for (int o = o0; o < o1; o += nt) {
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

__device__ __forceinline__ void store_tiles(const PlDev& d, CFac fn, const double* Sl, double* Sg, int t0, int nt,
                                            int tid) {
  (void)d;
  store_tiles_range(fn, Sl, Sg, tid - t0, fn->nunit * 64 * 16, nt);
}

template <int X, bool HL>
__global__ __launch_bounds__(NT) void k_fchain(PlDev d, int N, int m, int nnz, int S_stride, long long fs_stride,
                                               int nwm, int ny, int ncw, int fac_only, int gc, int ncm, int nxcm,
                                               int short_cw) {
  const int b = blockIdx.x;
  if (ip_skip(d, b)) return;
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
  double* sv = Acw;       // short lists: [X][4] values | [X][4] w columns (int), in the Acw region
  int* sk = reinterpret_cast<int*>(Acw + 4 * X);
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
    // ---- all waves: stage node i's coupling values (S_{i-1}, still in Sl, is stored in
    // slices interleaved with the sweep below)
    if (i < N && gc) {
      const int ncwi = (int)gcwptr[nc], nxci = (int)gxcptr[X];
      for (int q = tid; q < ncwi; q += NT) Acw[q] = Asb[gcwl[q] & 0xffff];
      for (int q = tid; q < nxci; q += NT) Axc[q] = Asb[gxcl[q] & 0xffff];
      for (int q = tid; q < nc; q += NT) rcl[q] = rhob[crow[q]];
    } else if (i < N) {
      const int ncwi = (int)cwptr[X];
      if (short_cw == 1 || short_cw == 3) {
        // per row: 4 values (0 past the list) | 4 w columns, so the E loop reads LDS only
        // (the global list words in its inner loop were a chain of dependent loads)
        for (int a = tid; a < X; a += NT) {
          const int q0 = (int)cwptr[a], q1 = (int)cwptr[a + 1];
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const bool ok = q0 + j < q1;
            const uint32_t wq = cwl[ok ? q0 + j : q0];
            sv[4 * a + j] = ok ? Asb[wq & 0xffff] : 0.0;
            sk[4 * a + j] = ok ? (int)((wq >> 16) & 0xff) : 0;
          }
        }
      } else {
        for (int q = tid; q < ncwi; q += NT) Acw[q] = Asb[cwl[q] & 0xffff];
      }
      for (int a = tid; a < X; a += NT) {
        const double ea = Asb[cent[a]];
        ev[a] = ea;
        cv[a] = rhob[crow[a]] * ea;
      }
    }
    T(7);
    {
      // ---- S_xx = (A' + E_i)^-1, one column per lane, rows over the four waves
      // (sweep_split).  The sweep runs on XS = X rounded up to 4 pivots: rows / columns
      // X..XS-1 are an identity pad (their pivots are no-ops), e.g. X = 30 for B2G
      // centroidal_vel (6 + nv).  Lanes >= XS duplicate column XS - 1: never pivot, never
      // published, never stored.
      constexpr int XS = (X + 3) & ~3;
      constexpr int NB = (XS / 4 + 3) / 4;
      double col[4 * NB];
      const int lc = min(l, XS - 1);
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int p = 0; p < 4; ++p) {
          const int r = 4 * (w + 4 * j) + p;
          const int rc = min(r, X - 1), cc = min(lc, X - 1);
          // clamped unconditional loads, arithmetic masks (a select would sink each load
          // into its own branch)
          const double v = Ag[rc * X + cc] + Eb[sidx(rc, cc)];
          col[4 * j + p] = fma(v, (r < X && lc < X) ? 1.0 : 0.0, (r == lc && !(r < X && lc < X)) ? 1.0 : 0.0);
        }
      unsigned long long ts0 = 0;
      if (TIMING) ts0 = __builtin_amdgcn_s_memtime();
      double pmin = 1.0;
      CFac fp = (CFac)d.fnodes + (i > 0 ? i - 1 : 0);
      const int stot = i > 0 ? fp->nunit * 64 * 16 : 0;
      constexpr int nblk = XS / 4;
      const int slice = ((stot + nblk - 1) / nblk + NT - 1) / NT * NT;
      sweep_split<NB, XS, 4, HL>(col, pb, pb, 8 * 64, l, w, true, XS, &pmin, [&](int B) {
        const int o0 = B * slice, o1 = min(o0 + slice, stot);
        if (o0 < o1) store_tiles_range(fp, Sl, Sg, o0 + tid, o1, NT);
      });
      if constexpr (HL) {
        if (l == 0 && !(pmin > 0.0)) d.ip_iflag[4 * b] = 1;
      }
      if (TIMING) {
        const unsigned long long ts1 = __builtin_amdgcn_s_memtime();
        if (tid == 0) tacc[5] += ts1 - ts0;
      }
      // symmetrise -col (sweep round-off) through the transpose buffer; the pivot rows of
      // the last block (pb, inside Yb) are read by every wave before the barrier
      constexpr int XP = X + 1;
      lds_barrier();  // LDS only: the tile stores issued during the sweep keep draining
      if (l < X) {
#pragma unroll
        for (int j = 0; j < NB; ++j)
#pragma unroll
          for (int p = 0; p < 4; ++p) {
            const int r = 4 * (w + 4 * j) + p;
            if (r < X) Yb[r * XP + l] = -col[4 * j + p];
          }
      }
      lds_barrier();
      for (int o = tid; o < X * X; o += NT) {
        const int r = o / X, c = o - r * X;
        if (c <= r) Sl[lidx(r, c)] = 0.5 * (Yb[r * XP + c] + Yb[c * XP + r]);
      }
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
    if (short_cw == 1 || short_cw == 3) {
      // short lists: E[a][b] = d_ab - c_a c_b sum_{q in a} A_q sum_{q' in b} A_q' S[c_q][c_q'] straight
      // from S, in the FMA order of the Y route below (the zero-padded list slots add exact 0s;
      // short_cw 3: lists of at most 2 entries, e.g. the integration rows of rnea / acc, so
      // only 2 x 2 products per entry)
      auto eshort = [&](auto lmc) __attribute__((always_inline)) {
        constexpr int LM = decltype(lmc)::value;
        for (int o = tid; o < X * X; o += NT) {
          const int a = o / X, bb = o - a * X;
          if (bb > a) continue;
          double vb[LM];
          int kb[LM];
#pragma unroll
          for (int k = 0; k < LM; ++k) {
            vb[k] = sv[4 * bb + k];
            kb[k] = sk[4 * bb + k];
          }
          double acc = 0.0;
#pragma unroll
          for (int j = 0; j < LM; ++j) {
            const int p = sk[4 * a + j];
            double y = 0.0;
#pragma unroll
            for (int k = 0; k < LM; ++k) y = fma(vb[k], Sl[sidx(p, kb[k])], y);
            acc = fma(sv[4 * a + j], y, acc);
          }
          const double ca = cv[a];
          Eb[lidx(a, bb)] = (a == bb ? ca * ev[a] : 0.0) - ca * cv[bb] * acc;
        }
      };
      if (short_cw == 3) eshort(std::integral_constant<int, 2>{});
      else eshort(std::integral_constant<int, 4>{});
      T(4);
      continue;
    }
    if (short_cw == 2) {
      // E_{i+1} = D - C (Wc S Wc^T) C on the f64 MFMA (r04): Wc (the coupling rows' w parts)
      // dense [X16][NWS] and Y = Wc S [X16][NWS] in the Y buffer (NWS = w width rounded to 16,
      // + 1 against bank conflicts); 16x16 tiles, wave w takes tiles w, w + 4, ...
      constexpr int X16 = (X + 15) & ~15;
      constexpr int MT = X16 / 16;
      const int nw = X + U;
      const int NWP = (nw + 15) & ~15, NWS = NWP + 1, NTl = NWP / 16;
      double* Wd = Yb;
      double* Yd = Yb + X16 * NWS;
      for (int o = tid; o < X16 * NWS; o += NT) Wd[o] = 0.0;
      __syncthreads();
      for (int o = tid; o < X * NWP; o += NT) {  // (row, list slot) items: independent loads
        const int a = o / NWP, j = o - a * NWP;
        const int q = (int)cwptr[a] + j;
        if (q < (int)cwptr[a + 1]) Wd[a * NWS + ((cwl[q] >> 16) & 0xff)] = Acw[q];
      }
      __syncthreads();
      T(3);
      for (int t = w; t < MT * NTl; t += 4) {  // Y = Wc S
        const int mt = t / NTl, nt = t - mt * NTl;
        const int ar = 16 * mt + (l & 15), bc = 16 * nt + (l & 15);
        f64x4 acc = {0.0, 0.0, 0.0, 0.0};
        for (int kk = 0; kk < NWP / 4; ++kk) {
          const int kc = 4 * kk + (l >> 4);
          const double bv0 = Sl[sidx(min(kc, nw - 1), min(bc, nw - 1))];
          acc = mfma4(Wd[ar * NWS + kc], bv0 * ((kc < nw && bc < nw) ? 1.0 : 0.0), acc);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) Yd[(16 * mt + (l >> 4) + 4 * r) * NWS + bc] = acc[r];
      }
      __syncthreads();
      for (int t = w; t < MT * (MT + 1) / 2; t += 4) {  // E' = Y Wc^T, lower tiles
        int mt = 0;
        while ((mt + 1) * (mt + 2) / 2 <= t) ++mt;
        const int nt = t - mt * (mt + 1) / 2;
        const int ar = 16 * mt + (l & 15), br = 16 * nt + (l & 15);
        f64x4 acc = {0.0, 0.0, 0.0, 0.0};
        for (int kk = 0; kk < NWP / 4; ++kk) {
          const int kc = 4 * kk + (l >> 4);
          acc = mfma4(Yd[ar * NWS + kc], Wd[br * NWS + kc], acc);
        }
        const int cb = 16 * nt + (l & 15);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int ra = 16 * mt + (l >> 4) + 4 * r;
          if (ra < X && cb <= ra) Eb[lidx(ra, cb)] = (ra == cb ? cv[ra] * ev[ra] : 0.0) - cv[ra] * cv[cb] * acc[r];
        }
      }
      T(4);
      continue;
    }
    // Y[pc][bb] = (S w_{s_bb})[pcl[pc]]: thread (w, l) -> bb = l, pc = w (mod 4).  The support
    // columns are taken in two halves (Y holds ceil(npc / 2) rows: the chain's LDS fits two
    // workgroups per CU); the E sums run over a coupling row's list in order, the first
    // half's entries (a prefix: pcl is sorted) in pass 0, the rest in pass 1, so every E
    // entry sees the same FMA sequence as with the whole Y.
    const int H = (npc + 1) >> 1;
    for (int h = 0; h < 2; ++h) {
      const int pc0 = h * H, pc1 = min(npc, pc0 + H);
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
        for (int pc = pc0 + w; pc < pc1; pc += 4) {
          const int p = (int)pcl[pc];
          double acc = 0.0;
#pragma unroll
          for (int j = 0; j < CR; ++j) acc = fma(av[j], Sl[sidx(p, qc[j])], acc);
          for (int q = q0 + CR; q < q1; ++q) acc = fma(Acw[q], Sl[sidx(p, (cwl[q] >> 16) & 0xff)], acc);
          Yb[(pc - pc0) * X + l] = acc;
        }
      }
      __syncthreads();
      T(3);
      if (l < X) {
        const double cb = cv[l];
        for (int a = w; a < X; a += 4) {  // lower triangle (l <= a) only: E is symmetric
          if (l > a) continue;
          double acc = h ? Eb[lidx(a, l)] : 0.0;
          for (int q = (int)cwptr[a]; q < (int)cwptr[a + 1]; ++q) {
            const int pq = (int)(cwl[q] >> 24);
            if (pq >= pc0 && pq < pc1) acc = fma(Acw[q], Yb[(pq - pc0) * X + l], acc);
          }
          if (h == 0) {
            Eb[lidx(a, l)] = acc;
          } else {
            const double ca = cv[a];
            Eb[lidx(a, l)] = (a == l ? ca * ev[a] : 0.0) - ca * cb * acc;
          }
        }
      }
      if (h == 0) __syncthreads();
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
                     h->fchain_nc, h->fchain_nxc, h->fchain_short);
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
