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

typedef const __attribute__((address_space(4))) PlFacNode* CFac;
typedef const __attribute__((address_space(4))) uint32_t* CU32;
typedef const __attribute__((address_space(4))) double* CF64;

}  // namespace

// ---------------------------------------------------------------------------------
// Stage 1: per (problem, node).  X = ndx, UM >= nu (register columns of the sweep).
template <int X, int UM>
__global__ __launch_bounds__(NT) void k_fnode(PlDev d, int n, int m, int nnz, int i0, int ni, long long fs_stride,
                                              double sigma) {
  const int task = blockIdx.x;
  const int b = task / ni;
  const int i = i0 + (task - b * ni);
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  CFac fn = (CFac)d.fnodes + i;
  const int nw = fn->nw, U = fn->nu, nent = fn->nent;
  const int nK = (nw * (nw + 1) / 2 + 1) & ~1;
  const int r2 = (max(2 * (nent + 1), U * X) + 1) & ~1;
  extern __shared__ double lds[];
  double* K = lds;         // packed lower Kt_ii
  double* Ar = K + nK;     // rho-scaled A values (nent + 1, the last one zero)
  double* Av = Ar + nent + 1;
  double* Gs = K + nK;     // after the sweep: G (U x X), row-major
  double* pb = K + nK + r2;

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
      for (int r = 0; r < UM; ++r) col[r] = (r < U && l < U) ? K[sidx(X + r, X + l)] : (r == l ? 1.0 : 0.0);
    } else if (w == 1) {
#pragma unroll
      for (int r = 0; r < UM; ++r) col[r] = (r < U && l < X) ? K[lidx(X + r, l)] : 0.0;
    }
    // pivots k >= U meet an identity pad (wave 0) and zero rows (wave 1): no-ops
    static_for<0, UM>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      double* pk = pb + (k & 1) * 64;
      if (w == 0) pk[l] = col[k];
      __syncthreads();
      if (w < 2) {
        const double pinv = 1.0 / pk[k];
        const double f = col[k];
        const bool piv = (w == 0 && l == k);
        const double g = piv ? 1.0 - pinv : f * pinv;
#pragma unroll
        for (int r = 0; r < UM; ++r)
          if (r != k) col[r] = fma(-pk[r], g, col[r]);
        col[k] = piv ? -pinv : f * pinv;
      }
    });
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
  // ---- A' = A - B G (lower, written to both triangles)
  if (l < X) {
    for (int r = w; r < X; r += 4) {
      if (r < l) continue;
      double acc = K[lidx(r, l)];
      for (int u = 0; u < U; ++u) acc = fma(-K[lidx(X + u, r)], Gs[u * X + l], acc);
      Ag[r * X + l] = acc;
      Ag[l * X + r] = acc;
    }
  }
}

// ---------------------------------------------------------------------------------
// Stage 2: the Schur chain of one problem (one 256-thread workgroup).
//
// Store S_i in the ADMM lane-tile layout (state.h): 4x4 tile t = K l + k of lane l,
// pair j at s_off + ((k * 8 + j) * 64 + l) * 2 (coalesced over o).  Threads [t0, t0 + nt).
__device__ __forceinline__ void store_tiles(const PlDev& d, CFac fn, const double* Sl, double* Sg, int t0, int nt) {
  double* Sn = Sg + fn->s_off;
  const int nunit = fn->nunit, ntl = fn->ntl, nw = fn->nw;
  const int tt = fn->ttab;
  const int total = nunit * 64 * 16;
  for (int o = (int)threadIdx.x - t0; o < total; o += nt) {
    const int slot = o & 1, ln = (o >> 1) & 63, j = (o >> 7) & 7, k = o >> 10;
    const int t = nunit * ln + k;
    double val = 0.0;
    if (t < ntl) {
      int I, J;
      if (tt >= 0) {
        const uint32_t e = d.ttab[tt + ln * PL_ADMM_KM + k];
        I = (int)(e >> 24);
        J = (int)((e >> 16) & 0xff);
      } else {
        I = (int)((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
        while (I * (I + 1) / 2 > t) --I;
        while ((I + 1) * (I + 2) / 2 <= t) ++I;
        J = t - I * (I + 1) / 2;
      }
      const int gi = 4 * I + (j >> 1), gj = 4 * J + 2 * (j & 1) + slot;
      if (gi < nw && gj < nw) val = Sl[sidx(gi, gj)];
    }
    Sn[o] = val;
  }
}

template <int X, bool TIMING>
__global__ __launch_bounds__(NT) void k_fchain(PlDev d, int N, int m, int nnz, int S_stride, long long fs_stride,
                                               int nwm, int ny, int ncw, int gsz) {
  const int b = blockIdx.x;
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  extern __shared__ double lds[];
  const int nS = (nwm * (nwm + 1) / 2 + 1) & ~1;
  double* Sl = lds;       // packed lower S_i
  double* Yb = Sl + nS;   // transpose buffer [X][X + 1], then Y [npc][X]
  double* Eb = Yb + ny;   // E_i [X][X]
  double* pb = Eb + X * X;  // pivot rows [2][64]
  double* Acw = pb + 128;   // A values of the coupling rows' w parts (ncw)
  double* cv = Acw + ncw;   // rho_a A_{e_a} (X)
  double* ev = cv + X;      // A_{e_a} (X)
  double* Gs = ev + X;      // G (U x X), staged
  double* Cs = Gs + gsz;    // C^-1, packed lower, staged
  unsigned long long tacc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long tlast = 0;
  auto T = [&](int slot) {
    if constexpr (TIMING) {
      if (tid == 0) {
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        if (slot >= 0) tacc[slot] += now - tlast;
        tlast = now;
      }
    }
  };
  for (int k = tid; k < X * X; k += NT) Eb[k] = 0.0;
  double* Sg = d.S + (size_t)b * S_stride;
  const double* __restrict__ FSb = d.FS + (size_t)b * fs_stride;
  for (int i = 0; i <= N; ++i) {
    CFac fn = (CFac)d.fnodes + i;
    const int U = fn->nu;
    const double* __restrict__ Ag = FSb + fn->fs_off;
    const double* __restrict__ Cg = Ag + X * X + U * X;
    CU32 cp = (CU32)d.kcpl + fn->cp_off;
    CU32 crow = cp;
    CU32 cent = cp + X;
    CU32 cwptr = cp + 2 * X;
    CU32 pcl = cp + 3 * X + 1;
    const int npc = fn->npc;
    CU32 cwl = pcl + npc;
    const double* __restrict__ Asb = d.As + (size_t)b * nnz + fn->ent_off;
    const double* __restrict__ rhob = d.rho + (size_t)b * m + fn->row_off;
    __syncthreads();
    T(-1);
    if (w == 0) {
      // ---- S_xx = (A' + E_i)^-1, one column per lane (identity past X)
      double col[X];
#pragma unroll
      for (int r = 0; r < X; ++r)
        col[r] = l < X ? Ag[r * X + l] + Eb[r >= l ? r * X + l : l * X + r] : (r == l ? 1.0 : 0.0);
      static_for<0, X>([&](auto kc) {
        constexpr int k = decltype(kc)::value;
        double* pk = pb + (k & 1) * 64;
        pk[l] = col[k];
        wsync();
        const double2* pk2 = reinterpret_cast<const double2*>(pk);
        double c[X];
#pragma unroll
        for (int r = 0; r < X / 2; ++r) {
          const double2 v = pk2[r];
          c[2 * r] = v.x;
          c[2 * r + 1] = v.y;
        }
        const double pinv = rcp_nr(c[k]);
        const double f = col[k];
        const bool piv = (l == k);
        const double g = piv ? 1.0 - pinv : f * pinv;
#pragma unroll
        for (int r = 0; r < X; ++r)
          if (r != k) col[r] = fma(-c[r], g, col[r]);
        col[k] = piv ? -pinv : f * pinv;
      });
      // symmetrise -col (sweep round-off) through the transpose buffer
      constexpr int XP = X + 1;
      if (l < X) {
#pragma unroll
        for (int r = 0; r < X; ++r) Yb[r * XP + l] = -col[r];
      }
      wsync();
#pragma unroll
      for (int r = 0; r < X; ++r) col[r] = 0.5 * (Yb[l * XP + r] - col[r]);
      __syncthreads();  // (a) the other waves are done with Sl (tile store of S_{i-1})
      if (l < X) {
#pragma unroll
        for (int r = 0; r < X; ++r)
          if (r >= l) Sl[lidx(r, l)] = col[r];
      }
    } else {
      // ---- waves 1-3, while wave 0 sweeps: store S_{i-1}, stage node i's coupling values
      for (int k = tid - 64; k < U * X; k += NT - 64) Gs[k] = Ag[X * X + k];
      for (int k = tid - 64; k < U * U; k += NT - 64) {
        const int u = k / U, j = k - u * U;
        if (u >= j) Cs[lidx(u, j)] = Cg[k];
      }
      if (i > 0) store_tiles(d, (CFac)d.fnodes + (i - 1), Sl, Sg, 64, NT - 64);
      if (i < N) {
        const int ncwi = (int)cwptr[X];
        for (int q = tid - 64; q < ncwi; q += NT - 64) Acw[q] = Asb[cwl[q] & 0xffff];
        for (int a = tid - 64; a < X; a += NT - 64) {
          const double ea = Asb[cent[a]];
          ev[a] = ea;
          cv[a] = rhob[crow[a]] * ea;
        }
      }
      __syncthreads();  // (a)
    }
    __syncthreads();
    T(0);
    // ---- S_ux = -G S_xx: thread (w, l) -> column l, rows u = w (mod 4); four partial
    // sums over r (mod 4) keep the FMA chains short
    if (l < X && U > 0) {
      double sx[X];
#pragma unroll
      for (int r = 0; r < X; ++r) sx[r] = Sl[sidx(r, l)];
      for (int u = w; u < U; u += 4) {
        const double2* gr = reinterpret_cast<const double2*>(Gs + u * X);
        double a[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int r = 0; r < X / 2; ++r) {
          const double2 g = gr[r];
          a[(2 * r) & 3] = fma(g.x, sx[2 * r], a[(2 * r) & 3]);
          a[(2 * r + 1) & 3] = fma(g.y, sx[2 * r + 1], a[(2 * r + 1) & 3]);
        }
        Sl[lidx(X + u, l)] = -((a[0] + a[1]) + (a[2] + a[3]));
      }
    }
    __syncthreads();
    T(1);
    // ---- S_uu = C^-1 - G S_ux^T (lower): thread (w, l) -> column l, rows u >= l, u = w (mod 4)
    if (l < U) {
      double wv[X];
#pragma unroll
      for (int r = 0; r < X; ++r) wv[r] = Sl[lidx(X + l, r)];
      for (int u = w; u < U; u += 4) {
        if (u < l) continue;
        const double2* gr = reinterpret_cast<const double2*>(Gs + u * X);
        double a[4] = {Cs[lidx(u, l)], 0.0, 0.0, 0.0};
#pragma unroll
        for (int r = 0; r < X / 2; ++r) {
          const double2 g = gr[r];
          a[(2 * r) & 3] = fma(-g.x, wv[2 * r], a[(2 * r) & 3]);
          a[(2 * r + 1) & 3] = fma(-g.y, wv[2 * r + 1], a[(2 * r + 1) & 3]);
        }
        Sl[lidx(X + u, X + l)] = (a[0] + a[1]) + (a[2] + a[3]);
      }
    }
    __syncthreads();
    T(2);
    if (i == N) break;
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
      for (int a = w; a < X; a += 4) {
        const double ca = cv[a];
        double acc = 0.0;
        for (int q = (int)cwptr[a]; q < (int)cwptr[a + 1]; ++q)
          acc = fma(Acw[q], Yb[(cwl[q] >> 24) * X + l], acc);
        Eb[a * X + l] = (a == l ? ca * ev[a] : 0.0) - ca * cb * acc;
      }
    }
    T(4);
  }
  store_tiles(d, (CFac)d.fnodes + N, Sl, Sg, 0, NT);
  T(5);
  if constexpr (TIMING) {
    if (tid == 0 && d.dbg)
      for (int k = 0; k < 6; ++k) d.dbg[(size_t)b * 16 + 16 * (size_t)gridDim.x + k] = (double)tacc[k];
  }
}

namespace {

template <int X, int UM>
void launch_fnode(PlOcpHandle* h, int g) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)k_fnode<X, UM>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((k_fnode<X, UM>), dim3(h->B * h->fg_n[g]), dim3(NT), h->fg_lds[g], h->stream, h->d, h->n, h->m,
                     h->nnz, h->fg_i0[g], h->fg_n[g], h->fs_stride, h->set.sigma);
}

template <int X>
void launch_fchain(PlOcpHandle* h) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)k_fchain<X, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)k_fchain<X, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const int nS = (h->nw_max * (h->nw_max + 1) / 2 + 1) & ~1;
  const int ny = h->fchain_ny;
  const int ncw = h->fchain_ncw;
  const int gsz = h->fchain_gsz;
  if (h->d.dbg)
    hipLaunchKernelGGL((k_fchain<X, true>), dim3(h->B), dim3(NT), h->fchain_lds, h->stream, h->d, h->N, h->m, h->nnz,
                       h->S_stride, h->fs_stride, h->nw_max, ny, ncw, gsz);
  else
    hipLaunchKernelGGL((k_fchain<X, false>), dim3(h->B), dim3(NT), h->fchain_lds, h->stream, h->d, h->N, h->m, h->nnz,
                       h->S_stride, h->fs_stride, h->nw_max, ny, ncw, gsz);
}

template <int X>
void launch_factor_x(PlOcpHandle* h) {
  for (int g = 0; g < h->nfgroup; ++g) {
    if (h->fg_um[g] <= 40) launch_fnode<X, 40>(h, g);
    else launch_fnode<X, 64>(h, g);
  }
  launch_fchain<X>(h);
}

}  // namespace

// ndx values of the shipped whole-body models: 36 (Go2 / B2), 48 (B2G); the handle
// refuses others.
bool factor_supports_ndx(int ndx) { return ndx == 36 || ndx == 48; }

void launch_factor(PlOcpHandle* h) {
  switch (h->ndx) {
    case 36: launch_factor_x<36>(h); break;
    case 48: launch_factor_x<48>(h); break;
    default: break;
  }
}
