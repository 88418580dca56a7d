// ADMM sweeps (OSQP 0.6 osqp_solve loop body, src/osqp.c: update_xz_tilde,
// update_x, update_z, update_y), one 256-thread workgroup per problem.
//
// Per iteration the reduced KKT system K x~ = rhs is solved with the block
// factor of k_factor (S_i = explicit inverse of the Schur-complemented block):
//     forward : bt_i = rhs_i - K_{i,i-1} w_{i-1},   w_i = S_i bt_i
//     backward: x~_i = S_i (bt_i - K_{i+1,i}^T x~_{i+1})
// K_{i,i-1} = A_{c,dx_i}^T R A_{c,w_{i-1}} is applied from the sparse scaled A over
// the coupling rows c of node i-1.  The backward step of node i also finishes
// the iteration for the rows / columns of node i: z~ = A x~, relaxed z and y
// updates, x update, and the next iteration's rhs = sigma x - q + A^T (rho z - y).
//
// The kernel is a stream over the schedule p = 0 .. 2 (N+1) niter - 1 (forward
// nodes 0..N, then backward N..0, repeated).  It is HBM-bound on the factor
// blocks, so it is written as a software pipeline:
//   * S of step p+1 is loaded into registers right after the mat-vec of step p
//     (one (tile, half) unit = 16 double2 per thread), so its latency hides
//     behind the rest of step p and the gather phases of step p+1;
//   * the small operands of step p+1 (A values of the node the step gathers
//     from, rhs / bt, x, q, z, y, rho, l, u) are loaded into one of two register
//     sets just before, so the in-order vmcnt wait for them at the start of step
//     p+1 never waits for the S stream;
//   * the A values are staged into LDS at the start of the step, and the gather
//     program (u16 lists, PlAdmmNode) of the current node type is staged in LDS
//     when the type changes (a few times per sweep); node-table fields are
//     uniform scalar loads.  So no structure read waits on vmcnt.
// All reductions are in a fixed order: results are bit-identical for a problem
// regardless of the batch it runs in.
#include <algorithm>
#include <type_traits>

#include "state.h"

namespace {

constexpr int NT = 256;

struct Sreg {
  double2 t[16];
};

// Operands a step needs before its mat-vec (double-buffered across steps).
template <int ASR>
struct Small {
  double as[ASR];  // A values of the node the step gathers from (entries tid + NT k)
  double v0;       // forward: rhs_i[c]; backward: bt_i[c]
  double rhoc;     // rho of coupling row tid of the gather node
};
// Operands a backward step needs after its mat-vec (single buffer, loaded at
// the end of the previous step: waited on only after the S loads ahead of
// them have retired).
struct Late {
  double xa, qs;           // x_i[c], q_i[c]
  double z, y, rho, l, u;  // row data of node i
};

__device__ __forceinline__ int sched_node(int p, int N, bool& fwd) {
  const int k = p % (2 * (N + 1));
  fwd = k <= N;
  return fwd ? k : 2 * N + 1 - k;
}

// Unconditional (clamped) loads: with no branch around them the waitcnt pass
// keeps exact vmcnt counts, so later waits never drain the whole queue.
__device__ __forceinline__ void load_S(const double* __restrict__ Sn, int nunit, Sreg& R) {
  const int u = min((int)threadIdx.x, nunit - 1);
  const double2* p = reinterpret_cast<const double2*>(Sn);
#pragma unroll
  for (int k = 0; k < 16; ++k) R.t[k] = p[(unsigned)(k * nunit + u)];
}

// Partial products of y = S v for this thread's unit: 8 row sums of the 8x4
// sub-block against v_J, and (off-diagonal tiles) 4 column sums against v_I.
__device__ __forceinline__ void matvec_partials(const Sreg& R, int nunit, const double* v, double* dpart,
                                                double* tpart) {
  const int u = threadIdx.x;
  if (u < nunit) {
    const int t = u >> 1, h = u & 1;
    int I = (int)((sqrtf(8.0f * t + 1.0f) - 1.0f) * 0.5f);
    while (I * (I + 1) / 2 > t) --I;
    while ((I + 1) * (I + 2) / 2 <= t) ++I;
    const int J = t - I * (I + 1) / 2;
    double vj[4], vi[8];
#pragma unroll
    for (int c = 0; c < 4; ++c) vj[c] = v[8 * J + 4 * h + c];
#pragma unroll
    for (int r = 0; r < 8; ++r) vi[r] = v[8 * I + r];
    double tp[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const double e0 = R.t[2 * r].x, e1 = R.t[2 * r].y, e2 = R.t[2 * r + 1].x, e3 = R.t[2 * r + 1].y;
      dpart[u * 8 + r] = e0 * vj[0] + e1 * vj[1] + e2 * vj[2] + e3 * vj[3];
      tp[0] += e0 * vi[r];
      tp[1] += e1 * vi[r];
      tp[2] += e2 * vi[r];
      tp[3] += e3 * vi[r];
    }
#pragma unroll
    for (int c = 0; c < 4; ++c) tpart[u * 4 + c] = (I != J) ? tp[c] : 0.0;
  }
}

__device__ __forceinline__ double matvec_reduce(int o, int ntile, const double* dpart, const double* tpart) {
  // fixed trip counts (ntile <= 14) so all LDS reads issue before the adds
  const int I = o >> 3, r = o & 7;
  const int t0 = I * (I + 1) / 2;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
#pragma unroll
  for (int J = 0; J < 14; ++J)
    if (J <= I) {
      a0 += dpart[(2 * (t0 + J)) * 8 + r];
      a1 += dpart[(2 * (t0 + J) + 1) * 8 + r];
    }
#pragma unroll
  for (int k = 1; k < 14; ++k) {
    const int Ip = I + k;
    if (Ip < ntile) a2 += tpart[(2 * (Ip * (Ip + 1) / 2 + I) + (r >> 2)) * 4 + (r & 3)];
  }
  return (a0 + a1) + a2;
}

struct LdsMap {
  int v, cpl, row, unit, ent;  // capacities (doubles); v >= nw_max + ndx
  int prog_len;                // LDS gather-program buffer (u16), the longest node program
  int chunk;                   // chunk partial sums
  __host__ __device__ size_t total() const {
    return (4 * (size_t)v + cpl + row + 12 * (size_t)unit + ent + chunk) * sizeof(double) + 2 * (size_t)prog_len;
  }
};

}  // namespace

template <int ASR, bool TIMING>
__global__ __launch_bounds__(256, 2) void k_admm(PlDev d, int N, int n, int m, int nnz, int ndx, int S_stride, LdsMap lm,
                                                 int niter, int check, double sigma, double alpha) {
  // optional phase timing (s_memtime, thread 0): [fwd: 6 phases][bwd: 8 phases]
  __shared__ unsigned long long tacc[TIMING ? 17 : 1];
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
  const int b = blockIdx.x;
  PlProbInfo* info = d.info + b;
  if (info->done) return;
  extern __shared__ double lds[];
  double* v = lds;          // mat-vec input, zero padded to 8 * ntile
  double* y = v + lm.v;     // mat-vec output; backward: [x~_i | x~_{i+1}(dx)]
  double* xn = y + lm.v;    // x~_{i+1} (dx part) across backward steps
  double* tcpl = xn + lm.v;
  double* trow = tcpl + lm.cpl;
  double* dpart = trow + lm.row;
  double* tpart = dpart + 8 * lm.unit;
  double* asb = tpart + 4 * lm.unit;
  double* v0fix = asb + lm.ent;  // rhs_0 handed from backward node 0 to forward node 0
  double* part = v0fix + lm.v;   // chunk partial sums
  uint16_t* lprog = reinterpret_cast<uint16_t*>(part + lm.chunk);

  const double* __restrict__ As = d.As + (size_t)b * nnz;
  const double* __restrict__ rho = d.rho + (size_t)b * m;
  const double* __restrict__ rhoc = d.rhoc + (size_t)b * (N + 1) * lm.cpl;
  const double* __restrict__ ls = d.ls + (size_t)b * m;
  const double* __restrict__ us = d.us + (size_t)b * m;
  const double* __restrict__ qs = d.qs + (size_t)b * n;
  const double* __restrict__ Sg = d.S + (size_t)b * S_stride;
  double* za = d.za + (size_t)b * m;
  double* ya = d.ya + (size_t)b * m;
  double* xa = d.xa + (size_t)b * n;
  double* rhs = d.rhs + (size_t)b * n;
  double* bt = d.bt + (size_t)b * n;
  double* dxs = d.dxs + (size_t)b * n;
  double* dys = d.dys + (size_t)b * m;
  // Node table: uniform reads through the constant address space are scalar
  // loads (lgkmcnt), which cannot drain the S stream.
  typedef const __attribute__((address_space(4))) PlAdmmNode* CNode;  // constant AS -> s_load
  CNode an = (CNode)d.anodes;
  const uint16_t* __restrict__ prog = d.aprog;
  const int tid = threadIdx.x;
  const int P = niter * 2 * (N + 1);

  int cur_prog = -1;
  // make node `i`'s gather program the one in LDS (synchronous; only when the
  // node type changes, a few times per sweep)
  auto use_prog = [&](int i) {
    const int pr = an[i].prog, len = an[i].prog_len;
    if (pr == cur_prog) return;
    __syncthreads();
    const uint32_t* src = reinterpret_cast<const uint32_t*>(prog + pr);
    uint32_t* dst = reinterpret_cast<uint32_t*>(lprog);
    for (int k = tid; k < (len >> 1); k += NT) dst[k] = src[k];
    cur_prog = pr;
    __syncthreads();
  };

  Sreg S;
  Small<ASR> QA, QB;
  double rhs_keep = 0.0;  // rhs of the dx part of node i+1 (thread c < ndx), completed at node i

  // Loads of step p's small operands.  No load here depends on another vector
  // load, so nothing waits before the S stream behind them is issued.
  auto prefetch_small = [&](int p, Small<ASR>& Q) {
    if (p >= P) return;
    bool f;
    const int i = sched_node(p, N, f);
    const int ia = f ? i - 1 : i;
    const int ia_c = ia >= 0 ? ia : 0;
    const int ne = an[ia_c].nent, eo = an[ia_c].ent_off, nc = an[ia_c].ncpl;
    const int xo = an[i].x_off, nw = an[i].nw;
    // clamped, unconditional loads (allocations are padded past the end)
    const int nemax = max(ne - 1, 0);
#pragma unroll
    for (int k = 0; k < ASR; ++k) Q.as[k] = As[eo + min(tid + NT * k, nemax)];
    Q.rhoc = rhoc[ia_c * lm.cpl + min(tid, lm.cpl - 1)];
    const double* vsrc = f ? rhs : bt;
    Q.v0 = vsrc[xo + min(tid, nw - 1)];
  };
  Late LT;
  auto prefetch_late = [&](int p) {
    if (p >= P) return;
    bool f;
    const int i = sched_node(p, N, f);
    const int xo = an[i].x_off, nw = an[i].nw, nrow = an[i].nrow, ro = an[i].row_off;
    if (f) return;
    const int j = xo + min(tid, nw - 1);
    LT.xa = xa[j];
    LT.qs = qs[j];
    const int r = ro + min(tid, max(nrow - 1, 0));
    LT.z = za[r];
    LT.y = ya[r];
    LT.rho = rho[r];
    LT.l = ls[r];
    LT.u = us[r];
  };
  auto prefetch_S = [&](int p) {
    if (p >= P) return;
    bool f;
    const int i = sched_node(p, N, f);
    const int so = an[i].s_off, nu = an[i].nunit;
    load_S(Sg + so, nu, S);
  };

  auto step = [&](auto bufsel, int p) {
    constexpr bool odd = decltype(bufsel)::value;
    Small<ASR>& Q = odd ? QB : QA;
    Small<ASR>& Qn = odd ? QA : QB;
    bool fwd;
    const int i = sched_node(p, N, fwd);
    const int nw = an[i].nw, ntile = an[i].ntile, nunit = an[i].nunit, x_off = an[i].x_off;
    const int ia = fwd ? i - 1 : i;
    const int ia_c = ia >= 0 ? ia : 0;
    const int ne = an[ia_c].nent, eo = an[ia_c].ent_off;
    // all node fields are read here, in uniform control flow (scalar loads)
    const int g = ia_c;
    const int g_ncpl = an[g].ncpl, g_cwptr = an[g].cwptr, g_cwp = an[g].cwp, g_xcptr = an[g].xcptr,
              g_xcp = an[g].xcp, g_cxptr = an[g].cxptr, g_cxp = an[g].cxp, g_ccptr = an[g].ccptr,
              g_ccp = an[g].ccp, g_rowptr = an[g].rowptr, g_rowp = an[g].rowp, g_colptr = an[g].colptr,
              g_colr = an[g].colr, g_nrow = an[g].nrow, g_row_off = an[g].row_off, g_rchn = an[g].rchn,
              g_rch = an[g].rch, g_rchptr = an[g].rchptr, g_cchn = an[g].cchn, g_cch = an[g].cch,
              g_cchptr = an[g].cchptr;
    const int x_next = (!fwd && i < N) ? an[i + 1].x_off : 0;
    const uint16_t* pg = lprog;
    T(-1);
    __syncthreads();  // previous step done with asb / trow / tcpl / v / y
    T(fwd ? 0 : 8);
    if (ia >= 0) {
      use_prog(ia);
      // A values of node ia into LDS: the first NT * ASR from registers, the
      // rest (nodes larger than the dominant type) straight from HBM
#pragma unroll
      for (int k = 0; k < ASR; ++k) {
        const int idx = tid + NT * k;
        if (idx < ne) asb[idx] = Q.as[k];
      }
      for (int idx = tid + NT * ASR; idx < ne; idx += NT) asb[idx] = As[eo + idx];
    }
    T(fwd ? 1 : 9);
    // ---------------- gathers before the mat-vec: v = bt_i (fwd) / bt_i - K_{i+1,i}^T x~_{i+1} (bwd)
    if (fwd) {
      if (i > 0) {
        const uint32_t* cw = reinterpret_cast<const uint32_t*>(pg + g_cwp);
        __syncthreads();
        if (tid < g_ncpl) {  // t_s = rho_s a_s(w_{i-1}) . w_{i-1}
          double acc = 0.0;
          const int q0 = pg[g_cwptr + tid], q1 = pg[g_cwptr + tid + 1];
#pragma unroll 4
          for (int q = q0; q < q1; ++q) {
            const uint32_t w = cw[q];
            acc += asb[w & 0xffff] * y[w >> 16];
          }
          tcpl[tid] = Q.rhoc * acc;
        }
        __syncthreads();
      }
      if (tid < nw) {  // bt_i = rhs_i - A_{c,dx_i}^T t
        double vv = i == 0 ? v0fix[tid] : Q.v0;
        if (i > 0 && tid < ndx) {
          const uint32_t* xc = reinterpret_cast<const uint32_t*>(pg + g_xcp);
          double acc = 0.0;
          const int q0 = pg[g_xcptr + tid], q1 = pg[g_xcptr + tid + 1];
#pragma unroll 4
          for (int q = q0; q < q1; ++q) {
            const uint32_t w = xc[q];
            acc += asb[w & 0xffff] * tcpl[w >> 16];
          }
          vv -= acc;
        }
        bt[x_off + tid] = vv;
        v[tid] = vv;
      } else if (tid < 8 * ntile) {
        v[tid] = 0.0;
      }
    } else {
      __syncthreads();
      if (i < N && tid < g_ncpl) {  // t_s = rho_s a_s(dx_{i+1}) . x~_{i+1}
        const uint32_t* cx = reinterpret_cast<const uint32_t*>(pg + g_cxp);
        double acc = 0.0;
        const int q0 = pg[g_cxptr + tid], q1 = pg[g_cxptr + tid + 1];
#pragma unroll 4
        for (int q = q0; q < q1; ++q) {
          const uint32_t w = cx[q];
          acc += asb[w & 0xffff] * xn[w >> 16];
        }
        tcpl[tid] = Q.rhoc * acc;
      }
      __syncthreads();
      if (tid < nw) {  // bt_i - A_{c,w_i}^T t
        double vv = Q.v0;
        if (i < N) {
          const uint32_t* cc = reinterpret_cast<const uint32_t*>(pg + g_ccp);
          double acc = 0.0;
          const int q0 = pg[g_ccptr + tid], q1 = pg[g_ccptr + tid + 1];
#pragma unroll 4
          for (int q = q0; q < q1; ++q) {
            const uint32_t w = cc[q];
            acc += asb[w & 0xffff] * tcpl[w >> 16];
          }
          vv -= acc;
        }
        v[tid] = vv;
      } else if (tid < 8 * ntile) {
        v[tid] = 0.0;
      }
    }
    __syncthreads();
    T(fwd ? 2 : 10);
    // ---------------- mat-vec with S_i, then issue the next step's operands
    matvec_partials(S, nunit, v, dpart, tpart);
    __syncthreads();
    T(fwd ? 3 : 11);
    prefetch_small(p + 1, Qn);
    __builtin_amdgcn_sched_barrier(0);
    prefetch_S(p + 1);
    T(fwd ? 4 : 12);
    if (tid < nw) y[tid] = matvec_reduce(tid, ntile, dpart, tpart);  // w_i / x~_i
    else if (!fwd && tid < nw + ndx && i < N) y[tid] = xn[tid - nw];  // x~_{i+1} (dx) behind x~_i
    T(fwd ? 5 : -1);
    if (!fwd) {
      // ---------------- backward: finish the iteration for the rows / columns of node i
      __syncthreads();
      T(13);
      const bool store_delta = check && (p >= P - (N + 1));
      // z~ = A x~ over balanced chunks of <= PL_CHUNK entries, one chunk per thread
      {
        const uint32_t* rw = reinterpret_cast<const uint32_t*>(pg + g_rowp);
        const uint32_t* rch = reinterpret_cast<const uint32_t*>(pg + g_rch);
        for (int t = tid; t < g_rchn; t += NT) {
          const uint32_t c = rch[t];
          const int q0 = c & 0xffff, len = (int)(c >> 16) - q0;
          double acc = 0.0;
#pragma unroll
          for (int k = 0; k < PL_CHUNK; ++k)
            if (k < len) {
              const uint32_t w = rw[q0 + k];
              acc += asb[w & 0xffff] * y[w >> 16];
            }
          part[t] = acc;
        }
      }
      __syncthreads();
      if (tid < g_nrow) {  // update_z, update_y (relaxed)
        const int k0 = pg[g_rchptr + tid], k1 = pg[g_rchptr + tid + 1];
        double zt = 0.0;
#pragma unroll 4
        for (int k = k0; k < k1; ++k) zt += part[k];
        const double zrel = alpha * zt + (1.0 - alpha) * LT.z;
        double zn = zrel + (1.0 / LT.rho) * LT.y;
        zn = fmin(fmax(zn, LT.l), LT.u);
        const double dy = LT.rho * (zrel - zn);
        const double yn = LT.y + dy;
        const int r = g_row_off + tid;
        za[r] = zn;
        ya[r] = yn;
        if (store_delta) dys[r] = dy;
        trow[tid] = LT.rho * zn - yn;
      }
      __syncthreads();
      T(14);
      // A^T (rho z - y) over column chunks
      if (i < N) {
        const uint16_t* colr = pg + g_colr;
        const uint32_t* cch = reinterpret_cast<const uint32_t*>(pg + g_cch);
        for (int t = tid; t < g_cchn; t += NT) {
          const uint32_t c = cch[t];
          const int e0 = c & 0xffff, len = (int)(c >> 16) - e0;
          double acc = 0.0;
#pragma unroll
          for (int k = 0; k < PL_CHUNK; ++k)
            if (k < len) acc += asb[e0 + k] * trow[colr[e0 + k]];
          part[t] = acc;
        }
        __syncthreads();
      }
      if (tid < nw) {  // update_x and next rhs = sigma x - q + A^T (rho z - y)
        const int j = x_off + tid;
        const double xnew = alpha * y[tid] + (1.0 - alpha) * LT.xa;
        xa[j] = xnew;
        if (store_delta) dxs[j] = xnew - LT.xa;
        double acc = sigma * xnew - LT.qs;
        if (i < N) {
          const int k0 = pg[g_cchptr + tid], k1 = pg[g_cchptr + tid + 1];
#pragma unroll 4
          for (int k = k0; k < k1; ++k) acc += part[k];
          if (tid < ndx) {  // rows of node i on dx_{i+1} complete rhs_{i+1}
            double a2 = 0.0;
            const int f0 = pg[g_cchptr + nw + tid], f1 = pg[g_cchptr + nw + tid + 1];
#pragma unroll 4
            for (int k = f0; k < f1; ++k) a2 += part[k];
            rhs[x_next + tid] = rhs_keep + a2;
          }
        }
        if (tid < ndx && i > 0) rhs_keep = acc;
        else rhs[j] = acc;
        // forward node 0 of the next iteration prefetched rhs_0 before it was written here
        if (i == 0) v0fix[tid] = acc;
        if (tid < ndx) xn[tid] = y[tid];
      }
      T(15);
    }
    prefetch_late(p + 1);
  };

  if (tid < an[0].nw) v0fix[tid] = rhs[tid];  // rhs_0 (node 0 starts at x_off 0)
  prefetch_small(0, QA);
  __builtin_amdgcn_sched_barrier(0);
  prefetch_S(0);
  for (int p = 0; p < P; p += 2) {
    step(std::integral_constant<bool, false>(), p);
    if (p + 1 < P) step(std::integral_constant<bool, true>(), p + 1);
  }
  if (tid == 0) info->iter += niter;
  if constexpr (TIMING) {
    if (tid == 0 && d.dbg)
      for (int k = 0; k < 16; ++k) d.dbg[(size_t)b * 16 + k] += (double)tacc[k];
  }
}

namespace {
template <int ASR, bool TIMING>
void launch_admm_t(PlOcpHandle* h, int niter, int check, size_t lds, const LdsMap& lm) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)k_admm<ASR, TIMING>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((k_admm<ASR, TIMING>), dim3(h->B), dim3(256), lds, h->stream, h->d, h->N, h->n, h->m, h->nnz,
                     h->ndx, h->S_stride, lm, niter, check, h->set.sigma, h->set.alpha);
}
}  // namespace

static LdsMap admm_lds_map(const PlOcpHandle* h) {
  return LdsMap{((h->nw_max + h->ndx + 7) / 8) * 8, std::max(h->ncpl_max, 1), std::max(h->nrow_max, 1), h->nunit_max,
                std::max(h->nent_max, 1), h->admm_dom_len, h->chunk_max};
}

int admm_lds_bytes(const PlOcpHandle* h) { return (int)admm_lds_map(h).total(); }

void launch_admm(PlOcpHandle* h, int niter, int check, int it_base) {
  (void)it_base;
  const LdsMap lm = admm_lds_map(h);
  const size_t lds = lm.total();
  const bool prof = h->profile && h->prof_n < 64;
  if (prof) hipEventRecord(h->prof_ev[h->prof_n][0], h->stream);
  if (h->d.dbg && h->admm_asr <= 4) launch_admm_t<4, true>(h, niter, check, lds, lm);
  else if (h->admm_asr <= 4) launch_admm_t<4, false>(h, niter, check, lds, lm);
  else if (h->admm_asr <= 6) launch_admm_t<6, false>(h, niter, check, lds, lm);
  else launch_admm_t<8, false>(h, niter, check, lds, lm);
  if (prof) {
    hipEventRecord(h->prof_ev[h->prof_n][1], h->stream);
    h->prof_n++;
    h->prof_admm_iters += (long long)h->B * niter;
  }
}
