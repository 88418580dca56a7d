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
//   * the A values are staged into LDS at the start of the step; the node table
//     lives in LDS for the launch and the gather program (u16 lists, PlAdmmNode)
//     of the current node type is staged in LDS when the type changes (a few
//     times per sweep), so structure reads never wait on vmcnt.
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

template <int ASR>
struct Small {
  double as[ASR];  // A values of the node the step gathers from (entries tid + NT k)
  double v0;       // forward: rhs_i[c]; backward: bt_i[c]
  double xa, qs;   // backward: x_i[c], q_i[c]
  double z, y, rho, l, u;  // backward: row data of node i
  double rhoc;     // rho of coupling row tid of the gather node
};

__device__ __forceinline__ int sched_node(int p, int N, bool& fwd) {
  const int k = p % (2 * (N + 1));
  fwd = k <= N;
  return fwd ? k : 2 * N + 1 - k;
}

__device__ __forceinline__ void load_S(const double* __restrict__ Sn, int nunit, Sreg& R) {
  const int u = threadIdx.x;
  if (u < nunit) {
    const double2* p = reinterpret_cast<const double2*>(Sn);
#pragma unroll
    for (int k = 0; k < 16; ++k) R.t[k] = p[(unsigned)(k * nunit + u)];
  }
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
  const int I = o >> 3, r = o & 7;
  double acc = 0.0;
  for (int J = 0; J <= I; ++J) {
    const int t = I * (I + 1) / 2 + J;
    acc += dpart[(2 * t) * 8 + r] + dpart[(2 * t + 1) * 8 + r];
  }
  for (int Ip = I + 1; Ip < ntile; ++Ip) {
    const int t = Ip * (Ip + 1) / 2 + I;
    acc += tpart[(2 * t + (r >> 2)) * 4 + (r & 3)];
  }
  return acc;
}

struct LdsMap {
  int v, cpl, row, unit, ent;  // capacities (doubles)
  int dom_prog, dom_len;       // unused / LDS program buffer length (longest node program, u16)
  int nodes;                   // N + 1 (LDS copy of the node table)
  __host__ __device__ size_t total() const {
    return (3 * (size_t)v + cpl + row + 12 * (size_t)unit + ent) * sizeof(double) + (size_t)nodes * sizeof(PlAdmmNode) +
           2 * (size_t)dom_len;
  }
};

}  // namespace

#define UF(x) __builtin_amdgcn_readfirstlane(x)

template <int ASR>
__global__ __launch_bounds__(256, 2) void k_admm(PlDev d, int N, int n, int m, int nnz, int ndx, int S_stride, LdsMap lm,
                                                 int niter, int check, double sigma, double alpha) {
  const int b = blockIdx.x;
  PlProbInfo* info = d.info + b;
  if (info->done) return;
  extern __shared__ double lds[];
  double* v = lds;
  double* y = v + lm.v;
  double* xn = y + lm.v;
  double* tcpl = xn + lm.v;
  double* trow = tcpl + lm.cpl;
  double* dpart = trow + lm.row;
  double* tpart = dpart + 8 * lm.unit;
  double* asb = tpart + 4 * lm.unit;
  PlAdmmNode* an = reinterpret_cast<PlAdmmNode*>(asb + lm.ent);
  uint16_t* lprog = reinterpret_cast<uint16_t*>(an + (N + 1));

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
  const uint16_t* __restrict__ prog = d.aprog;
  const int tid = threadIdx.x;
  const int P = niter * 2 * (N + 1);

  // The node table lives in LDS for the whole launch and the current node
  // type's gather program is staged in LDS, so structure reads inside the
  // pipeline are ds_reads (lgkmcnt) and never drain the outstanding S loads
  // (vmcnt retires in order).  Node fields are made wave-uniform (SGPRs).
  {
    const int* src = reinterpret_cast<const int*>(d.anodes);
    int* dst = reinterpret_cast<int*>(an);
    const int words = (N + 1) * (int)(sizeof(PlAdmmNode) / sizeof(int));
    for (int k = tid; k < words; k += NT) dst[k] = src[k];
  }
  __syncthreads();
  int cur_prog = -1;
  // make node `i`'s program the one in LDS (synchronous; only at type changes)
  auto use_prog = [&](int i) {
    const int pr = UF(an[i].prog), len = UF(an[i].prog_len);
    if (pr == cur_prog) return;
    __syncthreads();
    for (int k = tid; k < len; k += NT) lprog[k] = prog[pr + k];
    cur_prog = pr;
    __syncthreads();
  };

  Sreg S;
  Small<ASR> QA, QB;
  double rhs_keep = 0.0;  // rhs of the dx part of node i+1 (thread c < ndx), completed at node i

  // Loads of step p's small operands.  No load here depends on another load, so
  // nothing waits before the S stream behind them is issued.
  auto prefetch_small = [&](int p, Small<ASR>& Q) {
    if (p >= P) return;
    bool f;
    const int i = sched_node(p, N, f);
    const int ia = f ? i - 1 : i;
    if (ia >= 0) {
      const int ne = UF(an[ia].nent), eo = UF(an[ia].ent_off), nc = UF(an[ia].ncpl);
#pragma unroll
      for (int k = 0; k < ASR; ++k) {
        const int idx = tid + NT * k;
        if (idx < ne) Q.as[k] = As[eo + idx];
      }
      if (tid < nc) Q.rhoc = rhoc[ia * lm.cpl + tid];
    }
    const int xo = UF(an[i].x_off), nw = UF(an[i].nw);
    if (tid < nw) {
      if (f) {
        Q.v0 = rhs[xo + tid];
      } else {
        Q.v0 = bt[xo + tid];
        Q.xa = xa[xo + tid];
        Q.qs = qs[xo + tid];
      }
    }
    if (!f) {
      const int nrow = UF(an[i].nrow), ro = UF(an[i].row_off);
      if (tid < nrow) {
        const int r = ro + tid;
        Q.z = za[r];
        Q.y = ya[r];
        Q.rho = rho[r];
        Q.l = ls[r];
        Q.u = us[r];
      }
    }
  };
  auto prefetch_S = [&](int p) {
    if (p >= P) return;
    bool f;
    const int i = sched_node(p, N, f);
    load_S(Sg + UF(an[i].s_off), UF(an[i].nunit), S);
  };

  auto step = [&](auto bufsel, int p) {
    constexpr bool odd = decltype(bufsel)::value;
    Small<ASR>& Q = odd ? QB : QA;
    Small<ASR>& Qn = odd ? QA : QB;
    bool fwd;
    const int i = sched_node(p, N, fwd);
    const int nw = UF(an[i].nw), ntile = UF(an[i].ntile), nunit = UF(an[i].nunit), x_off = UF(an[i].x_off);
    const int ia = fwd ? i - 1 : i;
    __syncthreads();  // previous step done with asb / trow / tcpl / v / y
    if (ia >= 0) {
      use_prog(ia);
      // A values of node ia into LDS: the first NT * ASR from registers, the
      // rest (nodes larger than the dominant type) straight from HBM
      const int ne = UF(an[ia].nent), eo = UF(an[ia].ent_off);
#pragma unroll
      for (int k = 0; k < ASR; ++k) {
        const int idx = tid + NT * k;
        if (idx < ne) asb[idx] = Q.as[k];
      }
      for (int idx = tid + NT * ASR; idx < ne; idx += NT) asb[idx] = As[eo + idx];
    }
    const uint16_t* pg = lprog;
    if (fwd) {
      // ---------------- forward step, node i: gathers over node i-1's coupling rows
      if (i > 0) {
        const PlAdmmNode& pv = an[i - 1];
        const int ncpl = UF(pv.ncpl), cwptr = UF(pv.cwptr), cwe = UF(pv.cwe), cwc = UF(pv.cwc);
        __syncthreads();
        if (tid < ncpl) {  // t_s = rho_s a_s(w_{i-1}) . w_{i-1}
          double acc = 0.0;
          const int q1 = pg[cwptr + tid + 1];
          for (int q = pg[cwptr + tid]; q < q1; ++q) acc += asb[pg[cwe + q]] * y[pg[cwc + q]];
          tcpl[tid] = Q.rhoc * acc;
        }
        __syncthreads();
      }
      if (tid < nw) {  // bt_i = rhs_i - A_{c,dx_i}^T t
        double vv = Q.v0;
        if (i > 0 && tid < ndx) {
          const PlAdmmNode& pv = an[i - 1];
          const int xcptr = UF(pv.xcptr), xce = UF(pv.xce), xcs = UF(pv.xcs);
          double acc = 0.0;
          const int q1 = pg[xcptr + tid + 1];
          for (int q = pg[xcptr + tid]; q < q1; ++q) acc += asb[pg[xce + q]] * tcpl[pg[xcs + q]];
          vv -= acc;
        }
        bt[x_off + tid] = vv;
        v[tid] = vv;
      } else if (tid < 8 * ntile) {
        v[tid] = 0.0;
      }
      __syncthreads();
      matvec_partials(S, nunit, v, dpart, tpart);
      __syncthreads();
      prefetch_small(p + 1, Qn);
      __builtin_amdgcn_sched_barrier(0);
      prefetch_S(p + 1);
      if (tid < nw) y[tid] = matvec_reduce(tid, ntile, dpart, tpart);  // w_i
    } else {
      // ---------------- backward step, node i
      const PlAdmmNode& nd = an[i];
      const int ncpl = UF(nd.ncpl), nrow = UF(nd.nrow), row_off = UF(nd.row_off);
      __syncthreads();
      if (i < N && tid < ncpl) {  // t_s = rho_s a_s(dx_{i+1}) . x~_{i+1}
        const int cxptr = UF(nd.cxptr), cxe = UF(nd.cxe), cxc = UF(nd.cxc);
        double acc = 0.0;
        const int q1 = pg[cxptr + tid + 1];
        for (int q = pg[cxptr + tid]; q < q1; ++q) acc += asb[pg[cxe + q]] * xn[pg[cxc + q]];
        tcpl[tid] = Q.rhoc * acc;
      }
      __syncthreads();
      if (tid < nw) {  // bt_i - A_{c,w_i}^T t
        double vv = Q.v0;
        if (i < N) {
          const int ccptr = UF(nd.ccptr), cce = UF(nd.cce), ccs = UF(nd.ccs);
          double acc = 0.0;
          const int q1 = pg[ccptr + tid + 1];
          for (int q = pg[ccptr + tid]; q < q1; ++q) acc += asb[pg[cce + q]] * tcpl[pg[ccs + q]];
          vv -= acc;
        }
        v[tid] = vv;
      } else if (tid < 8 * ntile) {
        v[tid] = 0.0;
      }
      __syncthreads();
      matvec_partials(S, nunit, v, dpart, tpart);
      __syncthreads();
      prefetch_small(p + 1, Qn);
      __builtin_amdgcn_sched_barrier(0);
      prefetch_S(p + 1);
      if (tid < nw) y[tid] = matvec_reduce(tid, ntile, dpart, tpart);  // x~_i
      __syncthreads();
      const bool store_delta = check && (p >= P - (N + 1));
      if (tid < nrow) {  // z~ = A x~, update_z, update_y (relaxed)
        const int rowptr = UF(nd.rowptr), rowe = UF(nd.rowe), rowc = UF(nd.rowc);
        double zt = 0.0;
        const int q1 = pg[rowptr + tid + 1];
        for (int q = pg[rowptr + tid]; q < q1; ++q) {
          const int c = pg[rowc + q];
          zt += asb[pg[rowe + q]] * (c < nw ? y[c] : xn[c - nw]);
        }
        const double zrel = alpha * zt + (1.0 - alpha) * Q.z;
        double zn = zrel + (1.0 / Q.rho) * Q.y;
        zn = fmin(fmax(zn, Q.l), Q.u);
        const double dy = Q.rho * (zrel - zn);
        const double yn = Q.y + dy;
        const int r = row_off + tid;
        za[r] = zn;
        ya[r] = yn;
        if (store_delta) dys[r] = dy;
        trow[tid] = Q.rho * zn - yn;
      }
      __syncthreads();
      if (tid < nw) {  // update_x and next rhs = sigma x - q + A^T (rho z - y)
        const int j = x_off + tid;
        const double xnew = alpha * y[tid] + (1.0 - alpha) * Q.xa;
        xa[j] = xnew;
        if (store_delta) dxs[j] = xnew - Q.xa;
        double acc = sigma * xnew - Q.qs;
        if (i < N) {
          const int colptr = UF(nd.colptr), colr = UF(nd.colr);
          const int e1 = pg[colptr + tid + 1];
          for (int e = pg[colptr + tid]; e < e1; ++e) acc += asb[e] * trow[pg[colr + e]];
          if (tid < ndx) {  // rows of node i on dx_{i+1} complete rhs_{i+1}
            double a2 = 0.0;
            const int f1 = pg[colptr + nw + tid + 1];
            for (int e = pg[colptr + nw + tid]; e < f1; ++e) a2 += asb[e] * trow[pg[colr + e]];
            rhs[UF(an[i + 1].x_off) + tid] = rhs_keep + a2;
          }
        }
        if (tid < ndx && i > 0) rhs_keep = acc;
        else rhs[j] = acc;
        // the next step (forward node 0) prefetched rhs_0 before this phase wrote it
        if (i == 0) Qn.v0 = acc;
        if (tid < ndx) xn[tid] = y[tid];
      }
    }
  };

  prefetch_small(0, QA);
  __builtin_amdgcn_sched_barrier(0);
  prefetch_S(0);
  for (int p = 0; p < P; p += 2) {
    step(std::integral_constant<bool, false>(), p);
    if (p + 1 < P) step(std::integral_constant<bool, true>(), p + 1);
  }
  if (tid == 0) info->iter += niter;
}

namespace {
template <int ASR>
void launch_admm_t(PlOcpHandle* h, int niter, int check, size_t lds, const LdsMap& lm) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)k_admm<ASR>, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(k_admm<ASR>, dim3(h->B), dim3(256), lds, h->stream, h->d, h->N, h->n, h->m, h->nnz, h->ndx,
                     h->S_stride, lm, niter, check, h->set.sigma, h->set.alpha);
}
}  // namespace

static LdsMap admm_lds_map(const PlOcpHandle* h) {
  return LdsMap{((h->nw_max + 7) / 8) * 8, std::max(h->ncpl_max, 1), std::max(h->nrow_max, 1), h->nunit_max,
                std::max(h->nent_max, 1), h->admm_dom_prog, h->admm_dom_len, h->N + 1};
}

int admm_lds_bytes(const PlOcpHandle* h) { return (int)admm_lds_map(h).total(); }

void launch_admm(PlOcpHandle* h, int niter, int check, int it_base) {
  (void)it_base;
  const LdsMap lm = admm_lds_map(h);
  const size_t lds = lm.total();
  const bool prof = h->profile && h->prof_n < 64;
  if (prof) hipEventRecord(h->prof_ev[h->prof_n][0], h->stream);
  if (h->admm_asr <= 4) launch_admm_t<4>(h, niter, check, lds, lm);
  else if (h->admm_asr <= 6) launch_admm_t<6>(h, niter, check, lds, lm);
  else launch_admm_t<8>(h, niter, check, lds, lm);
  if (prof) {
    hipEventRecord(h->prof_ev[h->prof_n][1], h->stream);
    h->prof_n++;
    h->prof_admm_iters += (long long)h->B * niter;
  }
}
