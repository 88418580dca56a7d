// ADMM sweeps in REDUCED-CHAIN form: the small-batch kernel (one workgroup of W waves
// per problem).  Same OSQP 0.6 iteration as k_admm.hip (update_xz_tilde, update_x,
// update_z, update_y), same block factor S_i; only the order of the linear solve differs.
//
// Why.  k_admm / k_admm2 walk the horizon node by node: 2N sequential steps per ADMM
// iteration, each a full nw x nw block mat-vec plus the row / column gathers of the node.
// At B = 1024 that is the right shape (one wave per problem fills the chip and the factor
// stream is HBM-bound), but for a few hundred problems or one problem the chip idles and
// every step is a chain of LDS / memory round trips (config 3: 17 k cycles per step, 0.11
// of HBM; one Go2 problem: 17 ms per MPC step).
//
// K = P + sigma I + A^T R A is block tridiagonal in w_i = (dx_i, u_i) and the coupling
// block K_{i+1,i} touches only the dx_{i+1} rows: C_i (ndx x nw).  With
//     F_i = C_i S_i[:, dx]  (ndx x ndx),   G_i = S_i[dx, dx]
// (k_fred, after the factor) the two sweeps reduce to ndx-sized recurrences, and every
// full-block product becomes node-parallel (rhs = rhs' + [a2_{i-1}; 0]: the node's own
// column sums plus the previous node's coupling rows on dx_i):
//   P   (parallel)  g_i = S_i rhs'_i,  c'_i = C_i g_i,  h'_i = g_i[dx]
//   C1  (chain)     delta_0 = 0;  d_{i+1} = c'_i - F_i delta_i,  delta_{i+1} = d_{i+1} - a2_i
//   P2  (parallel)  w_i[dx] = h'_i - G_i delta_i
//   C2  (chain)     e_N = w_N[dx];  e_i = w_i[dx] - F_i^T e_{i+1}              (e_i = x~_i[dx])
//   P3  (parallel)  x~_i = S_i (rhs'_i - [delta_i; 0] - C_i^T e_{i+1}), then the node's
//                   z~ = A x~, z / y updates, x update and the next rhs'_i, a2_i, and
//                   (fused, S_i still in registers) the next iteration's P for node i.
// Per iteration: S_i is read once (the sweep kernels read it twice) plus 3 ndx^2 chain
// values per node; the sequential part is 2N ndx x ndx mat-vecs on one wave with no
// gathers, and the node-parallel phases spread the rest over the W waves.
// tools/proto_chain.py checks the rearrangement in numpy against the sweep and a sparse LU
// (same error level, 1e-11 after 100 ADMM iterations on the fixtures).
//
// Determinism: fixed node -> wave assignment, fixed per-lane summation orders and LDS f64
// adds applied in instruction order, so a problem gives the same bits in any batch that
// selects this kernel (the sweep kernels sum in other orders: results agree to round-off).
//
// Several workgroups per problem (r06, rc_groups).  The node-parallel phases P / P3 spread
// over G workgroups of W waves (node i on wave i mod (G W)), so the 21 Go2 nodes of config 2
// run in one round instead of three; the chains stay on workgroup 0.  The phases hand off
// through global memory inside the launch (MI355X_MICROARCH.md, inter-workgroup visibility):
//   fan-in   every workgroup g > 0, after its nodes: each wave s_waitcnt vmcnt(0), workgroup
//            barrier, one agent-scope atomic add to the problem's count; workgroup 0 polls it;
//   fan-out  workgroup 0, after the chains: the same drain, then one agent-scope store of the
//            iteration's epoch, which the others poll.
// Every handed-off value (c'_i, h'_i, a2_i from the nodes; delta_i, e_i from the chains; the
// last iteration's rhs) is stored write-through (sc1) and loaded sc1 (st_sc1 / ld_sc1: L2,
// never a stale L1 line), so no fence is needed.  Every poll is bounded: a workgroup that gives
// up writes a code into the problem's give-up word, poisons x (NaN) and exits, and a waiting
// workgroup that sees the word exits too.  All B G workgroups are resident together: rc_groups
// keeps B G <= the CU count (the kernel's LDS allows one workgroup per CU).  G = 1 is the r05
// kernel (PL_PATH_RC_ONE_GROUP); the node arithmetic does not depend on G, so the iterates are
// bit-identical for any G.
#include <algorithm>

#include "admm_common.h"
#include "pinoloco.h"  // PL_PATH_RC_ONE_GROUP
#include "state.h"

namespace {

using namespace admm;

struct RcLds {
  int prog_dbl, chn, per_wave;  // programs | chain buffers [2][64] | per-wave regions
  int v, y, acc, trow, tcpl, bc, asb, asb_cap;
};

// Handed-off values: write-through stores / L1-bypassing loads (buffer_{store,load}_dwordx2 sc1).
// Buffer ops, not relaxed atomics: the LDS-only barriers of the chains carry an acquire fence, and
// an acquire after an atomic load makes the compiler wait vmcnt(0), draining the chain-block
// prefetch every step.
typedef __attribute__((address_space(1))) unsigned gu32;
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
constexpr int RC_SC1 = 16;  // cache-policy bits of the buffer ops: sc1
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rc_rsrc(const double* base, int count) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(base), (short)0, count * 8, 0x00020000);
}
// SC: the launch runs several workgroups per problem (the hand-offs need sc1); with one
// workgroup per problem the same accesses are plain (L1 / L2 as in r05)
template <bool SC>
__device__ __forceinline__ double ld_sc1(__amdgpu_buffer_rsrc_t r, int idx) {
  return __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(r, idx * 8, 0, SC ? RC_SC1 : 0));
}
template <bool SC>
__device__ __forceinline__ void st_sc1(__amdgpu_buffer_rsrc_t r, int idx, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, idx * 8, 0, SC ? RC_SC1 : 0);
}

// hand-off words of one problem (d.rcsync, zeroed before every launch)
enum { RC_ARRIVE = 0, RC_EPOCH = 1, RC_GIVEUP = 2 };
constexpr unsigned RC_SPIN_MAX = 1u << 21;  // polls (s_sleep 2 each) before a workgroup gives up

// One wave polls *w >= target (relaxed sc1 loads); false when the give-up word is set or after
// RC_SPIN_MAX polls (then it sets the word to `code`).
__device__ __forceinline__ bool rc_poll(unsigned* sy, int word, unsigned target, unsigned code) {
  for (unsigned s = 0;; ++s) {
    if (__hip_atomic_load((gu32*)(sy + word), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >= target) return true;
    if (__hip_atomic_load((gu32*)(sy + RC_GIVEUP), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return false;
    if (s >= RC_SPIN_MAX) {
      __hip_atomic_store((gu32*)(sy + RC_GIVEUP), code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return false;
    }
    __builtin_amdgcn_s_sleep(2);
  }
}

struct Sb {
  double2 s[KM][8];
};

// Lane map of the chains (k_admm_rc): RW rows per wave, each split over NS lanes of SG columns;
// 2 RW NS <= 64 (forward: F and G rows side by side).  NS is a power of two (the row sum is a
// DPP butterfly inside a quad, r06; the r05 map summed 6 lanes by ds_bpermute, ~40 % of a step)
// and the stored rows are zero-padded to XP = NS SG columns, SG even (16-byte loads).  PD steps
// of chain blocks in flight per lane, within a register budget (2 waves per SIMD at W = 8).
constexpr int rc_pick_ns(int RW) { return 2 * RW * 4 <= 64 ? 4 : (2 * RW * 2 <= 64 ? 2 : 1); }
constexpr int rc_row_len(int X, int W) {  // XP
  const int ns = rc_pick_ns((X + W - 1) / W);
  return (X + 2 * ns - 1) / (2 * ns) * (2 * ns);
}
template <int X, int W>
struct RcChain {
  static constexpr int RW = (X + W - 1) / W;
  static constexpr int NS = rc_pick_ns(RW);
  static constexpr int XP = rc_row_len(X, W);
  static constexpr int SG = XP / NS;
  static constexpr int PD = (W >= 8 ? 72 : 144) / SG < 2 ? 2 : ((W >= 8 ? 72 : 144) / SG > 10 ? 10 : (W >= 8 ? 72 : 144) / SG);
};

// Chain blocks in the chains' lane order (r06): per node a forward part [W][SG/2][LF] and a
// backward part [W][SG/2][LB] of double2, LF = 2 RW NS lanes (F rows, then G rows), LB = RW NS
// (F^T rows), so the 16-byte load k of wave w is one contiguous run over its lanes (the
// row-major r05 blocks put every load's lanes on ~16 cache lines: the L1 request rate bound
// the chain steps).  Columns past X are zero.
struct RcMap {
  int W, RW, NS, XP, SG, LF, LB, fwd, node;  // fwd / node: doubles per part / per node
};
constexpr RcMap rc_map(int X, int W) {
  const int RW = (X + W - 1) / W, NS = rc_pick_ns(RW), XP = rc_row_len(X, W), SG = XP / NS;
  const int LF = 2 * RW * NS, LB = RW * NS;
  return RcMap{W, RW, NS, XP, SG, LF, LB, W * SG * LF, W * SG * (LF + LB)};
}

// x + (x of the lane whose index differs in bit 0 / bit 1): one DPP quad permutation per 32-bit
// half.  Both partners compute a + b with the same operands, so every lane of the group ends
// with the same bits.
template <int CTRL>
__device__ __forceinline__ double dpp_add(double x) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(x), CTRL, 0xF, 0xF, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(x), CTRL, 0xF, 0xF, false);
  return x + __hiloint2double(hi, lo);
}

// Workgroup barrier that orders LDS only (lgkmcnt(0) + s_barrier): __syncthreads() would also
// wait vmcnt(0) and drain the chain blocks kept in flight across the steps.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

}  // namespace

// ---------------------------------------------------------------------------
// Chain blocks of node i (one 256-thread workgroup per (problem, node)), from the stored
// (symmetrised, tiled) factor block that the ADMM kernels use: F_i, F_i^T and G_i = S_i[dx, dx]
// in the chains' lane order (RcMap), d.CH[b] + i * node doubles.
// F_i[a][k] = sum_{(e, s) in xc(a)} A_e rho_s sum_{(e', l) in cw(s)} A_e' S_i[l][k]
// (the coupling product the sweep kernels apply as t_s = rho_s a_s(w) . w).
__global__ __launch_bounds__(256) void k_fred(PlDev d, int N, int nnz, int ndx, int S_stride, int cpl_stride,
                                              long long ch_stride, RcMap mp) {
  extern __shared__ double sc[];  // S_i[:, 0:ndx] dense, sc[l * ndx + k]; then F_i
  const int b = blockIdx.x / (N + 1), i = blockIdx.x - b * (N + 1);
  typedef const __attribute__((address_space(4))) PlAdmmNode* CNode;
  const CNode an = (CNode)d.anodes;
  const int nw = an[i].nw, K = an[i].nunit;
  const double2* Sg = reinterpret_cast<const double2*>(d.S + (size_t)b * S_stride + an[i].s_off);
  for (int q = threadIdx.x; q < nw * ndx; q += 256) {
    const int l = q / ndx, k = q - l * ndx;
    int I = l >> 2, J = k >> 2, r = l & 3, c = k & 3;
    if (I < J) {  // upper triangle: the stored lower tile, transposed
      const int t1 = I, t2 = r;
      I = J; J = t1; r = c; c = t2;
    }
    const int t = I * (I + 1) / 2 + J;
    const int ln = t / K, sl = t - ln * K;
    const double2 p = Sg[(sl * 8 + 2 * r + (c >> 1)) * 64 + ln];
    sc[q] = (c & 1) ? p.y : p.x;
  }
  __syncthreads();
  double* fs = sc + nw * ndx;  // F_i, fs[a * ndx + k]
  const int X2 = ndx * ndx;
  if (i < N) {
    const uint16_t* P = d.aprog + an[i].prog;
    const double* As = d.As + (size_t)b * nnz + an[i].ent_off;
    const double* rc = d.rhoc + ((size_t)b * (N + 1) + i) * cpl_stride;
    const uint32_t* xc = reinterpret_cast<const uint32_t*>(P + an[i].xcp);
    const uint32_t* cw = reinterpret_cast<const uint32_t*>(P + an[i].cwp);
    const uint16_t* xcptr = P + an[i].xcptr;
    const uint16_t* cwptr = P + an[i].cwptr;
    for (int q = threadIdx.x; q < X2; q += 256) {
      const int a = q / ndx, k = q - a * ndx;
      double f = 0.0;
      for (int qq = xcptr[a]; qq < xcptr[a + 1]; ++qq) {
        const uint32_t w = xc[qq];
        const int s = (int)(w >> 16);
        double acc = 0.0;
        for (int q2 = cwptr[s]; q2 < cwptr[s + 1]; ++q2) {
          const uint32_t w2 = cw[q2];
          acc += As[w2 & 0xffff] * sc[(int)(w2 >> 16) * ndx + k];
        }
        f += As[w & 0xffff] * (rc[s] * acc);
      }
      fs[q] = f;
    }
  } else {
    for (int q = threadIdx.x; q < X2; q += 256) fs[q] = 0.0;  // F rows are not used at node N
  }
  __syncthreads();
  // lane order of the chains (RcMap): entry e -> (part, wave w, load k, lane, half h)
  double* CH = d.CH + (size_t)b * ch_stride + (size_t)i * mp.node;
  const int hs = mp.SG / 2;
  for (int e = threadIdx.x; e < mp.node; e += 256) {
    const bool fwd = e < mp.fwd;
    const int L = fwd ? mp.LF : mp.LB, e2 = (fwd ? e : e - mp.fwd) >> 1, h = e & 1;
    const int lane = e2 % L, wk = e2 / L, k = wk % hs, w = wk / hs;
    const int cq = lane / mp.NS, cs = lane - cq * mp.NS;
    const bool rowF = !fwd || cq < mp.RW;
    const int cj = rowF ? cq : cq - mp.RW;
    const int r0 = (ndx * w) / mp.W, nr = (ndx * (w + 1)) / mp.W - r0;
    const int row = r0 + min(cj, nr - 1), col = cs * mp.SG + 2 * k + h;
    double v = 0.0;
    if (col < ndx) v = !fwd ? fs[col * ndx + row] : (rowF ? fs[row * ndx + col] : sc[row * ndx + col]);
    CH[e] = v;
  }
}

// ---------------------------------------------------------------------------
template <int W, int X, bool SC>
__global__ __launch_bounds__(64 * W, 1) void k_admm_rc(PlDev d, int N, int n, int m, int nnz, int S_stride,
                                                       int cpl_stride, long long ch_stride, int chv_stride, RcLds lm,
                                                       int niter, int check, double sigma, double alpha, int G) {
  extern __shared__ double lds[];
  const int b = blockIdx.x / G, g = blockIdx.x - b * G;  // problem, workgroup of the problem
  PlProbInfo* info = d.info + b;
  if (info->done) return;  // every workgroup of the problem
  {
    const uint4* src = reinterpret_cast<const uint4*>(d.aprog);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    for (int k = threadIdx.x; k < lm.prog_dbl / 2; k += 64 * W) dst[k] = src[k];
  }
  __syncthreads();
  constexpr int ndx = X;
  typedef RcChain<X, W> CS;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint16_t* PG = reinterpret_cast<const uint16_t*>(lds);
  double* Wr = lds + lm.prog_dbl + 130 + wv * lm.per_wave;
  int* okw = reinterpret_cast<int*>(lds + lm.prog_dbl + 128);  // a poll's outcome, for the whole workgroup
  unsigned* sy = d.rcsync + (size_t)b * PL_RC_SYNC;
  double* v = Wr + lm.v;        // mat-vec input, zero padded to 4 T
  double* y = Wr + lm.y;        // mat-vec output [0, nw) | e_{i+1} [nw, nw + ndx)
  double* acc = Wr + lm.acc;    // LDS f64-add accumulators (mat-vec, row sums, column sums)
  double* trow = Wr + lm.trow;  // rho z - y of the node's rows
  double* tcpl = Wr + lm.tcpl;  // coupling-row products
  double* bc = Wr + lm.bc;      // chain / P2 broadcast vector
  double* asb = Wr + lm.asb;    // the node's A values
  const int cap = lm.asb_cap;

  const double* __restrict__ As = d.As + (size_t)b * nnz;
  const double* __restrict__ rho = d.rho + (size_t)b * m;
  const double* __restrict__ rhoc = d.rhoc + (size_t)b * (N + 1) * cpl_stride;
  const double* __restrict__ ls = d.ls + (size_t)b * m;
  const double* __restrict__ us = d.us + (size_t)b * m;
  const double* __restrict__ qs = d.qs + (size_t)b * n;
  const double* __restrict__ Sg = d.S + (size_t)b * S_stride;
  const double* CH = d.CH + (size_t)b * ch_stride;  // no __restrict__: keeps the chains' first rows from being hoisted out of the iteration loop
  double* za = d.za + (size_t)b * m;
  double* ya = d.ya + (size_t)b * m;
  double* xa = d.xa + (size_t)b * n;
  double* rhs = d.rhs + (size_t)b * n;
  double* dxs = d.dxs + (size_t)b * n;
  double* dys = d.dys + (size_t)b * m;
  // chain vectors, (N + 2) ndx each: delta_i, w_i[dx], e_i, a2_{i-1} (A2[i] = a2_{i-1}), c'_i, h'_i
  const int L = (N + 2) * ndx;
  double* DL = d.chv + (size_t)b * chv_stride;
  // DL + L: w_i[dx] until r06 (now kept in LDS by the chains, whist)
  double* EE = DL + 2 * L;
  double* A2 = DL + 3 * L;
  double* CP = DL + 4 * L;
  double* HP = DL + 5 * L;
  // the handed-off vectors through buffer descriptors (uniform: kernel arguments + blockIdx)
  const __amdgpu_buffer_rsrc_t rchv = rc_rsrc(DL, 6 * L), rrhs = rc_rsrc(rhs, n);
  constexpr int oDL = 0;
  const int oEE = 2 * L, oA2 = 3 * L, oCP = 4 * L, oHP = 5 * L;
  typedef const __attribute__((address_space(4))) PlAdmmNode* CNode;
  const CNode an = (CNode)d.anodes;
  const int rr = min(lane, ndx - 1);  // chain row / column of the lane (clamped)

  auto load_S = [&](int i, int kbase, Sb& R) __attribute__((always_inline)) {
    const int K = an[i].nunit;
    const double2* p = reinterpret_cast<const double2*>(Sg + an[i].s_off);
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int kk = min(kbase + k, K - 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) R.s[k][j] = gld(p, (kk * 8 + j) * 64 + lane);
    }
  };

  // y[0..nw) = S_i v (v zero padded to 4 T).  R holds slots 0..KM-1 on entry when `have`.
  auto matvec = [&](int i, Sb& R, bool have) __attribute__((always_inline)) {
    const int K = an[i].nunit, T = an[i].ntile, ntl = an[i].ntl, nw = an[i].nw;
    for (int o = lane; o < 5 * T; o += 64) acc[o] = 0.0;
    wsync();
    const double2* v2 = reinterpret_cast<const double2*>(v);
    int curI = -1;
    double sa[4] = {0.0, 0.0, 0.0, 0.0};
    auto emit_row = [&](int I0) __attribute__((always_inline)) {
#pragma unroll
      for (int r = 0; r < 4; ++r) lds_add(acc + I0 * 5 + r, sa[r]);
    };
    for (int kb = 0; kb < K; kb += KM) {
      if (!(kb == 0 && have)) load_S(i, kb, R);
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        const int kk = kb + k;
        const int t = K * lane + kk;
        if (kk < K && t < ntl) {
          int I, J;
          tile_ij(t, I, J);
          const double2 a0 = v2[2 * J], a1 = v2[2 * J + 1];
          double rp[4];
#pragma unroll
          for (int r = 0; r < 4; ++r)
            rp[r] = R.s[k][2 * r].x * a0.x + R.s[k][2 * r].y * a0.y + R.s[k][2 * r + 1].x * a1.x +
                    R.s[k][2 * r + 1].y * a1.y;
          if (I != J) {
            const double2 c0 = v2[2 * I], c1 = v2[2 * I + 1];
            const double vi[4] = {c0.x, c0.y, c1.x, c1.y};
            double cp[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              cp[0] += R.s[k][2 * r].x * vi[r];
              cp[1] += R.s[k][2 * r].y * vi[r];
              cp[2] += R.s[k][2 * r + 1].x * vi[r];
              cp[3] += R.s[k][2 * r + 1].y * vi[r];
            }
#pragma unroll
            for (int c = 0; c < 4; ++c) lds_add(acc + J * 5 + c, cp[c]);
          }
          if (I != curI) {
            if (curI >= 0) emit_row(curI);
            curI = I;
#pragma unroll
            for (int r = 0; r < 4; ++r) sa[r] = rp[r];
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) sa[r] += rp[r];
          }
        }
      }
    }
    if (curI >= 0) emit_row(curI);
    wsync();
    for (int o = lane; o < nw; o += 64) y[o] = acc[(o >> 2) * 5 + (o & 3)];
    wsync();
  };

  // c'_i = C_i y, h'_i = y[dx]  (y = g_i = S_i rhs'_i)
  auto coupling_out = [&](int i, auto A) __attribute__((always_inline)) {
    const uint16_t* P = PG + an[i].prog;
    if (i < N) {
      const int ncp = an[i].ncpl;
      if (lane < ncp) {
        const uint32_t* cw = reinterpret_cast<const uint32_t*>(P + an[i].cwp);
        const int q0 = P[an[i].cwptr + lane], q1 = P[an[i].cwptr + lane + 1];
        double a = 0.0;
        for (int qq = q0; qq < q1; ++qq) {
          const uint32_t w = cw[qq];
          a += A(w & 0xffff) * y[w >> 16];
        }
        tcpl[lane] = rhoc[i * cpl_stride + lane] * a;
      }
      wsync();
      if (lane < ndx) {
        const uint32_t* xc = reinterpret_cast<const uint32_t*>(P + an[i].xcp);
        const int q0 = P[an[i].xcptr + lane], q1 = P[an[i].xcptr + lane + 1];
        double c = 0.0;
        for (int qq = q0; qq < q1; ++qq) {
          const uint32_t w = xc[qq];
          c += A(w & 0xffff) * tcpl[w >> 16];
        }
        st_sc1<SC>(rchv, oCP + i * ndx + lane, c);
      }
    }
    if (lane < ndx) st_sc1<SC>(rchv, oHP + i * ndx + lane, y[lane]);
    wsync();
  };

#ifndef PL_RC_SUBTIMING
#define PL_RC_SUBTIMING 0
#endif
#if PL_RC_SUBTIMING  // experiment builds (PL_HIPCC_DEFS=-DPL_RC_SUBTIMING=1): sub-phases of pnode, wave 0 of workgroup 0
  unsigned long long sacc[7] = {0, 0, 0, 0, 0, 0, 0}, sl = 0;
  const bool stim = d.dbg != nullptr && blockIdx.x % G == 0 && threadIdx.x < 64;
  auto SUB = [&](int slot) __attribute__((always_inline)) {
    if (stim) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      if (slot >= 0) sacc[slot] += now - sl;
      sl = now;
    }
  };
  unsigned long long cacc[4] = {0, 0, 0, 0}, cl = 0;
  auto CSUB = [&](int slot) __attribute__((always_inline)) {
    if (stim) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      if (slot >= 0) cacc[slot] += now - cl;
      cl = now;
    }
  };
#else
  auto SUB = [&](int) __attribute__((always_inline)) {};
  auto CSUB = [&](int) __attribute__((always_inline)) {};
#endif
  // ---- one node of a parallel phase.  mode 0: P only (rhs complete, a2 = 0); 1: P3 + the
  // next iteration's P; 2: P3 only (the launch's last iteration)
  auto pnode = [&](int i, int mode, bool store_delta) __attribute__((always_inline)) {
    SUB(-1);
    const int nw = an[i].nw, T4 = 4 * an[i].ntile, x_off = an[i].x_off;
    const int eo = an[i].ent_off, ne = an[i].nent;
    const bool term = i == N;
    const uint16_t* P = PG + an[i].prog;
    const double* __restrict__ Ai = As + eo;
    // every operand of the node is issued at once: the factor block (registers), the node's
    // vectors, then the node's A values straight into LDS (global_load_lds, no VGPRs); one
    // vmcnt(0) then covers them all (one memory latency per node)
    Sb R;
    load_S(i, 0, R);
    double rh[MV], xo[MV], qo[MV];
#pragma unroll
    for (int mm = 0; mm < MV; ++mm) {
      const int c = x_off + min(lane + 64 * mm, nw - 1);
      rh[mm] = rhs[c];
      xo[mm] = mode ? xa[c] : 0.0;
      qo[mm] = mode ? qs[c] : 0.0;
    }
    const int nrow = an[i].nrow, ro = an[i].row_off;
    double lz[MR], ly[MR], lr[MR], ll[MR], lu[MR];
    if (mode) {
#pragma unroll
      for (int mm = 0; mm < MR; ++mm) {
        const int r = ro + min(lane + 64 * mm, max(nrow - 1, 0));
        lz[mm] = za[r];
        ly[mm] = ya[r];
        lr[mm] = rho[r];
        ll[mm] = ls[r];
        lu[mm] = us[r];
      }
    }
    const double dl = mode ? ld_sc1<SC>(rchv, oDL + i * ndx + rr) : 0.0;
    const double ee = (mode && !term) ? ld_sc1<SC>(rchv, oEE + (i + 1) * ndx + rr) : 0.0;
    const int na = min(ne, cap);
    const int sh = (int)(((size_t)Ai >> 3) & 1);  // 16-byte alignment of the DMA source
    {
      typedef __attribute__((address_space(1))) const void* GP;
      typedef __attribute__((address_space(3))) void* LP;
      const double* g0 = Ai - sh;
      const int n2 = (na + sh + 1) >> 1;
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the previous node's reads of the area are done
      for (int j = 0; j * 64 < n2; ++j)
        if (j * 64 + lane < n2) __builtin_amdgcn_global_load_lds((GP)(g0 + 2 * (j * 64 + lane)), (LP)(asb + 128 * j), 16, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0xF70);  // vmcnt(0)
    SUB(0);
    const double* asbs = asb + sh;
    auto A = [&](int e) __attribute__((always_inline)) { return e < na ? asbs[e] : Ai[e]; };
    if (mode == 0) {
#pragma unroll
      for (int mm = 0; mm < MV; ++mm) {
        const int c = lane + 64 * mm;
        if (c < nw) v[c] = rh[mm];
        else if (c < T4) v[c] = 0.0;
      }
      if (lane < ndx) st_sc1<SC>(rchv, oA2 + (i + 1) * ndx + lane, 0.0);
      wsync();
      matvec(i, R, true);
      coupling_out(i, A);
      return;
    }
    // ---- P3
    if (!term && lane < ndx) y[nw + lane] = ee;
    wsync();
    // t_s = rho_s a_s(dx_{i+1}) . e_{i+1}
    if (!term) {
      const int ncp = an[i].ncpl;
      if (lane < ncp) {
        const uint32_t* cx = reinterpret_cast<const uint32_t*>(P + an[i].cxp);
        const int q0 = P[an[i].cxptr + lane], q1 = P[an[i].cxptr + lane + 1];
        double a = 0.0;
        for (int qq = q0; qq < q1; ++qq) {
          const uint32_t w = cx[qq];
          a += A(w & 0xffff) * y[nw + (w >> 16)];
        }
        tcpl[lane] = rhoc[i * cpl_stride + lane] * a;
      }
      wsync();
    }
    // u = rhs'_i - [delta_i; 0] - C_i^T e_{i+1}
    {
      const uint32_t* cc = reinterpret_cast<const uint32_t*>(P + an[i].ccp);
#pragma unroll
      for (int mm = 0; mm < MV; ++mm) {
        const int c = lane + 64 * mm;
        if (c < nw) {
          double u = rh[mm] - (mm == 0 && c < ndx ? dl : 0.0);
          if (!term) {
            const int q0 = P[an[i].ccptr + c], q1 = P[an[i].ccptr + c + 1];
            double s = 0.0;
            for (int qq = q0; qq < q1; ++qq) {
              const uint32_t w = cc[qq];
              s += A(w & 0xffff) * tcpl[w >> 16];
            }
            u -= s;
          }
          v[c] = u;
        } else if (c < T4) {
          v[c] = 0.0;
        }
      }
    }
    wsync();
    SUB(1);
    matvec(i, R, true);  // y[0..nw) = x~_i
    SUB(2);
    double kz[MR], ky[MR], kd[MR];
    if (!term) {
      // z~ = A [x~_i; e_{i+1}] over row chunks
      const uint16_t* rowe = P + an[i].rowe;
      const uint8_t* rowc = reinterpret_cast<const uint8_t*>(P + an[i].rowc);
      const uint32_t* rch = reinterpret_cast<const uint32_t*>(P + an[i].rch);
      const uint8_t* rchr = reinterpret_cast<const uint8_t*>(P + an[i].rchr);
      const int rchn = an[i].rchn;
      for (int o = lane; o < nrow; o += 64) acc[o] = 0.0;
      wsync();
      for (int c0 = 0; c0 < rchn; c0 += 64) {
        const int ch = c0 + lane;
        const uint32_t cw = rch[min(ch, rchn - 1)];
        const int q0 = cw & 0xffff, len = ch < rchn ? (int)(cw >> 16) - q0 : 0;
        double a = 0.0;
#pragma unroll
        for (int k = 0; k < PL_CHUNK; ++k) {
          const int qq = q0 + min(k, max(len - 1, 0));
          const double t = A(rowe[qq]) * y[rowc[qq]];
          a += k < len ? t : 0.0;
        }
        if (ch < rchn) lds_add(acc + rchr[ch], a);
      }
      wsync();
      // update_z, update_y (relaxed)
#pragma unroll
      for (int mm = 0; mm < MR; ++mm) {
        const int r = lane + 64 * mm;
        kz[mm] = ky[mm] = kd[mm] = 0.0;
        if (r < nrow) {
          const double zrel = alpha * acc[r] + (1.0 - alpha) * lz[mm];
          double zn = zrel + (1.0 / lr[mm]) * ly[mm];
          zn = fmin(fmax(zn, ll[mm]), lu[mm]);
          const double dy = lr[mm] * (zrel - zn);
          const double yn = ly[mm] + dy;
          trow[r] = lr[mm] * zn - yn;
          kz[mm] = zn;
          ky[mm] = yn;
          kd[mm] = dy;
        }
      }
      wsync();
      // A^T (rho z - y) over column chunks (own columns and dx_{i+1})
      const uint8_t* colr = reinterpret_cast<const uint8_t*>(P + an[i].colr);
      const uint32_t* cch = reinterpret_cast<const uint32_t*>(P + an[i].cch);
      const uint8_t* cchc = reinterpret_cast<const uint8_t*>(P + an[i].cchc);
      const int cchn = an[i].cchn;
      for (int o = lane; o < an[i].ncol; o += 64) acc[o] = 0.0;
      wsync();
      for (int c0 = 0; c0 < cchn; c0 += 64) {
        const int ch = c0 + lane;
        const uint32_t cw = cch[min(ch, cchn - 1)];
        const int e0 = cw & 0xffff, len = ch < cchn ? (int)(cw >> 16) - e0 : 0;
        double a = 0.0;
#pragma unroll
        for (int k = 0; k < PL_CHUNK; ++k) {
          const int e = e0 + min(k, max(len - 1, 0));
          const double t = A(e) * trow[colr[e]];
          a += k < len ? t : 0.0;
        }
        if (ch < cchn) lds_add(acc + cchc[ch], a);
      }
      wsync();
    }
    SUB(3);
    // update_x and the next rhs'_i = sigma x - q + (own rows)^T (rho z - y); a2_i
    double rn[MV];
#pragma unroll
    for (int mm = 0; mm < MV; ++mm) {
      const int c = lane + 64 * mm;
      rn[mm] = 0.0;
      if (c < nw) {
        const double xnew = alpha * y[c] + (1.0 - alpha) * xo[mm];
        rn[mm] = sigma * xnew - qo[mm] + (term ? 0.0 : acc[c]);
        gst(xa, x_off + c, xnew);
        if (store_delta) gst(dxs, x_off + c, xnew - xo[mm]);
        if (mode == 2) st_sc1<SC>(rrhs, x_off + c, rn[mm]);  // read by workgroup 0's closing pass
        else gst(rhs, x_off + c, rn[mm]);
      }
    }
    if (!term) {
      if (lane < ndx) st_sc1<SC>(rchv, oA2 + (i + 1) * ndx + lane, acc[nw + lane]);
#pragma unroll
      for (int mm = 0; mm < MR; ++mm) {
        const int r = lane + 64 * mm;
        if (r < nrow) {
          gst(za, ro + r, kz[mm]);
          gst(ya, ro + r, ky[mm]);
          if (store_delta) gst(dys, ro + r, kd[mm]);
        }
      }
    }
    SUB(4);
    if (mode == 2) return;
    wsync();
#pragma unroll
    for (int mm = 0; mm < MV; ++mm) {
      const int c = lane + 64 * mm;
      if (c < nw) v[c] = rn[mm];
      else if (c < T4) v[c] = 0.0;
    }
    wsync();
    matvec(i, R, an[i].nunit <= KM);  // y = g_i = S_i rhs'_i: the block is still in R unless it took several passes
    SUB(5);
    coupling_out(i, A);
    SUB(6);
  };

  // ---- The chains, spread over the whole workgroup: wave w owns rows [r0, r0 + nr) of the
  // recurrence and every row is split over NS lanes (SG columns each), so a step is SG FMAs,
  // an NS-lane reduction and one LDS barrier; PD steps of chain blocks are in flight per lane.
  //   C1 (steps i = 0..N): lanes q < RW: d_{i+1}[r] = c'_i[r] - F_i[r] . delta_i,
  //                          delta_{i+1}[r] = d_{i+1}[r] - a2_i[r];
  //                        lanes RW <= q < 2 RW: w_i[r] = h'_i[r] - G_i[r] . delta_i
  //   C2 (steps i = N-1..1): lanes q < RW: e_i[r] = w_i[r] - F_i^T[r] . e_{i+1}
  // delta / e are double-buffered in LDS (read one buffer, write the other), so one barrier
  // per step suffices.  Fixed lane -> (row, segment) map and a fixed-order reduction.
  constexpr int RW = CS::RW, NS = CS::NS, SG = CS::SG, PD = CS::PD;
  constexpr RcMap MP = rc_map(X, W);
  constexpr int LF = MP.LF, LB = MP.LB;
  const int r0 = (X * wv) / W, nr = (X * (wv + 1)) / W - r0;
  const int cq = lane / NS, cs = lane - cq * NS;
  const bool cF = cq < RW;
  const int cj = cF ? cq : cq - RW;
  const bool cvalid = cj < nr && cq < 2 * RW;
  const int crow = r0 + min(cj, nr - 1);
  double* cbuf = lds + lm.chn;  // [2][64] shared by the workgroup
  // The chains' outputs of this wave's rows live in the wave's A-staging area (idle during the
  // chains): the steps store no vector memory (a store in the step loop made the compiler drain
  // the chain-block prefetch at every step); publish() writes delta / e out with sc1 stores once
  // per chain, spread over the wave's lanes.  rc_config keeps the area >= (2N + 3) rows.
  double* hist = asb;                    // [N + 2][nr]: delta_k (chain_fwd), then e_k (chain_bwd)
  double* whist = asb + (N + 2) * nr;    // [N + 1][nr]: w_k[dx] from chain_fwd's G rows
  auto publish = [&](int off, int k0, int k1) __attribute__((always_inline)) {  // k in [k0, k1)
    wsync();
    const int cnt = (k1 - k0) * nr;
    for (int t = lane; t < cnt; t += 64) {
      const int kk = t / nr, j = t - kk * nr;
      st_sc1<SC>(rchv, off + (k0 + kk) * X + r0 + j, hist[(k0 + kk) * nr + j]);
    }
  };

  auto reduce_row = [&](double p) __attribute__((always_inline)) {
    // sum of the NS partials of this lane's row (its NS lanes are one aligned group of a quad)
    if constexpr (NS >= 2) p = dpp_add<0xB1>(p);  // quad_perm [1, 0, 3, 2]
    if constexpr (NS >= 4) p = dpp_add<0x4E>(p);  // quad_perm [2, 3, 0, 1]
    return p;
  };

  // Each chain runs in blocks of PD steps whose slots refill unconditionally (fetches past the
  // end are clamped to valid nodes), then a tail without refills: no skipped step inside the
  // refilling loop, so the compiler's wait counts follow the PD-deep prefetch (a conditional step
  // there merged skip paths into the loop state and it waited for the newest loads every step).
  auto chain_fwd = [&]() __attribute__((always_inline)) {
    double2 rg[PD][SG / 2];
    double u1[PD], u2[PD];
    // per-lane offsets (constant over the steps) from wave-uniform bases: saddr + voffset loads;
    // load k of the wave is one contiguous run of LF 16-byte entries
    const int boff = wv * (SG / 2) * LF + min(lane, LF - 1);
    const int o1 = (cF ? 4 : 5) * L + crow, o2 = 3 * L + crow;
    auto fetch = [&](int s, int i) __attribute__((always_inline)) {
      const int ig = min(i, N);  // F rows are not used at step N (its block holds G_N only)
      const double2* pp = reinterpret_cast<const double2*>(CH + (size_t)ig * MP.node);
#pragma unroll
      for (int k = 0; k < SG / 2; ++k) rg[s][k] = gld(pp, boff + k * LF);
      u1[s] = ld_sc1<SC>(rchv, ig * X + o1);        // c'_i (F rows) / h'_i (G rows)
      u2[s] = ld_sc1<SC>(rchv, (ig + 1) * X + o2);  // a2_i
    };
    auto step = [&](int s, int i, bool refill) __attribute__((always_inline)) {
      CSUB(-1);
      const double2* dc = reinterpret_cast<const double2*>(cbuf + (i & 1) * 64) + cs * (SG / 2);
      double p0 = 0.0, p1 = 0.0;
#pragma unroll
      for (int k = 0; k < SG / 2; ++k) {
        const double2 t = dc[k];
        if (k & 1) p1 += rg[s][k].x * t.x + rg[s][k].y * t.y;
        else p0 += rg[s][k].x * t.x + rg[s][k].y * t.y;
      }
      CSUB(0);
      const double sum = reduce_row(p0 + p1);
      if (cs == 0 && cvalid) {
        if (cF) {
          if (i < N) {
            const double de = (u1[s] - sum) - u2[s];
            cbuf[((i + 1) & 1) * 64 + crow] = de;
            hist[(i + 1) * nr + cj] = de;
          }
        } else {
          whist[i * nr + cj] = u1[s] - sum;  // w_i[dx], read back by this wave's chain_bwd
        }
      }
      // the refill after the slot's last use: old and new values are never live together, so
      // the compiler keeps one register set per slot (no latch copies that wait for the refill)
      CSUB(1);
      __builtin_amdgcn_sched_barrier(0);
      if (refill) fetch(s, i + PD);
      CSUB(2);
      lds_barrier();
      CSUB(3);
    };
    int z0;  // an opaque 0: keeps the prologue's (iteration-invariant) addresses out of registers across phases
    asm volatile("s_mov_b32 %0, 0" : "=s"(z0));
#pragma unroll
    for (int s = 0; s < PD; ++s) fetch(s, s + z0);
    if (wv == 0) {
      cbuf[lane] = 0.0;  // delta_0
      cbuf[64 + lane] = 0.0;  // the padding columns [X, XP) of both buffers stay 0
      if (lane < X) st_sc1<SC>(rchv, oDL + lane, 0.0);
    }
    lds_barrier();
    int i0 = 0;
    for (; i0 + PD <= N + 1; i0 += PD) {
#pragma unroll
      for (int s = 0; s < PD; ++s) step(s, i0 + s, true);
    }
#pragma unroll
    for (int s = 0; s < PD; ++s)
      if (i0 + s <= N) step(s, i0 + s, false);
    publish(oDL, 1, N + 1);  // delta_1 .. delta_N (delta_0 = 0 went out in the prologue)
  };

  auto chain_bwd = [&]() __attribute__((always_inline)) {
    double2 rg[PD][SG / 2];
    const int boff = MP.fwd / 2 + wv * (SG / 2) * LB + min(lane, LB - 1);
    auto fetch = [&](int s, int i) __attribute__((always_inline)) {
      const int ic = max(i, 1);
      const double2* pp = reinterpret_cast<const double2*>(CH + (size_t)ic * MP.node);
#pragma unroll
      for (int k = 0; k < SG / 2; ++k) rg[s][k] = gld(pp, boff + k * LB);
    };
    auto step = [&](int s, int i, bool refill) __attribute__((always_inline)) {
      const double2* ec = reinterpret_cast<const double2*>(cbuf + ((i + 1) & 1) * 64) + cs * (SG / 2);
      double p0 = 0.0, p1 = 0.0;
#pragma unroll
      for (int k = 0; k < SG / 2; ++k) {
        const double2 t = ec[k];
        if (k & 1) p1 += rg[s][k].x * t.x + rg[s][k].y * t.y;
        else p0 += rg[s][k].x * t.x + rg[s][k].y * t.y;
      }
      const double w = whist[i * nr + cj];
      const double sum = reduce_row(p0 + p1);
      if (cF && cs == 0 && cvalid) {
        const double e = w - sum;
        cbuf[(i & 1) * 64 + crow] = e;
        hist[i * nr + cj] = e;
      }
      __builtin_amdgcn_sched_barrier(0);  // the refill after the slot's last use (chain_fwd)
      if (refill) fetch(s, i - PD);
      lds_barrier();
    };
    int z0;
    asm volatile("s_mov_b32 %0, 0" : "=s"(z0));
#pragma unroll
    for (int s = 0; s < PD; ++s) fetch(s, N - 1 - s + z0);
    if (cF && cs == 0 && cvalid) {
      const double e = whist[N * nr + cj];
      cbuf[(N & 1) * 64 + crow] = e;
      st_sc1<SC>(rchv, oEE + N * X + crow, e);
    }
    lds_barrier();
    int j0 = 0;  // e_i for i = N-1 .. 1: steps j = N - 1 - i
    for (; j0 + PD <= N - 1; j0 += PD) {
#pragma unroll
      for (int s = 0; s < PD; ++s) step(s, N - 1 - (j0 + s), true);
    }
#pragma unroll
    for (int s = 0; s < PD; ++s)
      if (j0 + s < N - 1) step(s, N - 1 - (j0 + s), false);
    publish(oEE, 1, N);  // e_1 .. e_{N-1} (e_N went out in the prologue)
  };

  // optional phase timing (PL_ADMM_TIMING=1: s_memtime on wave 0 of workgroup 0, cycles into
  // d.dbg[b][0..5]): P, C1, P2, C2, P3, barrier / hand-off waits
  const bool tim = d.dbg != nullptr && g == 0;
  unsigned long long tacc[6] = {0, 0, 0, 0, 0, 0}, tl = 0;
  auto T = [&](int slot) __attribute__((always_inline)) {
    if (tim) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      if (slot >= 0) tacc[slot] += now - tl;
      tl = now;
    }
  };
  // ---- hand-offs between the node phases (all workgroups) and the chains (workgroup 0).
  // Returns false on every wave of the workgroup when a poll gave up.
  auto drain = [&]() __attribute__((always_inline)) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's sc1 stores have reached L2
    __syncthreads();
  };
  auto poll_all = [&](int word, unsigned target, unsigned code) __attribute__((always_inline)) {
    if (wv == 0) {
      const bool ok = rc_poll(sy, word, target, code);
      if (lane == 0) *okw = ok ? 1 : 0;
    }
    __syncthreads();
    return *okw != 0;
  };
  auto give_up = [&]() __attribute__((always_inline)) {  // poison the problem's x: its solve reports NaN
    if (threadIdx.x == 0) xa[0] = __builtin_nan("");
  };
  // fan-in e (e = 1: the first P, e = it + 2: iteration it's P3): false if workgroup 0 gave up
  auto fan_in = [&](unsigned e) __attribute__((always_inline)) {
    if (G == 1) {
      drain();  // the sc1 stores have reached L2 before another wave's sc1 loads
      return true;
    }
    drain();
    if (g != 0) {
      if (threadIdx.x == 0) __hip_atomic_fetch_add((gu32*)(sy + RC_ARRIVE), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return true;
    }
    return poll_all(RC_ARRIVE, (unsigned)(G - 1) * e, 0x100u + e);
  };
  // fan-out of iteration it's chains (workgroup 0 publishes, the others wait)
  auto fan_out = [&](int it) __attribute__((always_inline)) {
    if (G == 1) {
      drain();
      return true;
    }
    if (g == 0) {
      drain();
      if (threadIdx.x == 0) __hip_atomic_store((gu32*)(sy + RC_EPOCH), (unsigned)(it + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      return true;
    }
    return poll_all(RC_EPOCH, (unsigned)(it + 1), 0x10000u + (unsigned)it);
  };
  const int i0 = g * W + wv, istep = G * W;  // this wave's nodes
  T(-1);
  if (g == 0 && wv == 0 && lane < ndx) st_sc1<SC>(rchv, oA2 + lane, 0.0);  // a2_{-1}
  for (int i = i0; i <= N; i += istep) pnode(i, 0, false);
  T(0);
  if (!fan_in(1)) { give_up(); return; }
  T(5);
  for (int it = 0; it < niter; ++it) {
    if (g == 0) {
      chain_fwd();  // C1 (+ w_i[dx], formerly P2)
      T(1);
      __syncthreads();
      T(5);
      chain_bwd();  // C2
      T(3);
    }
    if (!fan_out(it)) { give_up(); return; }
    T(5);
    const bool lastit = it == niter - 1;
    for (int i = i0; i <= N; i += istep) pnode(i, lastit ? 2 : 1, check && lastit);
    T(4);
    if (!fan_in((unsigned)it + 2)) { give_up(); return; }
    T(5);
  }
  if (g != 0) return;
  if (tim && wv == 0 && lane == 0) {
    for (int k = 0; k < 6; ++k) d.dbg[(size_t)b * 16 + k] += (double)tacc[k];
    d.dbg[(size_t)b * 16 + 6] += niter;
#if PL_RC_SUBTIMING
    for (int k = 0; k < 7; ++k) d.dbg[(size_t)b * 16 + 8 + k] += (double)sacc[k];
    if (b == 0)
      for (int k = 0; k < 4; ++k) d.dbg[16 + k] += (double)cacc[k];  // B = 1 runs: chain_fwd step sub-phases
#endif
  }
  // the complete rhs for the next launch / kernel: rhs_i[dx] += a2_{i-1} (workgroup 0, all nodes)
  for (int i = wv; i <= N; i += W) {
    if (i >= 1 && lane < ndx) {
      const int c = an[i].x_off + lane;
      rhs[c] = ld_sc1<SC>(rrhs, c) + ld_sc1<SC>(rchv, oA2 + i * ndx + lane);
    }
  }
  if (wv == 0 && lane == 0) {
    info->iter += niter;
    info->iter_prof += niter;
  }
}

namespace {

struct RcCfg {
  RcLds lm;
  int w;
  size_t lds;
};

RcCfg rc_config(const PlOcpHandle* h, int w) {
  RcCfg c{};
  RcLds& lm = c.lm;
  auto up2 = [](int x) { return (x + 1) & ~1; };
  lm.prog_dbl = up2((h->aprog_len + 3) / 4);
  lm.chn = lm.prog_dbl;  // then [2][64] chain buffers and the 2-double poll word
  const int T = h->ntile_max;
  int o = 0;
  lm.v = o;
  o += up2(4 * T);
  lm.y = o;
  o += up2(h->nw_max + h->ndx);
  lm.acc = o;
  o += up2(std::max(std::max(5 * T, h->nrow_max), h->ncol_max));
  lm.trow = o;
  o += up2(std::max(h->nrow_max, 1));
  lm.tcpl = o;
  o += 64;
  lm.bc = o;
  o += 64;
  lm.asb = o;
  c.w = w;
  const int budget = 160 * 1024 / 8;
  int cap = ((budget - lm.prog_dbl - 130) / w - o - 2) & ~1;
  cap = std::max(0, std::min(up2(std::max(h->nent_max, 1)), cap));
  lm.asb_cap = cap;
  lm.per_wave = o + cap + 2;  // + the 16-byte alignment shift of the A staging DMA
  c.lds = (size_t)(lm.prog_dbl + 130 + w * lm.per_wave) * sizeof(double);
  return c;
}

template <int W, int X>
void launch_rc_t(PlOcpHandle* h, int niter, int check, const RcCfg& c) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)k_admm_rc<W, X, true>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    hipFuncSetAttribute((const void*)k_admm_rc<W, X, false>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const int G = rc_groups(h);
  if (G > 1) (void)hipMemsetAsync(h->d.rcsync, 0, (size_t)h->B * PL_RC_SYNC * sizeof(unsigned), h->stream);
  if (G > 1)
    hipLaunchKernelGGL((k_admm_rc<W, X, true>), dim3(h->B * G), dim3(64 * W), c.lds, h->stream, h->d, h->N, h->n, h->m,
                       h->nnz, h->S_stride, std::max(h->ncpl_max, 1), h->ch_stride, h->chv_stride, c.lm, niter, check,
                       h->set.sigma, h->set.alpha, G);
  else
    hipLaunchKernelGGL((k_admm_rc<W, X, false>), dim3(h->B), dim3(64 * W), c.lds, h->stream, h->d, h->N, h->n, h->m,
                       h->nnz, h->S_stride, std::max(h->ncpl_max, 1), h->ch_stride, h->chv_stride, c.lm, niter, check,
                       h->set.sigma, h->set.alpha, 1);
}

}  // namespace

long long rc_ch_stride(int N, int ndx, int W) { return (long long)(N + 1) * rc_map(ndx, W).node; }

// Workgroups per problem of k_admm_rc: enough for one round of node phases, as long as the
// batch's workgroups are all resident at once (one per CU: the kernel's LDS), which the
// in-launch hand-offs require.
int rc_groups(const PlOcpHandle* h) {
  if ((h->debug_paths & PL_PATH_RC_ONE_GROUP) || !h->d.rcsync) return 1;
  const int W = h->rc_waves;
  int G = (h->N + W) / W;  // ceil((N + 1) / W)
  while (G > 1 && (long long)h->B * G > h->num_cu) --G;
  return std::max(G, 1);
}
int rc_chv_stride(int N, int ndx) { return 6 * (N + 2) * ndx; }

bool admm_rc_supported(const PlOcpHandle* h) {
  // the chain blocks F_i = C_i S_i[:, dx] assume one coupling row per dx_{i+1} column
  return !h->fac_gc && (h->ndx == 24 || h->ndx == 30 || h->ndx == 36 || h->ndx == 48) && (h->rc_waves == 4 || h->rc_waves == 8) && h->nw_max <= 64 * MV && h->nrow_max <= 64 * MR && h->ncpl_max <= 64 &&
         rc_config(h, h->rc_waves).lds <= 160 * 1024 &&
         rc_config(h, h->rc_waves).lm.asb_cap >= (2 * h->N + 3) * ((h->ndx + h->rc_waves - 1) / h->rc_waves);  // chain history
}

void launch_fred(PlOcpHandle* h) {
  const size_t lds = (size_t)(h->nw_max + h->ndx) * h->ndx * sizeof(double);
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)k_fred, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(k_fred, dim3(h->B * (h->N + 1)), dim3(256), lds, h->stream, h->d, h->N, h->nnz, h->ndx,
                     h->S_stride, std::max(h->ncpl_max, 1), h->ch_stride, rc_map(h->ndx, h->rc_waves));
}

void launch_admm_rc(PlOcpHandle* h, int niter, int check) {
  const RcCfg c = rc_config(h, h->rc_waves);
  switch (h->ndx * 16 + h->rc_waves) {
    case 24 * 16 + 4: launch_rc_t<4, 24>(h, niter, check, c); break;
    case 30 * 16 + 4: launch_rc_t<4, 30>(h, niter, check, c); break;
    case 30 * 16 + 8: launch_rc_t<8, 30>(h, niter, check, c); break;
    case 36 * 16 + 4: launch_rc_t<4, 36>(h, niter, check, c); break;
    case 48 * 16 + 4: launch_rc_t<4, 48>(h, niter, check, c); break;
    case 24 * 16 + 8: launch_rc_t<8, 24>(h, niter, check, c); break;
    case 36 * 16 + 8: launch_rc_t<8, 36>(h, niter, check, c); break;
    case 48 * 16 + 8: launch_rc_t<8, 48>(h, niter, check, c); break;
    default: break;
  }
}
