// ADMM sweeps (OSQP 0.6 osqp_solve loop body, src/osqp.c: update_xz_tilde,
// update_x, update_z, update_y) -- ONE WAVE PER PROBLEM.
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
// Schedule of one launch (every step consumes exactly one factor block S_i):
//     F0 | { FWD 1..N-1, TN, BWD N-1..1, T0 } x niter   (the last T0 is B0)
// TN fuses forward N and backward N (x~_N = w_N, so S_N is read once); T0 fuses
// backward 0 with the next iteration's forward 0 (S_0 stays in registers).  Per
// iteration 2N factor blocks are streamed instead of 2(N+1).
//
// MI355X mapping.  The kernel streams the factor (4.14 MB algorithmic per problem-iteration
// for B2G whole_body_rnea N=50, 4.69 MB measured with the tile padding and vector gathers),
// so the design goal is to keep the whole batch resident with one factor block per problem
// in flight:
//   * one 64-lane wave per problem, PPW problems per workgroup: 1024 problems =
//     256 workgroups x 4 waves = one wave per SIMD on every CU, all resident
//     (the previous 256-thread-per-problem kernel fit only 2 problems per CU and
//     ran the batch in two rounds);
//   * no s_barrier in the sweep: all cross-lane exchange goes through the wave's
//     private LDS region (in-order LDS, wave-scope fences only);
//   * S_i is streamed through a register double buffer (PL_ADMM_KM 4x4 tile slots
//     per lane, 1 KiB-contiguous 16-byte loads): step q issues the loads of step
//     q+1's block before it touches its own, so every block has a whole step of
//     latency cover; the small operands of step q+1 follow the same pipeline;
//   * every distinct node program (u16 gather lists) is LDS-resident for the whole
//     launch and shared by the PPW waves.
// The symmetric mat-vec uses the packed lower 4x4 tiles: each tile gives 4 row
// partials (accumulated per lane over the lane's run of tiles in a tile row) and, off the
// diagonal, 4 column partials; both go straight into a per-wave LDS accumulator with
// ds_add_f64 (PL_ADMM_ATOMIC, r02e; the segment / column-partial arrays of r01 remain as
// the #else branch).  The backward step's A x~ and A^T (rho z - y) are chunked CSR / CSC
// gathers (entry-order scatters into LDS row / column sums were measured slower in r04 and
// removed).  The lanes of one ds_add instruction and the instructions
// of one wave apply in a fixed order, so results are bit-identical for a problem
// regardless of the batch or workgroup it runs in.
#include <algorithm>
#include <type_traits>

#include "admm_common.h"
#include "state.h"

namespace {

using namespace admm;

struct Sbuf {
  double2 s[KM][8];
};
// operands of a step needed at its start (double-buffered across steps)
struct Early {
  double acw[CWM];  // forward: A of the w part of coupling row `lane` of node i-1
  double axc[XCM];  // forward: A of the coupling entries of dx_i column `lane`
  double rhoc;      // rho of coupling row `lane` (node i-1 forward, node i backward)
  double vv[MV];    // forward: rhs_i, backward: bt_i (columns lane, lane + 64)
  uint4 tt;         // lane-tile table words of the step's factor block (k_factor layout)
};
struct LateR {  // backward rows of node i (lane, lane + 64, lane + 128)
  double z[MR], y[MR], rho[MR], l[MR], u[MR];
};
struct LateC {  // backward columns of node i
  double x[MV], q[MV];
};

// Per-wave LDS carve-up (offsets in doubles from the wave's region).
struct AdmmLds {
  int prog_dbl;  // all ADMM programs (u16), rounded to 16 bytes, in doubles
  int per_wave;
  int v, y, xn, r1, tcpl, trow, red, colp, zero, asb, asb_cap;
};

}  // namespace

template <int PPW, int ASR, bool TIMING, bool NT>
__global__ __launch_bounds__(64 * PPW, 1) void k_admm(PlDev d, int B, int N, int n, int m, int nnz, int ndx,
                                                      int S_stride, int cpl_stride, AdmmLds lm, int niter, int check,
                                                      int fwd_asb, double sigma, double alpha) {
  extern __shared__ double lds[];
  {  // every node program, shared by the waves of the workgroup
    const uint4* src = reinterpret_cast<const uint4*>(d.aprog);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    for (int k = threadIdx.x; k < lm.prog_dbl / 2; k += 64 * PPW) dst[k] = src[k];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform: scalar bases
  const int b = blockIdx.x * PPW + wv;
  if (b >= B) return;
  PlProbInfo* info = d.info + b;
  if (info->done) return;
  // optional phase timing (s_memtime, per wave) into d.dbg[b][0..15]
  unsigned long long tacc[TIMING ? 14 : 1] = {}, tlast = 0;
  auto T = [&](int slot) __attribute__((always_inline)) {
    if constexpr (TIMING) {
      const unsigned long long now = __builtin_amdgcn_s_memtime();
      if (slot >= 0) tacc[slot] += now - tlast;
      tlast = now;
    }
  };
  const uint16_t* PG = reinterpret_cast<const uint16_t*>(lds);
  double* W = lds + lm.prog_dbl + wv * lm.per_wave;
  double* v = W + lm.v;        // mat-vec input (zero padded to 4 T)
  double* y = W + lm.y;        // mat-vec output; backward: [x~_i | x~_{i+1}(dx)]
  double* xn = W + lm.xn;      // x~_{i+1} (dx part) across backward steps
  double* r1 = W + lm.r1;      // rhs_1 (dx part) completed by T0, read by the next forward 1
  double* tcpl = W + lm.tcpl;  // coupling-row products (before the mat-vec; aliases `red`)
  double* trow = W + lm.trow;  // rho z - y of the node's rows (after the mat-vec; aliases `red`)
  double* seg = W + lm.red;    // mat-vec row segments [(lane + I) * 4 + r]
  double* colp = W + lm.colp;  // mat-vec column partials, off-diagonal tiles in column-major order
  double* part = W + lm.red;   // chunk sums of the row / column gathers (after the mat-vec)
  double* asb = W + lm.asb;    // A values of the backward node
  double* zslot = W + lm.zero; // a 0.0 read by the clamped reductions
  if (lane == 0) *zslot = 0.0;

  const double* __restrict__ As = d.As + (size_t)b * nnz;
  const double* __restrict__ rho = d.rho + (size_t)b * m;
  const double* __restrict__ rhoc = d.rhoc + (size_t)b * (N + 1) * cpl_stride;
  const double* __restrict__ Acp = d.Acpl + (size_t)b * (N + 1) * PL_ACPL;
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
  // NT: the batch's factor far exceeds the 256 MB Infinity Cache (admm_config), so the streams
  // (factor blocks, A, the row / column operands) are non-temporal loads; below it the sweeps'
  // re-reads partly hit the cache and plain loads are kept (Go2 centroidal_vel at B = 1024:
  // 328 MB of factor, nt was 2 % slower)
  // node table: uniform reads through the constant address space are scalar loads
  typedef const __attribute__((address_space(4))) PlAdmmNode* CNode;
  CNode an = (CNode)d.anodes;
  const int Q = 1 + niter * 2 * N;

  // Software pipeline.  Step q opens with its one vector-memory wait (vmcnt(0): everything
  // issued during step q-1, its stores included), then issues, in this order: the row /
  // column operands of step q+1 (LR, LC -- right after their step-q copies become current),
  // the deferred end-of-step stores of step q-1, the A staging, then the other step q+1
  // operands (E, las) and the factor block of step q+1 slot by slot inside its own mat-vec.
  // So the wait at a step's start is for data issued a whole step earlier.
  //
  // Invariant that makes it safe to read step q+1's LR / LC BEFORE step q-1's deferred stores
  // are issued (requires N >= 2, which pl_ocp_create enforces).  LR / LC are consumed only by
  // a backward step (rows z, y, rho, l, u and columns x, q of node i1) or TN (columns of node
  // N).  Step q-1's pending stores are bt_i (forward), or z, y, x of node i and rhs of nodes
  // i, i + 1 (backward / TN / T0).  The schedule F0 | FWD 1..N-1, TN, BWD N-1..1, T0 moves one
  // node per step, so a consumed prefetch could meet a pending store only at a turn: at
  // FWD N-1 -> TN -> BWD N-1 step q-1 is forward and stores only bt, which LR / LC never read;
  // at BWD 1 -> T0 -> FWD 1 step q+1 is forward and consumes no LR / LC.  (With N = 1,
  // TN -> T0 -> TN would read x of node N before the first TN's store of it.)  The other
  // operands of step q+1 (E, las) are issued after the stores, in order.
  Sbuf SR;  // factor slots of the current block; refilled with the next block's as they are consumed
  Early E, En;  // current / next step (the copy at the start of a step is its only vmcnt wait)
  double las[ASR];
  LateR LR, LRn;
  LateC LC, LCn;
  double rkeep = 0.0;           // rhs of node i (dx part, lane < ndx) completed at node i-1
  double2 r0v = make_double2(0.0, 0.0);  // rhs_0 of the backward-0 half of T0 (columns lane, lane + 64)
  bool fix1 = false;

  // ---------------- loads (unconditional and clamped: exact vmcnt accounting)
  auto load_S = [&](int i, int kbase, Sbuf& R) __attribute__((always_inline)) {
    const int K = an[i].nunit;
    const double2* p = reinterpret_cast<const double2*>(Sg + an[i].s_off);
#pragma unroll
    for (int k = 0; k < KM; ++k) {
      const int kk = min(kbase + k, K - 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) R.s[k][j] = gldx<NT>(p, (kk * 8 + j) * 64 + lane);
    }
  };
  auto prefetch_E = [&](int kind1, int i1, Early& E) __attribute__((always_inline)) {
    const bool fw = kind1 == KFWD || kind1 == KTN;
    const int g = fw ? i1 - 1 : i1;
    const int ncp = an[g].ncpl;
    const int s = min(lane, max(ncp - 1, 0));
    {  // coupling A values through registers, contiguous per node (d.Acpl, k_acpl)
      const double* Ac = Acp + (size_t)g * PL_ACPL;
      const int o1 = fw ? lane * CWM : 0, o2 = fw ? 64 * CWM + lane * XCM : 0;  // backward: unused, one line
#pragma unroll
      for (int k = 0; k < CWM; ++k) E.acw[k] = gld(Ac, o1 + k);
#pragma unroll
      for (int k = 0; k < XCM; ++k) E.axc[k] = gld(Ac, o2 + k);
    }
    E.rhoc = gld(rhoc, g * cpl_stride + s);
    E.tt = gld(reinterpret_cast<const uint4*>(d.ttab), max(an[i1].ttab, 0) / 4 + lane);
    const double* src = (kind1 == KF0 || fw) ? rhs : bt;
    const int xo = an[i1].x_off, nw1 = an[i1].nw;
#pragma unroll
    for (int mm = 0; mm < MV; ++mm) E.vv[mm] = gld(src, xo + min(lane + 64 * mm, nw1 - 1));
  };
  auto prefetch_as = [&](int kind1, int i1) __attribute__((always_inline)) {
    // backward steps: A of node i1; forward steps with dense coupling rows: A of node i1 - 1
    const bool fa = fwd_asb && (kind1 == KFWD || kind1 == KTN);
    const bool bw = bwd_kind(kind1) || fa;
    const int ia = fa ? i1 - 1 : i1;
    const int eo = an[ia].ent_off, ne = an[ia].nent;
#pragma unroll
    for (int k = 0; k < ASR; ++k) las[k] = gldx<NT>(As, eo + (bw ? min(lane + 64 * k, ne - 1) : 0));
  };
  auto prefetch_LR = [&](int kind1, int i1, LateR& LR) __attribute__((always_inline)) {
    const bool bw = bwd_kind(kind1);
    const int ro = an[i1].row_off, nr = an[i1].nrow;
#pragma unroll
    for (int mm = 0; mm < MR; ++mm) {
      const int r = ro + (bw ? min(lane + 64 * mm, max(nr - 1, 0)) : 0);
      LR.z[mm] = gldx<NT>(za, r);
      LR.y[mm] = gldx<NT>(ya, r);
      LR.rho[mm] = gldx<NT>(rho, r);
      LR.l[mm] = gldx<NT>(ls, r);
      LR.u[mm] = gldx<NT>(us, r);
    }
  };
  auto prefetch_LC = [&](int kind1, int i1, LateC& LC) __attribute__((always_inline)) {
    const bool need = bwd_kind(kind1) || kind1 == KTN;
    const int xo = an[i1].x_off, nw1 = an[i1].nw;
#pragma unroll
    for (int mm = 0; mm < MV; ++mm) {
      const int j = xo + (need ? min(lane + 64 * mm, nw1 - 1) : 0);
      LC.x[mm] = gldx<NT>(xa, j);
      LC.q[mm] = gldx<NT>(qs, j);
    }
  };

  // ---------------- y[0..nw) = S_i v  (R holds slots 0..KM-1 unless reload).  Slot k
  // of node next's block is loaded into R as soon as the last pass has consumed slot
  // k (the software pipeline of the factor stream; next = i re-reads the block).
  auto matvec = [&](Sbuf& R, int i, bool reload, int next, uint4 tt) __attribute__((always_inline)) {
    const int K = an[i].nunit, T = an[i].ntile, ntl = an[i].ntl, nw = an[i].nw;
    const int Kn = an[next].nunit;
    const double2* pn = reinterpret_cast<const double2*>(Sg + an[next].s_off);
    const unsigned km = an[i].kmagic;
    const double2* v2 = reinterpret_cast<const double2*>(v);
    int curI = -1;
    double sa[4] = {0.0, 0.0, 0.0, 0.0};
    bool use_tt = false;
#if PL_ADMM_ATOMIC
    // accumulate y in LDS with ds_add_f64 (no return, no dependent round trips):
    // output 4 I + r lives at acc5[5 I + r] (a stride of 5 doubles spreads the banks)
    double* acc5 = seg;
    for (int o = lane; o < 5 * T; o += 64) acc5[o] = 0.0;
    wsync();
    auto emit_row = [&](int I0) __attribute__((always_inline)) {
#pragma unroll
      for (int r = 0; r < 4; ++r) lds_add(acc5 + I0 * 5 + r, sa[r]);
    };
#else
    auto emit_row = [&](int I0) __attribute__((always_inline)) {
      double2* sp = reinterpret_cast<double2*>(seg + (lane + I0) * 4);
      sp[0] = make_double2(sa[0], sa[1]);
      sp[1] = make_double2(sa[2], sa[3]);
    };
#endif
    auto pass = [&](int kb, bool last_pass) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < KM; ++k) {
        const int kk = kb + k;
        const int t = K * lane + kk;
        int I, J, cidx;
        bool valid;
        if (use_tt) {  // precomputed (uniform choice)
          const uint32_t w = k == 0 ? tt.x : (k == 1 ? tt.y : (k == 2 ? tt.z : tt.w));
          I = (int)(w >> 24);
          J = (int)((w >> 16) & 0xff);
          cidx = (int)(w & 0xffff);
          valid = I != 0xff;
        } else {
          valid = kk < K && t < ntl;
          tile_ij(t, I, J);
          cidx = (J * (2 * T - J - 1)) / 2 + I - J - 1;
        }
        if (valid) {
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
#if PL_ADMM_ATOMIC
            (void)cidx;
#pragma unroll
            for (int c = 0; c < 4; ++c) lds_add(acc5 + J * 5 + c, cp[c]);
#else
            // column-major packed off-diagonal index: the partials of one output tile
            // column are contiguous
            double2* cpp = reinterpret_cast<double2*>(colp + cidx * 4);
            cpp[0] = make_double2(cp[0], cp[1]);
            cpp[1] = make_double2(cp[2], cp[3]);
#endif
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
        if (last_pass) {  // uniform; always true for blocks of <= KM slots per lane
          const int kq = min(k, Kn - 1);
#pragma unroll
          for (int j = 0; j < 8; ++j) R.s[k][j] = gldx<NT>(pn, (kq * 8 + j) * 64 + lane);
        }
      }
    };
    if (K <= KM && !reload) {
      use_tt = true;
      pass(0, true);  // the common case, straight-line: the refill loads never force a wait
    } else {
      // blocks with more than KM slots per lane: slots 0..KM-1 are already in R (the
      // previous step's refill) unless `reload`; the rest load synchronously
      for (int kb = 0; kb < K; kb += KM) {
        if (kb > 0 || reload) load_S(i, kb, R);
        pass(kb, kb + KM >= K);
      }
    }
    if (curI >= 0) emit_row(curI);
    wsync();
#if PL_ADMM_ATOMIC
    (void)km;
#pragma unroll
    for (int mm = 0; mm < MV; ++mm) {
      const int o = lane + 64 * mm;
      if (o < nw) y[o] = acc5[(o >> 2) * 5 + (o & 3)];
    }
#else
#pragma unroll
    for (int mm = 0; mm < MV; ++mm) {
      const int o = lane + 64 * mm;
      if (o < nw) {
        const int I = o >> 2, r = o & 3;
        const int t0 = I * (I + 1) / 2;
        const int lf = div_k(t0, K, km), ll = div_k(t0 + I, K, km);
        const double rs = lds_sum(seg + I * 4 + r, lf, ll + 1, 4, zslot);
        const int cb = (I * (2 * T - I - 1)) / 2;
        const double cs = lds_sum(colp + r, cb, cb + T - 1 - I, 4, zslot);
        y[o] = rs + cs;
      }
    }
#endif
    wsync();
  };

  // ---------------- the stores of a step (bt of a forward step; rows z, y (dy) and columns x
  // (dx), rhs of a backward step).  They are issued right after the next step's wait, from
  // registers carried across the boundary, so that wait covers only loads and the stores retire
  // behind a whole step (stores count in vmcnt; issued at the step's end, as until r04, the
  // next wait also waited for them: profiles/r04o, 24.12 -> 23.46 ms per launch).
  struct StoreSet {
    double kz[MR], ky[MR], kd[MR], kb[MV];
    double2 pxa, pdx, prh;
    double prn;
    int kind, i;
    bool delta;
  };
  StoreSet pend;
  pend.kind = -1;
  auto issue_stores = [&](const StoreSet& ss) __attribute__((always_inline)) {
    const int kind = ss.kind, i = ss.i;
    const bool bw = bwd_kind(kind);
    const int nw = an[i].nw, x_off = an[i].x_off;
    if (!bw || kind == KT0) {  // bt_i of a forward (part of a) step
#pragma unroll
      for (int mm = 0; mm < MV; ++mm)
        if (lane + 64 * mm < nw) gst(bt, x_off + lane + 64 * mm, ss.kb[mm]);
    }
    if (bw) {  // rows of node i
      const int nrow = an[i].nrow, ro = an[i].row_off;
#pragma unroll
      for (int mm = 0; mm < MR; ++mm) {
        const int r = lane + 64 * mm;
        if (r < nrow) {
          gst(za, ro + r, ss.kz[mm]);
          gst(ya, ro + r, ss.ky[mm]);
          if (ss.delta) gst(dys, ro + r, ss.kd[mm]);
        }
      }
    }
    if (bw || kind == KTN) {  // x update and rhs of node i
      const int xnx = bw ? an[i + 1].x_off : 0;
#pragma unroll
      for (int mm = 0; mm < MV; ++mm) {
        const int c = lane + 64 * mm;
        if (c < nw) {
          gst(xa, x_off + c, sel2(ss.pxa, mm));
          if (ss.delta) gst(dxs, x_off + c, sel2(ss.pdx, mm));
          if (bw) {
            if (c < ndx) gst(rhs, xnx + c, ss.prn);
            if (!(c < ndx && i > 0)) gst(rhs, x_off + c, sel2(ss.prh, mm));
          }
        }
      }
    }
  };

  // ---------------- one step of the schedule
  auto step = [&](int q) __attribute__((always_inline)) {
    // No store is issued mid-step: on CDNA4 a store's source VGPRs may be reused only after
    // its vmcnt retires, so a mid-step store followed by register reuse would wait and drain
    // the factor stream.  The step's results go out after the next step's vmcnt(0).
    double kz[MR], ky[MR], kd[MR], kb[MV];
#pragma unroll
    for (int mm = 0; mm < MR; ++mm) kz[mm] = ky[mm] = kd[mm] = 0.0;
#pragma unroll
    for (int mm = 0; mm < MV; ++mm) kb[mm] = 0.0;
    double2 pxa = make_double2(0.0, 0.0), pdx = pxa, prh = pxa;
    double prn = 0.0;
    int i, it;
    const int kind = step_kind(q, N, niter, i, it);
    const bool has_next = q + 1 < Q;
    int i1 = 0, it1 = 0;
    const int kind1 = has_next ? step_kind(q + 1, N, niter, i1, it1) : kind;
    if (!has_next) i1 = i;
    const bool bw = bwd_kind(kind);
    const bool store_delta = check && it == niter - 1;
    const int nw = an[i].nw, x_off = an[i].x_off, T4 = 4 * an[i].ntile;
    const int eo = an[i].ent_off, ne = an[i].nent;
    const double* __restrict__ Ai = As + eo;
    const int cap = lm.asb_cap;
    const uint16_t* P = PG + an[i].prog;
    auto stage = [&](int ns, const double* __restrict__ src) __attribute__((always_inline)) {
#pragma unroll
      for (int k = 0; k < ASR; ++k) {
        const int e = lane + 64 * k;
        if (e < ns && e < cap) asb[e] = las[k];
      }
      for (int e = 64 * ASR + lane; e < min(ns, cap); e += 64) asb[e] = src[e];
      wsync();
    };
    // gathers over A: LDS only when the node's A fits (uniform), else LDS + global
    // (the overflow path ends with vmcnt(0) so its global loads never leave pending
    // state behind for the wait-count bookkeeping of the common path)
    auto with_A = [&](int ns, const double* __restrict__ src, auto body) __attribute__((always_inline)) {
      if (ns <= cap) {
        body([&](int e) __attribute__((always_inline)) { return asb[e]; });
      } else {
        typedef const __attribute__((address_space(1))) double* GPtr;
        const GPtr gs = (GPtr)src;
        body([&](int e) __attribute__((always_inline)) { return e < cap ? asb[e] : gs[e]; });
        __builtin_amdgcn_s_waitcnt(0xF70);
      }
    };
    T(-1);
    // ---- start: everything prefetched for this step becomes current (the one wait),
    // this step's A goes to LDS, then the previous step's deferred stores
    __builtin_amdgcn_s_waitcnt(0xF70);  // vmcnt(0): step q-1's loads (and stores) are done
    T(10);
    E = En;
    LR = LRn;
    LC = LCn;
    // the next step's row / column operands right away: a whole step of cover (r05; issued after
    // the mat-vec / the row gathers until r04, the x update then waited ~2 k cycles for them)
    prefetch_LR(kind1, i1, LRn);
    T(11);
    prefetch_LC(kind1, i1, LCn);
    T(12);
    if (pend.kind >= 0) issue_stores(pend);  // step q-1's stores, behind its wait
    T(13);
    if (bw) stage(ne, Ai);
    else if (fwd_asb && kind != KF0) stage(an[i - 1].nent, As + an[i - 1].ent_off);
    T(0);
    T(1);
    if (bw) {
      with_A(ne, Ai, [&](auto A) __attribute__((always_inline)) {
        // ---- t_s = rho_s a_s(dx_{i+1}) . x~_{i+1}
        const int ncp = an[i].ncpl;
        if (lane < ncp) {
          const uint32_t* cx = reinterpret_cast<const uint32_t*>(P + an[i].cxp);
          const int q0 = P[an[i].cxptr + lane], q1 = P[an[i].cxptr + lane + 1];
          const double acc = range_sum<2>(q0, q1, [&](int qq) {
            const uint32_t w = cx[qq];
            return A(w & 0xffff) * xn[w >> 16];
          });
          tcpl[lane] = E.rhoc * acc;
        }
        wsync();
        // ---- v = bt_i - A_{c,w_i}^T t
        const uint32_t* cc = reinterpret_cast<const uint32_t*>(P + an[i].ccp);
#pragma unroll
        for (int mm = 0; mm < MV; ++mm) {
          const int c = lane + 64 * mm;
          if (c < nw) {
            const int q0 = P[an[i].ccptr + c], q1 = P[an[i].ccptr + c + 1];
            v[c] = E.vv[mm] - range_sum<4>(q0, q1, [&](int qq) {
                     const uint32_t w = cc[qq];
                     return A(w & 0xffff) * tcpl[w >> 16];
                   });
          } else if (c < T4) {
            v[c] = 0.0;
          }
        }
      });
      if (lane < ndx) y[nw + lane] = xn[lane];  // x~_{i+1} (dx) behind x~_i for the row gathers
      wsync();
    } else if (kind == KF0) {
#pragma unroll
      for (int mm = 0; mm < MV; ++mm) {
        const int c = lane + 64 * mm;
        if (c < nw) {
          kb[mm] = E.vv[mm];
          v[c] = E.vv[mm];
        } else if (c < T4) {
          v[c] = 0.0;
        }
      }
      wsync();
    } else {  // KFWD, KTN: coupling rows of node g = i - 1
      const int g = i - 1;
      const uint16_t* Pg = PG + an[g].prog;
      const int ncp = an[g].ncpl;
      const double* __restrict__ Ag = As + an[g].ent_off;
      const bool fx = fix1 && i == 1;
      fix1 = false;
      auto fwd_gathers = [&](auto A, bool dense) __attribute__((always_inline)) {
        if (lane < ncp) {  // t_s = rho_s a_s(w_{i-1}) . w_{i-1}
          const uint32_t* cw = reinterpret_cast<const uint32_t*>(Pg + an[g].cwp);
          const int q0 = Pg[an[g].cwptr + lane], q1 = Pg[an[g].cwptr + lane + 1];
          double acc = 0.0;
          if (dense) {
            for (int qq = q0; qq < q1; ++qq) {
              const uint32_t w = cw[qq];
              acc += A(w & 0xffff) * y[w >> 16];
            }
          } else {
#pragma unroll
            for (int k = 0; k < CWM; ++k)
              if (q0 + k < q1) acc += E.acw[k] * y[cw[q0 + k] >> 16];
          }
          tcpl[lane] = E.rhoc * acc;
        }
        wsync();
        const uint32_t* xc = reinterpret_cast<const uint32_t*>(Pg + an[g].xcp);
#pragma unroll
        for (int mm = 0; mm < MV; ++mm) {
          const int c = lane + 64 * mm;
          if (c < nw) {  // bt_i = rhs_i - A_{c,dx_i}^T t
            double vv = (fx && c < ndx) ? r1[c] : E.vv[mm];
            if (c < ndx) {
              const int q0 = Pg[an[g].xcptr + c], q1 = Pg[an[g].xcptr + c + 1];
              if (dense) {
                for (int qq = q0; qq < q1; ++qq) {
                  const uint32_t w = xc[qq];
                  vv -= A(w & 0xffff) * tcpl[w >> 16];
                }
              } else {
#pragma unroll
                for (int k = 0; k < XCM; ++k)
                  if (q0 + k < q1) vv -= E.axc[k] * tcpl[xc[q0 + k] >> 16];
              }
            }
            kb[mm] = vv;
            v[c] = vv;
          } else if (c < T4) {
            v[c] = 0.0;
          }
        }
      };
      if (fwd_asb) with_A(an[g].nent, Ag, [&](auto A) __attribute__((always_inline)) { fwd_gathers(A, true); });
      else fwd_gathers([&](int e) __attribute__((always_inline)) { return asb[e]; }, false);
      wsync();
    }
    // ---- operands of step q+1 (this step's E and las are consumed), then w_i / x~_i
    // with the factor block of step q+1 streamed in behind the mat-vec
    T(2);
    prefetch_E(kind1, i1, En);
    prefetch_as(kind1, i1);
    T(3);
    matvec(SR, i, false, kind == KT0 ? i : i1, E.tt);
    T(4);
    if (bw) {
      with_A(ne, Ai, [&](auto A) __attribute__((always_inline)) {
        // ---- z~ = A x~
        {
          const uint16_t* rowe = P + an[i].rowe;
          const uint8_t* rowc = reinterpret_cast<const uint8_t*>(P + an[i].rowc);
          const uint32_t* rch = reinterpret_cast<const uint32_t*>(P + an[i].rch);
          const int rchn = an[i].rchn;
#if PL_ADMM_ATOMIC
          const uint8_t* rchr = reinterpret_cast<const uint8_t*>(P + an[i].rchr);
          for (int o = lane; o < an[i].nrow; o += 64) part[o] = 0.0;  // row sums, by LDS f64 adds
          wsync();
#endif
          for (int c0 = 0; c0 < rchn; c0 += 128) {  // two rounds of chunks per batch
            double acc[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              const int ch = c0 + lane + 64 * u;
              const uint32_t cw = rch[min(ch, rchn - 1)];
              const int q0 = cw & 0xffff, len = ch < rchn ? (int)(cw >> 16) - q0 : 0;
              double a = 0.0;
#pragma unroll
              for (int k = 0; k < PL_CHUNK; ++k) {
                const int qq = q0 + min(k, max(len - 1, 0));
                const double t = A(rowe[qq]) * y[rowc[qq]];
                a += k < len ? t : 0.0;
              }
              acc[u] = a;
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              const int ch = c0 + lane + 64 * u;
#if PL_ADMM_ATOMIC
              if (ch < rchn) lds_add(part + rchr[ch], acc[u]);
#else
              if (ch < rchn) part[ch] = acc[u];
#endif
            }
          }
        }
        wsync();
        T(5);
        // ---- update_z, update_y (relaxed)
        {
          const int nrow = an[i].nrow, ro = an[i].row_off, rcp = an[i].rchptr;
#pragma unroll
          for (int mm = 0; mm < MR; ++mm) {
            const int r = lane + 64 * mm;
            if (r < nrow) {
#if PL_ADMM_ATOMIC
              (void)rcp;
              const double zt = part[r];
#else
              const int k0 = P[rcp + r], k1 = P[rcp + r + 1];
              const double zt = lds_sum<4>(part, k0, k1, 1, zslot);
#endif
              const double zrel = alpha * zt + (1.0 - alpha) * LR.z[mm];
              double zn = zrel + (1.0 / LR.rho[mm]) * LR.y[mm];
              zn = fmin(fmax(zn, LR.l[mm]), LR.u[mm]);
              const double dy = LR.rho[mm] * (zrel - zn);
              const double yn = LR.y[mm] + dy;
              trow[r] = LR.rho[mm] * zn - yn;
              kz[mm] = zn;
              ky[mm] = yn;
              kd[mm] = dy;
            }
          }
        }
        wsync();
        T(6);
        // ---- A^T (rho z - y)
        {
          const uint8_t* colr = reinterpret_cast<const uint8_t*>(P + an[i].colr);
          const uint32_t* cch = reinterpret_cast<const uint32_t*>(P + an[i].cch);
          const int cchn = an[i].cchn;
#if PL_ADMM_ATOMIC
          // column sums by LDS f64 adds (the z update's reads of `part` are ahead in LDS order)
          const uint8_t* cchc = reinterpret_cast<const uint8_t*>(P + an[i].cchc);
          for (int o = lane; o < an[i].ncol; o += 64) part[o] = 0.0;
          wsync();
#endif
          for (int c0 = 0; c0 < cchn; c0 += 128) {  // two rounds of chunks per batch
            double acc[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              const int ch = c0 + lane + 64 * u;
              const uint32_t cw = cch[min(ch, cchn - 1)];
              const int e0 = cw & 0xffff, len = ch < cchn ? (int)(cw >> 16) - e0 : 0;
              double a = 0.0;
#pragma unroll
              for (int k = 0; k < PL_CHUNK; ++k) {
                const int e = e0 + min(k, max(len - 1, 0));
                const double t = A(e) * trow[colr[e]];
                a += k < len ? t : 0.0;
              }
              acc[u] = a;
            }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              const int ch = c0 + lane + 64 * u;
#if PL_ADMM_ATOMIC
              if (ch < cchn) lds_add(part + cchc[ch], acc[u]);
#else
              if (ch < cchn) part[ch] = acc[u];
#endif
            }
          }
        }
      });
      wsync();
      T(7);
      // ---- update_x and the next rhs = sigma x - q + A^T (rho z - y) (stores deferred)
      {
        const int ccp0 = an[i].cchptr;
#pragma unroll
        for (int mm = 0; mm < MV; ++mm) {
          const int c = lane + 64 * mm;
          if (c < nw) {
            const double xnew = alpha * y[c] + (1.0 - alpha) * LC.x[mm];
            set2(pxa, mm, xnew);
            set2(pdx, mm, xnew - LC.x[mm]);
            double acc = sigma * xnew - LC.q[mm];
#if PL_ADMM_ATOMIC
            (void)ccp0;
            acc += part[c];
#else
            const int k0 = P[ccp0 + c], k1 = P[ccp0 + c + 1];
            acc += lds_sum<4>(part, k0, k1, 1, zslot);
#endif
            if (c < ndx) {  // rows of node i on dx_{i+1} complete rhs_{i+1}
#if PL_ADMM_ATOMIC
              const double a2 = part[nw + c];
#else
              const int f0 = P[ccp0 + nw + c], f1 = P[ccp0 + nw + c + 1];
              const double a2 = lds_sum<4>(part, f0, f1, 1, zslot);
#endif
              prn = rkeep + a2;
              if (i == 0) r1[c] = prn;
            }
            set2(prh, mm, acc);
            if (c < ndx && i > 0) rkeep = acc;
            set2(r0v, mm, acc);
            if (c < ndx) xn[c] = y[c];
          }
        }
      }
    } else if (kind == KTN) {
      // ---- backward N: x~_N = w_N; node N has no rows
#pragma unroll
      for (int mm = 0; mm < MV; ++mm) {
        const int c = lane + 64 * mm;
        if (c < nw) {
          const double xnew = alpha * y[c] + (1.0 - alpha) * LC.x[mm];
          set2(pxa, mm, xnew);
          set2(pdx, mm, xnew - LC.x[mm]);
          rkeep = sigma * xnew - LC.q[mm];
          xn[c] = y[c];
        }
      }
    }
    T(8);
    if (kind == KT0) {
      // ---- forward 0 of the next iteration with the same S_0
      wsync();
#pragma unroll
      for (int mm = 0; mm < MV; ++mm) {
        const int c = lane + 64 * mm;
        if (c < nw) {
          kb[mm] = sel2(r0v, mm);
          v[c] = sel2(r0v, mm);
        } else if (c < T4) {
          v[c] = 0.0;
        }
      }
      wsync();
      matvec(SR, 0, an[0].nunit > KM, i1, E.tt);
      fix1 = true;
    }
    wsync();
    // ---- the step's stores (now, or deferred behind the next step's wait)
    {
      StoreSet cur;
#pragma unroll
      for (int mm = 0; mm < MR; ++mm) { cur.kz[mm] = kz[mm]; cur.ky[mm] = ky[mm]; cur.kd[mm] = kd[mm]; }
#pragma unroll
      for (int mm = 0; mm < MV; ++mm) cur.kb[mm] = kb[mm];
      cur.pxa = pxa; cur.pdx = pdx; cur.prh = prh; cur.prn = prn;
      cur.kind = kind; cur.i = i; cur.delta = store_delta;
      pend = cur;
    }
    T(9);
  };

  prefetch_E(KF0, 0, En);  // operands of step 0 (F0)
  prefetch_as(KF0, 0);
  prefetch_LR(KF0, 0, LRn);
  prefetch_LC(KF0, 0, LCn);
  load_S(0, 0, SR);
  for (int q = 0; q < Q; ++q) step(q);
  issue_stores(pend);
  if (lane == 0) {
    info->iter += niter;
    info->iter_prof += niter;  // only problems still iterating reach here (done ones return above)
  }
  if constexpr (TIMING) {
    if (lane == 0 && d.dbg)
      for (int k = 0; k < 14; ++k) d.dbg[(size_t)b * 16 + k] += (double)tacc[k];
  }
}

// Compact coupling A values of node i (one 64-lane block per (problem, node)), refreshed with
// every factorisation: the forward step of the sweep gathers, per coupling row s, the A values
// of its w part (cw list, PL_ADMM_CWM clamped slots) and, per dx_{i+1} column c, those of its
// coupling entries (xc list, PL_ADMM_XCM slots).  Gathered from As they touch up to the
// node's whole A slice (~56 lines of 128 B) for ~150 values; here they are 1.5 KB contiguous.
__global__ __launch_bounds__(64) void k_acpl(PlDev d, int N, int nnz, int ndx) {
  const int b = blockIdx.x / (N + 1), i = blockIdx.x - b * (N + 1);
  if (ip_skip(d, b)) return;
  const int lane = threadIdx.x;
  const PlAdmmNode& a = d.anodes[i];
  double* out = d.Acpl + ((size_t)b * (N + 1) + i) * PL_ACPL;
  const double* As = d.As + (size_t)b * nnz + a.ent_off;
  const uint16_t* P = d.aprog + a.prog;
  const int ncp = a.ncpl;
  {
    const int s = min(lane, max(ncp - 1, 0));
    const int q0 = ncp ? P[a.cwptr + s] : 0, cnt = ncp ? P[a.cwptr + s + 1] - q0 : 0;
    const uint32_t* cw = reinterpret_cast<const uint32_t*>(P + a.cwp);
    for (int k = 0; k < PL_ADMM_CWM; ++k)
      out[lane * PL_ADMM_CWM + k] = cnt > 0 ? As[cw[q0 + min(k, cnt - 1)] & 0xffff] : 0.0;
  }
  {
    const int c = min(lane, ndx - 1);
    const int q0 = a.ncol ? P[a.xcptr + c] : 0, cnt = a.ncol ? P[a.xcptr + c + 1] - q0 : 0;
    const uint32_t* xc = reinterpret_cast<const uint32_t*>(P + a.xcp);
    for (int k = 0; k < PL_ADMM_XCM; ++k)
      out[64 * PL_ADMM_CWM + lane * PL_ADMM_XCM + k] = cnt > 0 ? As[xc[q0 + min(k, cnt - 1)] & 0xffff] : 0.0;
  }
}

void launch_acpl(PlOcpHandle* h) {
  hipLaunchKernelGGL(k_acpl, dim3(h->B * (h->N + 1)), dim3(64), 0, h->stream, h->d, h->N, h->nnz, h->ndx);
}

namespace {

struct AdmmCfg {
  AdmmLds lm;
  int ppw;
  size_t lds;
  bool nt;  // non-temporal streams: the batch's factor > 2 x the 256 MB Infinity Cache
};

AdmmCfg admm_config(const PlOcpHandle* h) {
  AdmmCfg c{};
  AdmmLds& lm = c.lm;
  auto up2 = [](int x) { return (x + 1) & ~1; };
  lm.prog_dbl = up2((h->aprog_len + 3) / 4);
  const int T = h->ntile_max;
  int o = 0;
  lm.v = o;
  o += up2(4 * T);
  lm.y = o;
  o += up2(h->nw_max + h->ndx);
  lm.xn = o;
  o += up2(h->ndx);
  lm.zero = o;
  o += 2;
  lm.r1 = o;
  o += up2(h->ndx);
  // `red` is time-shared: coupling products (gathers) | mat-vec segments and column
  // partials (mat-vec) | chunk sums and rho z - y (row / column gathers)
  lm.red = o;
  lm.tcpl = o;
#if PL_ADMM_ATOMIC
  const int matv = 5 * T;  // the mat-vec accumulator acc5 (no segments, no column partials)
  lm.colp = o;
#else
  const int segn = (64 + T) * 4;
  const int matv = segn + T * (T - 1) / 2 * 4;
  lm.colp = o + segn;
#endif
  // `part` holds the chunk sums (chunked gathers) or the row / column sums (scatters)
  const int partn = up2(std::max(h->chunk_max, std::max(h->nrow_max, h->ncol_max)));
  lm.trow = o + partn;
  o += up2(std::max(std::max(matv, partn + h->nrow_max), std::max(h->ncpl_max, 1)));
  lm.asb = o;
  // problems per workgroup: 4 puts one wave on every SIMD of every CU once B >= 4 x 256
  c.ppw = h->B >= 1024 ? 4 : (h->B >= 512 ? 2 : 1);
  const int budget = 160 * 1024 / 8;
  int cap = ((budget - lm.prog_dbl) / c.ppw - o) & ~1;
  cap = std::max(0, std::min(up2(std::max(h->nent_max, 1)), cap));
  lm.asb_cap = cap;
  lm.per_wave = o + cap;
  c.lds = (size_t)(lm.prog_dbl + c.ppw * lm.per_wave) * sizeof(double);
  c.nt = (double)h->B * h->S_stride * sizeof(double) > 512.0 * 1024 * 1024;
  return c;
}

template <int PPW, int ASR, bool TIMING, bool NT>
void launch_admm_nt(PlOcpHandle* h, int niter, int check, const AdmmCfg& c) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)k_admm<PPW, ASR, TIMING, NT>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const int grid = (h->B + PPW - 1) / PPW;
  hipLaunchKernelGGL((k_admm<PPW, ASR, TIMING, NT>), dim3(grid), dim3(64 * PPW), c.lds, h->stream, h->d, h->B, h->N,
                     h->n, h->m, h->nnz, h->ndx, h->S_stride, std::max(h->ncpl_max, 1), c.lm, niter, check,
                     h->admm_fwd_asb, h->set.sigma, h->set.alpha);
}

template <int PPW, int ASR, bool TIMING = false>
void launch_admm_t(PlOcpHandle* h, int niter, int check, const AdmmCfg& c) {
  if (c.nt) launch_admm_nt<PPW, ASR, TIMING, true>(h, niter, check, c);
  else launch_admm_nt<PPW, ASR, TIMING, false>(h, niter, check, c);
}

template <int ASR>
void launch_admm_a(PlOcpHandle* h, int niter, int check, const AdmmCfg& c) {
  if (c.ppw == 4 && ASR == 16 && h->d.dbg) launch_admm_t<4, 16, true>(h, niter, check, c);  // phase timing
  else if (c.ppw == 4) launch_admm_t<4, ASR>(h, niter, check, c);
  else if (c.ppw == 2) launch_admm_t<2, ASR>(h, niter, check, c);
  else launch_admm_t<1, ASR>(h, niter, check, c);
}

}  // namespace

int admm_lds_bytes(const PlOcpHandle* h) { return (int)admm_config(h).lds; }

int admm_ppw(const PlOcpHandle* h) { return admm_config(h).ppw; }

int admm_asb_cap(const PlOcpHandle* h) { return admm_config(h).lm.asb_cap; }

void launch_admm(PlOcpHandle* h, int niter, int check, int it_base) {
  (void)it_base;
  const AdmmCfg c = admm_config(h);
  const bool prof = h->profile && h->prof_n < 64;
  if (prof) hipEventRecord(h->prof_ev[h->prof_n][0], h->stream);
  if (h->admm_rc) launch_admm_rc(h, niter, check);
  else if (h->admm_waves == 2 && !h->d.dbg) launch_admm2(h, niter, check);
  else if (h->admm_asr <= 16) launch_admm_a<16>(h, niter, check, c);
  else launch_admm_a<32>(h, niter, check, c);
  if (prof) {
    hipEventRecord(h->prof_ev[h->prof_n][1], h->stream);
    h->prof_n++;
  }
}
