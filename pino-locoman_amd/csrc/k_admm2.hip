// ADMM sweeps with TWO WAVES PER PROBLEM (same algorithm and schedule as k_admm.hip:
// OSQP 0.6 update_xz_tilde / update_x / update_z / update_y over the block factor).
//
// Why: the one-wave kernel is latency-bound (≈24 k cycles per step, of which only
// ≈1.4 k wait on the factor stream; every phase is a chain of LDS round trips) and at
// B = 1024 it places one wave on each SIMD, so nothing hides that latency.  Here the
// two waves of a problem split every phase of a step and each SIMD holds two waves:
//   * factor block: wave h owns the tile slots kk = h, h + 2, ... of every lane (half
//     the register buffer, half the 16-byte loads);
//   * mat-vec: per-wave row-segment arrays (zero-filled over the lane's tile rows, so
//     a segment the other wave owns reads as 0) and shared per-tile column partials;
//     wave h reduces the outputs lane + 64 h;
//   * columns (v, x update, rhs): c = lane + 64 h; rows (z / y update): lane + 64 (2 j + h);
//     row / column chunk gathers: chunk lane + 64 h of every 128;
//   * the coupling products t_s (<= 64 values) are computed by both waves into
//     per-wave copies (no barrier).
// The phases are separated by workgroup barriers (PPW problems x 2 waves per
// workgroup share the LDS-resident node programs); the schedule is uniform across
// the workgroup, and waves of terminated or padding problems keep hitting the same
// barriers without doing work.
//
// Selection (api.hip::admm_select, AUTO): the reduced-chain kernel k_admm_rc up to
// B = 256 problems where it supports the OCP, this kernel for B <= 512, k_admm above.
// Measured: at B = 1024 this kernel is slower than k_admm (26.3 vs 25.2 ms per launch,
// r02e; the two waves of a SIMD compete for the same VALU issue and the 7-9 barriers per
// step add latency), at B = 512 it is faster (15.2 vs 18.5 ms: k_admm leaves half the
// SIMDs idle there).  PL_ADMM_KERNEL=sweep2 / pl_ocp_set_admm_kernel force it.
#include <algorithm>
#include <type_traits>

#include "admm_common.h"
#include "state.h"

namespace {

using namespace admm;
constexpr int KH = 2;  // factor tile slots per lane held in registers by each wave

struct Sbuf2 {
  double2 s[KH][8];
};
struct Early2 {
  double acw[CWM];
  double axc[XCM];
  double rhoc;
  double vv;        // forward: rhs_i, backward: bt_i (column lane + 64 h)
  uint2 tt;         // lane-tile table words of this wave's slots (h, h + 2)
};
struct LateR2 {  // rows lane + 64 (2 j + h), j < 2
  double z[2], y[2], rho[2], l[2], u[2];
};
struct LateC2 {  // column lane + 64 h
  double x, q;
};

// Workgroup barrier that orders LDS only.  __syncthreads() fences global memory at
// workgroup scope, i.e. waits vmcnt(0): that would drain the factor stream the
// kernel keeps in flight across a whole step.  Here: this wave's LDS operations are
// complete (lgkmcnt(0)), then s_barrier; the wave-scope fences keep the compiler from
// moving memory operations across it.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

struct AdmmLds2 {
  int prog_dbl;
  int per_prob;
  int v, y, xn, r1, red, segn, colp, trow, zero, asb, asb_cap, accn;
};

}  // namespace

template <int PPW, int ASR>
__global__ __launch_bounds__(128 * PPW, 1) void k_admm2(PlDev d, int B, int N, int n, int m, int nnz, int ndx,
                                                        int S_stride, int cpl_stride, AdmmLds2 lm, int niter, int check,
                                                        int fwd_asb, double sigma, double alpha) {
  extern __shared__ double lds[];
  {
    const uint4* src = reinterpret_cast<const uint4*>(d.aprog);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    for (int k = threadIdx.x; k < lm.prog_dbl / 2; k += 128 * PPW) dst[k] = src[k];
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int pw = wv >> 1, h = wv & 1;
  const int b = blockIdx.x * PPW + pw;
  // every wave runs the schedule (barriers); `act` problems do the work
  const bool act = __builtin_amdgcn_readfirstlane((b < B && !d.info[min(b, B - 1)].done) ? 1 : 0) != 0;
  const int bb = min(b, B - 1);
  PlProbInfo* info = d.info + bb;
  const uint16_t* PG = reinterpret_cast<const uint16_t*>(lds);
  double* W = lds + lm.prog_dbl + pw * lm.per_prob;
  double* v = W + lm.v;
  double* y = W + lm.y;
  double* xn = W + lm.xn;
  double* r1 = W + lm.r1;
  double* tcpl = W + lm.red + 64 * h;          // this wave's copy of the coupling products
  double* segh = W + lm.red + lm.segn * h;     // this wave's mat-vec row segments
  double* seg0 = W + lm.red;
  double* seg1 = W + lm.red + lm.segn;
  double* colp = W + lm.colp;
  double* part = W + lm.red;
  double* trow = W + lm.trow;
  // PL_ADMM_ATOMIC: per-wave LDS f64-add accumulators (the mat-vec outputs, then the row
  // and column sums); the two waves' halves are added in a fixed order, so the sums stay
  // deterministic
  double* acch = W + lm.red + lm.accn * h;
  double* acc0 = W + lm.red;
  double* acc1 = W + lm.red + lm.accn;
  double* asb = W + lm.asb;
  double* zslot = W + lm.zero;
  if (lane == 0 && h == 0) *zslot = 0.0;

  const double* __restrict__ As = d.As + (size_t)bb * nnz;
  const double* __restrict__ rho = d.rho + (size_t)bb * m;
  const double* __restrict__ rhoc = d.rhoc + (size_t)bb * (N + 1) * cpl_stride;
  const double* __restrict__ Acp = d.Acpl + (size_t)bb * (N + 1) * PL_ACPL;
  const double* __restrict__ ls = d.ls + (size_t)bb * m;
  const double* __restrict__ us = d.us + (size_t)bb * m;
  const double* __restrict__ qs = d.qs + (size_t)bb * n;
  const double* __restrict__ Sg = d.S + (size_t)bb * S_stride;
  double* za = d.za + (size_t)bb * m;
  double* ya = d.ya + (size_t)bb * m;
  double* xa = d.xa + (size_t)bb * n;
  double* rhs = d.rhs + (size_t)bb * n;
  double* bt = d.bt + (size_t)bb * n;
  double* dxs = d.dxs + (size_t)bb * n;
  double* dys = d.dys + (size_t)bb * m;
  typedef const __attribute__((address_space(4))) PlAdmmNode* CNode;
  CNode an = (CNode)d.anodes;
  const int Q = 1 + niter * 2 * N;
  const int cl = lane + 64 * h;  // this wave's column of every node

  Sbuf2 SR;
  Early2 E, En;
  double las[ASR];  // A entries lane + 64 (2 k + h) of the next staged node
  LateR2 LR, LRn;
  LateC2 LC, LCn;
  double rkeep = 0.0;
  double r0v = 0.0;
  bool fix1 = false;

  auto load_S = [&](int i, int j0, Sbuf2& R) __attribute__((always_inline)) {
    const int K = an[i].nunit;
    const double2* p = reinterpret_cast<const double2*>(Sg + an[i].s_off);
#pragma unroll
    for (int k = 0; k < KH; ++k) {
      const int kk = min(2 * (j0 + k) + h, K - 1);
#pragma unroll
      for (int j = 0; j < 8; ++j) R.s[k][j] = gld(p, (kk * 8 + j) * 64 + lane);
    }
  };
  auto prefetch_E = [&](int kind1, int i1, Early2& E) __attribute__((always_inline)) {
    const bool fw = kind1 == KFWD || kind1 == KTN;
    const int g = fw ? i1 - 1 : i1;
    const int ncp = an[g].ncpl;
    const int s = min(lane, max(ncp - 1, 0));
    {  // coupling A values, contiguous per node (d.Acpl, k_acpl)
      const double* Ac = Acp + (size_t)g * PL_ACPL;
      const int o1 = fw ? lane * CWM : 0, o2 = fw ? 64 * CWM + lane * XCM : 0;  // backward: unused, one line
#pragma unroll
      for (int k = 0; k < CWM; ++k) E.acw[k] = gld(Ac, o1 + k);
#pragma unroll
      for (int k = 0; k < XCM; ++k) E.axc[k] = gld(Ac, o2 + k);
    }
    E.rhoc = gld(rhoc, g * cpl_stride + s);
    {
      const uint4 t4 = gld(reinterpret_cast<const uint4*>(d.ttab), max(an[i1].ttab, 0) / 4 + lane);
      E.tt = h == 0 ? make_uint2(t4.x, t4.z) : make_uint2(t4.y, t4.w);
    }
    const double* src = (kind1 == KF0 || fw) ? rhs : bt;
    const int xo = an[i1].x_off, nw1 = an[i1].nw;
    E.vv = gld(src, xo + min(cl, nw1 - 1));
  };
  auto prefetch_as = [&](int kind1, int i1) __attribute__((always_inline)) {
    const bool fa = fwd_asb && (kind1 == KFWD || kind1 == KTN);
    const bool bw = bwd_kind(kind1) || fa;
    const int ia = fa ? i1 - 1 : i1;
    const int eo = an[ia].ent_off, ne = an[ia].nent;
#pragma unroll
    for (int k = 0; k < ASR; ++k) las[k] = gld(As, eo + (bw ? min(lane + 64 * (2 * k + h), ne - 1) : 0));
  };
  auto prefetch_LR = [&](int kind1, int i1, LateR2& LR) __attribute__((always_inline)) {
    const bool bw = bwd_kind(kind1);
    const int ro = an[i1].row_off, nr = an[i1].nrow;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = ro + (bw ? min(lane + 64 * (2 * j + h), max(nr - 1, 0)) : 0);
      LR.z[j] = gld(za, r);
      LR.y[j] = gld(ya, r);
      LR.rho[j] = gld(rho, r);
      LR.l[j] = gld(ls, r);
      LR.u[j] = gld(us, r);
    }
  };
  auto prefetch_LC = [&](int kind1, int i1, LateC2& LC) __attribute__((always_inline)) {
    const bool need = bwd_kind(kind1) || kind1 == KTN;
    const int xo = an[i1].x_off, nw1 = an[i1].nw;
    const int j = xo + (need ? min(cl, nw1 - 1) : 0);
    LC.x = gld(xa, j);
    LC.q = gld(qs, j);
  };

  // ---------------- y[0..nw) = S_i v.  Wave h: slots kk = 2 j + h of every lane.
  auto matvec = [&](Sbuf2& R, int i, bool reload, int next, uint2 tt) __attribute__((always_inline)) {
    const int K = an[i].nunit, T = an[i].ntile, ntl = an[i].ntl, nw = an[i].nw;
    const int Kn = an[next].nunit;
    const double2* pn = reinterpret_cast<const double2*>(Sg + an[next].s_off);
    const unsigned km = an[i].kmagic;
    const double2* v2 = reinterpret_cast<const double2*>(v);
    if (act) {
#if PL_ADMM_ATOMIC
      for (int o = lane; o < 5 * T; o += 64) acch[o] = 0.0;
      wsync();
#else
      // zero the segments of every tile row the lane's run touches (the other wave may
      // own that row's tiles of this lane)
      {
        const int ta = K * lane, tb = min(K * lane + K, ntl) - 1;
        if (ta <= tb) {
          int Ia, Ja, Ib, Jb;
          tile_ij(ta, Ia, Ja);
          tile_ij(tb, Ib, Jb);
          for (int I = Ia; I <= Ib; ++I) {
            double2* sp = reinterpret_cast<double2*>(segh + (lane + I) * 4);
            sp[0] = make_double2(0.0, 0.0);
            sp[1] = make_double2(0.0, 0.0);
          }
        }
      }
#endif
      int curI = -1;
      double sa[4] = {0.0, 0.0, 0.0, 0.0};
      bool use_tt = false;
      auto emit_row = [&](int I0) __attribute__((always_inline)) {
#if PL_ADMM_ATOMIC
#pragma unroll
        for (int r = 0; r < 4; ++r) lds_add(acch + I0 * 5 + r, sa[r]);
#else
        double2* sp = reinterpret_cast<double2*>(segh + (lane + I0) * 4);
        sp[0] = make_double2(sa[0], sa[1]);
        sp[1] = make_double2(sa[2], sa[3]);
#endif
      };
      auto pass = [&](int j0, bool last_pass) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < KH; ++k) {
          const int kk = 2 * (j0 + k) + h;
          const int t = K * lane + kk;
          int I, J, cidx;
          bool valid;
          if (use_tt) {
            const uint32_t w = k == 0 ? tt.x : tt.y;
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
              for (int c = 0; c < 4; ++c) lds_add(acch + J * 5 + c, cp[c]);
#else
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
          if (last_pass) {
            const int kq = min(2 * k + h, Kn - 1);
#pragma unroll
            for (int j = 0; j < 8; ++j) R.s[k][j] = gld(pn, (kq * 8 + j) * 64 + lane);
          }
        }
      };
      const int nh = (K - h + 1) / 2;  // slots of this wave
      if (K <= 2 * KH && !reload) {
        use_tt = true;
        pass(0, true);
      } else {  // slots of pass 0 are in R already (the previous step's refill) unless `reload`
        for (int j0 = 0; j0 < max(nh, 1); j0 += KH) {
          if (j0 > 0 || reload) load_S(i, j0, R);
          pass(j0, j0 + KH >= nh);
        }
      }
      if (curI >= 0) emit_row(curI);
    }
    lds_barrier();
#if PL_ADMM_ATOMIC
    (void)km;
    if (act && cl < nw) {
      const int o = (cl >> 2) * 5 + (cl & 3);
      y[cl] = acc0[o] + acc1[o];
    }
#else
    if (act && cl < nw) {
      const int I = cl >> 2, r = cl & 3;
      const int t0 = I * (I + 1) / 2;
      const int lf = div_k(t0, K, km), ll = div_k(t0 + I, K, km);
      const double rs = lds_sum(seg0 + I * 4 + r, lf, ll + 1, 4, zslot) + lds_sum(seg1 + I * 4 + r, lf, ll + 1, 4, zslot);
      const int cb = (I * (2 * T - I - 1)) / 2;
      const double cs = lds_sum(colp + r, cb, cb + T - 1 - I, 4, zslot);
      y[cl] = rs + cs;
    }
#endif
    lds_barrier();
  };

  auto step = [&](int q) __attribute__((always_inline)) {
    double kz[2], ky[2], kd[2], kb = 0.0;
#pragma unroll
    for (int j = 0; j < 2; ++j) kz[j] = ky[j] = kd[j] = 0.0;
    double pxa = 0.0, pdx = 0.0, prh = 0.0, prn = 0.0;
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
        const int e = lane + 64 * (2 * k + h);
        if (e < ns && e < cap) asb[e] = las[k];
      }
      for (int e = 128 * ASR + 64 * h + lane; e < min(ns, cap); e += 128) asb[e] = src[e];
    };
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
    // ---- start: the step's prefetched operands become current (the one vmcnt wait),
    // the node's A values go to LDS
    __builtin_amdgcn_s_waitcnt(0xF70);
    E = En;
    LR = LRn;
    LC = LCn;
    if (act) {
      if (bw) stage(ne, Ai);
      else if (fwd_asb && kind != KF0) stage(an[i - 1].nent, As + an[i - 1].ent_off);
    }
    lds_barrier();
    if (bw) {
      if (act) {
        with_A(ne, Ai, [&](auto A) __attribute__((always_inline)) {
          // ---- t_s = rho_s a_s(dx_{i+1}) . x~_{i+1} (each wave its own copy)
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
          // ---- v = bt_i - A_{c,w_i}^T t (column cl)
          const uint32_t* cc = reinterpret_cast<const uint32_t*>(P + an[i].ccp);
          if (cl < nw) {
            const int q0 = P[an[i].ccptr + cl], q1 = P[an[i].ccptr + cl + 1];
            v[cl] = E.vv - range_sum<4>(q0, q1, [&](int qq) {
                      const uint32_t w = cc[qq];
                      return A(w & 0xffff) * tcpl[w >> 16];
                    });
          } else if (cl < T4) {
            v[cl] = 0.0;
          }
        });
        if (h == 0 && lane < ndx) y[nw + lane] = xn[lane];
      }
    } else if (kind == KF0) {
      if (act) {
        if (cl < nw) {
          kb = E.vv;
          v[cl] = E.vv;
        } else if (cl < T4) {
          v[cl] = 0.0;
        }
      }
    } else {  // KFWD, KTN: coupling rows of node g = i - 1
      const int g = i - 1;
      const uint16_t* Pg = PG + an[g].prog;
      const int ncp = an[g].ncpl;
      const double* __restrict__ Ag = As + an[g].ent_off;
      const bool fx = fix1 && i == 1;
      fix1 = false;
      auto fwd_gathers = [&](auto A, bool dense) __attribute__((always_inline)) {
        if (lane < ncp) {
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
        if (cl < nw) {
          double vv = (fx && cl < ndx) ? r1[cl] : E.vv;
          if (cl < ndx) {
            const int q0 = Pg[an[g].xcptr + cl], q1 = Pg[an[g].xcptr + cl + 1];
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
          kb = vv;
          v[cl] = vv;
        } else if (cl < T4) {
          v[cl] = 0.0;
        }
      };
      if (act) {
        if (fwd_asb) with_A(an[g].nent, Ag, [&](auto A) __attribute__((always_inline)) { fwd_gathers(A, true); });
        else fwd_gathers([&](int e) __attribute__((always_inline)) { return asb[e]; }, false);
      }
    }
    lds_barrier();  // v complete (and every read of the coupling products done)
    if (act) {
      prefetch_E(kind1, i1, En);
      prefetch_as(kind1, i1);
    }
    matvec(SR, i, false, kind == KT0 ? i : i1, E.tt);
    if (!bw && act) {
      prefetch_LR(kind1, i1, LRn);
      prefetch_LC(kind1, i1, LCn);
    }
    if (bw) {
      if (act) {
        with_A(ne, Ai, [&](auto A) __attribute__((always_inline)) {
          // ---- z~ = A x~ over row chunks (chunk lane + 64 h of every 128)
          const uint16_t* rowe = P + an[i].rowe;
          const uint8_t* rowc = reinterpret_cast<const uint8_t*>(P + an[i].rowc);
          const uint32_t* rch = reinterpret_cast<const uint32_t*>(P + an[i].rch);
          const int rchn = an[i].rchn;
#if PL_ADMM_ATOMIC
          const uint8_t* rchr = reinterpret_cast<const uint8_t*>(P + an[i].rchr);
          for (int o = lane; o < an[i].nrow; o += 64) acch[o] = 0.0;
          wsync();
#endif
          for (int c0 = 0; c0 < rchn; c0 += 128) {
            const int ch = c0 + cl;
            const uint32_t cw = rch[min(ch, rchn - 1)];
            const int q0 = cw & 0xffff, len = ch < rchn ? (int)(cw >> 16) - q0 : 0;
            double a = 0.0;
#pragma unroll
            for (int k = 0; k < PL_CHUNK; ++k) {
              const int qq = q0 + min(k, max(len - 1, 0));
              const double t = A(rowe[qq]) * y[rowc[qq]];
              a += k < len ? t : 0.0;
            }
#if PL_ADMM_ATOMIC
            if (ch < rchn) lds_add(acch + rchr[ch], a);
#else
            if (ch < rchn) part[ch] = a;
#endif
          }
        });
        prefetch_LR(kind1, i1, LRn);
        prefetch_LC(kind1, i1, LCn);
      }
      lds_barrier();
      // ---- update_z, update_y (rows lane + 64 (2 j + h))
      if (act) {
        const int nrow = an[i].nrow, rcp = an[i].rchptr;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int r = lane + 64 * (2 * j + h);
          if (r < nrow) {
#if PL_ADMM_ATOMIC
            (void)rcp;
            const double zt = acc0[r] + acc1[r];
#else
            const int k0 = P[rcp + r], k1 = P[rcp + r + 1];
            const double zt = lds_sum<4>(part, k0, k1, 1, zslot);
#endif
            const double zrel = alpha * zt + (1.0 - alpha) * LR.z[j];
            double zn = zrel + (1.0 / LR.rho[j]) * LR.y[j];
            zn = fmin(fmax(zn, LR.l[j]), LR.u[j]);
            const double dy = LR.rho[j] * (zrel - zn);
            const double yn = LR.y[j] + dy;
            trow[r] = LR.rho[j] * zn - yn;
            kz[j] = zn;
            ky[j] = yn;
            kd[j] = dy;
          }
        }
      }
      lds_barrier();
      // ---- A^T (rho z - y) over column chunks
      if (act) {
        with_A(ne, Ai, [&](auto A) __attribute__((always_inline)) {
          const uint8_t* colr = reinterpret_cast<const uint8_t*>(P + an[i].colr);
          const uint32_t* cch = reinterpret_cast<const uint32_t*>(P + an[i].cch);
          const int cchn = an[i].cchn;
#if PL_ADMM_ATOMIC
          const uint8_t* cchc = reinterpret_cast<const uint8_t*>(P + an[i].cchc);
          for (int o = lane; o < an[i].ncol; o += 64) acch[o] = 0.0;
          wsync();
#endif
          for (int c0 = 0; c0 < cchn; c0 += 128) {
            const int ch = c0 + cl;
            const uint32_t cw = cch[min(ch, cchn - 1)];
            const int e0 = cw & 0xffff, len = ch < cchn ? (int)(cw >> 16) - e0 : 0;
            double a = 0.0;
#pragma unroll
            for (int k = 0; k < PL_CHUNK; ++k) {
              const int e = e0 + min(k, max(len - 1, 0));
              const double t = A(e) * trow[colr[e]];
              a += k < len ? t : 0.0;
            }
#if PL_ADMM_ATOMIC
            if (ch < cchn) lds_add(acch + cchc[ch], a);
#else
            if (ch < cchn) part[ch] = a;
#endif
          }
        });
      }
      lds_barrier();
      // ---- update_x and the next rhs = sigma x - q + A^T (rho z - y) (column cl)
      if (act && cl < nw) {
        const int ccp0 = an[i].cchptr;
        const double xnew = alpha * y[cl] + (1.0 - alpha) * LC.x;
        pxa = xnew;
        pdx = xnew - LC.x;
        double acc = sigma * xnew - LC.q;
#if PL_ADMM_ATOMIC
        (void)ccp0;
        acc += acc0[cl] + acc1[cl];
#else
        const int k0 = P[ccp0 + cl], k1 = P[ccp0 + cl + 1];
        acc += lds_sum<4>(part, k0, k1, 1, zslot);
#endif
        if (cl < ndx) {
#if PL_ADMM_ATOMIC
          const double a2 = acc0[nw + cl] + acc1[nw + cl];
#else
          const int f0 = P[ccp0 + nw + cl], f1 = P[ccp0 + nw + cl + 1];
          const double a2 = lds_sum<4>(part, f0, f1, 1, zslot);
#endif
          prn = rkeep + a2;
          if (i == 0) r1[cl] = prn;
        }
        prh = acc;
        if (cl < ndx && i > 0) rkeep = acc;
        r0v = acc;
        if (cl < ndx) xn[cl] = y[cl];
      }
    } else if (kind == KTN) {
      if (act && cl < nw) {
        const double xnew = alpha * y[cl] + (1.0 - alpha) * LC.x;
        pxa = xnew;
        pdx = xnew - LC.x;
        rkeep = sigma * xnew - LC.q;
        xn[cl] = y[cl];
      }
    }
    if (kind == KT0) {
      // ---- forward 0 of the next iteration with the same S_0
      if (act) {
        if (cl < nw) {
          kb = r0v;
          v[cl] = r0v;
        } else if (cl < T4) {
          v[cl] = 0.0;
        }
      }
      lds_barrier();
      matvec(SR, 0, an[0].nunit > 2 * KH, i1, E.tt);
      fix1 = true;
    }
    // ---- the step's stores
    if (act) {
      if ((!bw || kind == KT0) && cl < nw) gst(bt, x_off + cl, kb);
      if (bw) {
        const int nrow = an[i].nrow, ro = an[i].row_off;
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const int r = lane + 64 * (2 * j + h);
          if (r < nrow) {
            gst(za, ro + r, kz[j]);
            gst(ya, ro + r, ky[j]);
            if (store_delta) gst(dys, ro + r, kd[j]);
          }
        }
      }
      if ((bw || kind == KTN) && cl < nw) {
        const int xnx = bw ? an[i + 1].x_off : 0;
        gst(xa, x_off + cl, pxa);
        if (store_delta) gst(dxs, x_off + cl, pdx);
        if (bw) {
          if (cl < ndx) gst(rhs, xnx + cl, prn);
          if (!(cl < ndx && i > 0)) gst(rhs, x_off + cl, prh);
        }
      }
    }
  };

  if (act) {
    prefetch_E(KF0, 0, En);
    prefetch_as(KF0, 0);
    prefetch_LR(KF0, 0, LRn);
    prefetch_LC(KF0, 0, LCn);
    load_S(0, 0, SR);
  }
  for (int q = 0; q < Q; ++q) step(q);
  if (act && h == 0 && lane == 0) {
    info->iter += niter;
    info->iter_prof += niter;
  }
}

namespace {

struct AdmmCfg2 {
  AdmmLds2 lm;
  int ppw;
  size_t lds;
};

AdmmCfg2 admm2_config(const PlOcpHandle* h) {
  AdmmCfg2 c{};
  AdmmLds2& lm = c.lm;
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
  // `red` is time-shared (phases separated by barriers): the two waves' coupling
  // products [2][64] | the two row-segment arrays [2][(64 + T) 4] and the column
  // partials | row / column chunk sums and rho z - y
  lm.red = o;
  lm.segn = (64 + T) * 4;
#if PL_ADMM_ATOMIC
  // [acc0 | acc1 | rho z - y]: per-wave accumulators of the mat-vec (5 T) and of the
  // row / column sums, then trow
  lm.accn = up2(std::max(5 * T, std::max(std::max(h->nrow_max, h->ncol_max), 1)));
  lm.colp = o;
  lm.trow = o + 2 * lm.accn;
  o += up2(std::max(2 * lm.accn + h->nrow_max, 128));
#else
  lm.accn = 0;
  lm.colp = o + 2 * lm.segn;
  lm.trow = o + up2(h->chunk_max);
  o += up2(std::max(std::max(2 * lm.segn + T * (T - 1) / 2 * 4, up2(h->chunk_max) + h->nrow_max), 128));
#endif
  lm.asb = o;
  c.ppw = h->B >= 1024 ? 4 : (h->B >= 512 ? 2 : 1);
  const int budget = 160 * 1024 / 8;
  int cap = ((budget - lm.prog_dbl) / c.ppw - o) & ~1;
  cap = std::max(0, std::min(up2(std::max(h->nent_max, 1)), cap));
  lm.asb_cap = cap;
  lm.per_prob = o + cap;
  c.lds = (size_t)(lm.prog_dbl + c.ppw * lm.per_prob) * sizeof(double);
  return c;
}

template <int PPW, int ASR>
void launch_admm2_t(PlOcpHandle* h, int niter, int check, const AdmmCfg2& c) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)k_admm2<PPW, ASR>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  const int grid = (h->B + PPW - 1) / PPW;
  hipLaunchKernelGGL((k_admm2<PPW, ASR>), dim3(grid), dim3(128 * PPW), c.lds, h->stream, h->d, h->B, h->N, h->n,
                     h->m, h->nnz, h->ndx, h->S_stride, std::max(h->ncpl_max, 1), c.lm, niter, check,
                     h->admm_fwd_asb, h->set.sigma, h->set.alpha);
}

}  // namespace

bool admm2_supported(const PlOcpHandle* h) {
  return h->nw_max <= 128 && h->nrow_max <= 256 && h->ndx <= 64 && admm2_config(h).lds <= 160 * 1024;
}

void launch_admm2(PlOcpHandle* h, int niter, int check) {
  const AdmmCfg2 c = admm2_config(h);
  // per wave: A entries lane + 64 (2 k + h), k < ASR; both waves cover 128 ASR entries
  const int asr = h->admm_asr <= 16 ? 8 : 16;
  if (c.ppw == 4) {
    if (asr == 8) launch_admm2_t<4, 8>(h, niter, check, c);
    else launch_admm2_t<4, 16>(h, niter, check, c);
  } else if (c.ppw == 2) {
    if (asr == 8) launch_admm2_t<2, 8>(h, niter, check, c);
    else launch_admm2_t<2, 16>(h, niter, check, c);
  } else {
    if (asr == 8) launch_admm2_t<1, 8>(h, niter, check, c);
    else launch_admm2_t<1, 16>(h, niter, check, c);
  }
}
