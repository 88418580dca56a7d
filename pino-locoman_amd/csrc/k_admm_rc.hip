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
#include <algorithm>

#include "admm_common.h"
#include "state.h"

namespace {

using namespace admm;

struct RcLds {
  int prog_dbl, per_wave;
  int v, y, acc, trow, tcpl, bc, asb, asb_cap;
};

struct Sb {
  double2 s[KM][8];
};

}  // namespace

// ---------------------------------------------------------------------------
// Chain blocks of node i (one 256-thread workgroup per (problem, node)), from the stored
// (symmetrised, tiled) factor block that the ADMM kernels use:
//   d.CH[b] + i * 3 ndx^2:  FR (F_i row-major) | FT (F_i^T row-major) | G (S_i[dx, dx])
// Every chain lane reads one contiguous row (16-byte loads, one VGPR offset + immediates).
// F_i[a][k] = sum_{(e, s) in xc(a)} A_e rho_s sum_{(e', l) in cw(s)} A_e' S_i[l][k]
// (the coupling product the sweep kernels apply as t_s = rho_s a_s(w) . w).
__global__ __launch_bounds__(256) void k_fred(PlDev d, int N, int nnz, int ndx, int S_stride, int cpl_stride,
                                              long long ch_stride) {
  extern __shared__ double sc[];  // S_i[:, 0:ndx] dense, sc[l * ndx + k]
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
  const int X2 = ndx * ndx;
  double* CH = d.CH + (size_t)b * ch_stride + (size_t)i * 3 * X2;
  for (int q = threadIdx.x; q < X2; q += 256) CH[2 * X2 + q] = sc[q];  // rows l < ndx of sc: G
  if (i >= N) return;
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
    CH[a * ndx + k] = f;       // FR: (a, k)
    CH[X2 + k * ndx + a] = f;  // FT: (k, a)
  }
}

// ---------------------------------------------------------------------------
template <int W, int X>
__global__ __launch_bounds__(64 * W, 1) void k_admm_rc(PlDev d, int N, int n, int m, int nnz, int S_stride,
                                                       int cpl_stride, long long ch_stride, int chv_stride, RcLds lm,
                                                       int niter, int check, double sigma, double alpha) {
  extern __shared__ double lds[];
  const int b = blockIdx.x;
  PlProbInfo* info = d.info + b;
  if (info->done) return;  // the whole workgroup (one problem)
  {
    const uint4* src = reinterpret_cast<const uint4*>(d.aprog);
    uint4* dst = reinterpret_cast<uint4*>(lds);
    for (int k = threadIdx.x; k < lm.prog_dbl / 2; k += 64 * W) dst[k] = src[k];
  }
  __syncthreads();
  constexpr int ndx = X;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint16_t* PG = reinterpret_cast<const uint16_t*>(lds);
  double* Wr = lds + lm.prog_dbl + wv * lm.per_wave;
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
  double* WD = DL + L;
  double* EE = DL + 2 * L;
  double* A2 = DL + 3 * L;
  double* CP = DL + 4 * L;
  double* HP = DL + 5 * L;
  typedef const __attribute__((address_space(4))) PlAdmmNode* CNode;
  const CNode an = (CNode)d.anodes;
  constexpr int X2 = X * X;
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
        CP[i * ndx + lane] = c;
      }
    }
    if (lane < ndx) HP[i * ndx + lane] = y[lane];
    wsync();
  };

  // ---- one node of a parallel phase.  mode 0: P only (rhs complete, a2 = 0); 1: P3 + the
  // next iteration's P; 2: P3 only (the launch's last iteration)
  auto pnode = [&](int i, int mode, bool store_delta) __attribute__((always_inline)) {
    const int nw = an[i].nw, T4 = 4 * an[i].ntile, x_off = an[i].x_off;
    const int eo = an[i].ent_off, ne = an[i].nent;
    const bool term = i == N;
    const uint16_t* P = PG + an[i].prog;
    const double* __restrict__ Ai = As + eo;
    Sb R;
    load_S(i, 0, R);  // the factor block streams in behind the gathers
    for (int e = lane; e < min(ne, cap); e += 64) asb[e] = Ai[e];
    auto A = [&](int e) __attribute__((always_inline)) { return e < cap ? asb[e] : Ai[e]; };
    if (mode == 0) {
#pragma unroll
      for (int mm = 0; mm < MV; ++mm) {
        const int c = lane + 64 * mm;
        if (c < nw) v[c] = rhs[x_off + c];
        else if (c < T4) v[c] = 0.0;
      }
      if (lane < ndx) A2[(i + 1) * ndx + lane] = 0.0;
      wsync();
      matvec(i, R, true);
      coupling_out(i, A);
      return;
    }
    // ---- P3: operands
    double rh[MV], xo[MV], qo[MV];
#pragma unroll
    for (int mm = 0; mm < MV; ++mm) {
      const int c = x_off + min(lane + 64 * mm, nw - 1);
      rh[mm] = rhs[c];
      xo[mm] = xa[c];
      qo[mm] = qs[c];
    }
    const int nrow = an[i].nrow, ro = an[i].row_off;
    double lz[MR], ly[MR], lr[MR], ll[MR], lu[MR];
#pragma unroll
    for (int mm = 0; mm < MR; ++mm) {
      const int r = ro + min(lane + 64 * mm, max(nrow - 1, 0));
      lz[mm] = za[r];
      ly[mm] = ya[r];
      lr[mm] = rho[r];
      ll[mm] = ls[r];
      lu[mm] = us[r];
    }
    const double dl = DL[i * ndx + rr];
    if (!term && lane < ndx) y[nw + lane] = EE[(i + 1) * ndx + lane];
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
    matvec(i, R, true);  // y[0..nw) = x~_i
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
        gst(rhs, x_off + c, rn[mm]);
      }
    }
    if (!term) {
      if (lane < ndx) A2[(i + 1) * ndx + lane] = acc[nw + lane];
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
    if (mode == 2) return;
    wsync();
#pragma unroll
    for (int mm = 0; mm < MV; ++mm) {
      const int c = lane + 64 * mm;
      if (c < nw) v[c] = rn[mm];
      else if (c < T4) v[c] = 0.0;
    }
    wsync();
    matvec(i, R, false);  // y = g_i = S_i rhs'_i (the block again, from L2: registers are not kept across)
    coupling_out(i, A);
  };

  // ---- C1: delta_{i+1} = (c'_i - F_i delta_i) - a2_i, lane r = chain row (wave 0).  Row r of
  // F_{i+1} is streamed into the registers of row r of F_i as they are consumed (one step of
  // latency cover, one register buffer).
  auto chain_fwd = [&]() __attribute__((always_inline)) {
    double2 fr[X / 2];
    double cv, av;
    auto rowp = [&](int i) __attribute__((always_inline)) {
      return reinterpret_cast<const double2*>(CH + (size_t)min(i, N - 1) * 3 * X2 + rr * ndx);
    };
    {
      const double2* fm = rowp(0);
#pragma unroll
      for (int k = 0; k < X / 2; ++k) fr[k] = fm[k];
      cv = CP[rr];
      av = A2[ndx + rr];
    }
    if (lane < ndx) {
      bc[lane] = 0.0;
      DL[lane] = 0.0;
    }
    wsync();
    for (int i = 0; i < N; ++i) {
      const double2* fn = rowp(i + 1);
      const double cvn = CP[min(i + 1, N - 1) * ndx + rr];
      const double avn = A2[(min(i + 1, N - 1) + 1) * ndx + rr];
      double a[4] = {0.0, 0.0, 0.0, 0.0};
      const double2* b2 = reinterpret_cast<const double2*>(bc);
#pragma unroll
      for (int k = 0; k < X / 2; ++k) {
        const double2 t = b2[k];
        a[k & 3] += fr[k].x * t.x + fr[k].y * t.y;
        fr[k] = fn[k];
      }
      const double de = (cv - ((a[0] + a[1]) + (a[2] + a[3]))) - av;
      cv = cvn;
      av = avn;
      wsync();
      bc[lane] = de;  // every lane (no branch for the compiler to sink the FMAs into)
      if (lane < ndx) DL[(i + 1) * ndx + lane] = de;
      wsync();
    }
  };

  // ---- C2: e_i = w_i[dx] - F_i^T e_{i+1}, lane k = chain column (wave 0)
  auto chain_bwd = [&]() __attribute__((always_inline)) {
    double2 fr[X / 2];
    double wd;
    auto rowp = [&](int i) __attribute__((always_inline)) {
      return reinterpret_cast<const double2*>(CH + (size_t)max(i, 0) * 3 * X2 + X2 + rr * ndx);
    };
    {
      const double2* fm = rowp(N - 1);
#pragma unroll
      for (int r = 0; r < X / 2; ++r) fr[r] = fm[r];
      wd = WD[(N - 1) * ndx + rr];
      const double e = WD[N * ndx + rr];
      if (lane < ndx) {
        bc[lane] = e;
        EE[N * ndx + lane] = e;
      }
    }
    wsync();
    for (int i = N - 1; i >= 1; --i) {  // e_i for i = N-1 .. 1
      const double2* fn = rowp(i - 1);
      const double wdn = WD[max(i - 1, 0) * ndx + rr];
      double a[4] = {0.0, 0.0, 0.0, 0.0};
      const double2* b2 = reinterpret_cast<const double2*>(bc);
#pragma unroll
      for (int r = 0; r < X / 2; ++r) {
        const double2 t = b2[r];
        a[r & 3] += fr[r].x * t.x + fr[r].y * t.y;
        fr[r] = fn[r];
      }
      const double e = wd - ((a[0] + a[1]) + (a[2] + a[3]));
      wd = wdn;
      wsync();
      bc[lane] = e;
      if (lane < ndx) EE[i * ndx + lane] = e;
      wsync();
    }
  };

  // ---- P2: w_i[dx] = h'_i - G_i delta_i
  auto p2node = [&](int i) __attribute__((always_inline)) {
    if (lane < ndx) bc[lane] = DL[i * ndx + lane];
    const double h = HP[i * ndx + rr];
    wsync();
    const double2* G = reinterpret_cast<const double2*>(CH + (size_t)i * 3 * X2 + 2 * X2 + rr * ndx);
    double a[4] = {0.0, 0.0, 0.0, 0.0};
    const double2* b2 = reinterpret_cast<const double2*>(bc);
#pragma unroll
    for (int k = 0; k < X / 2; ++k) {
      const double2 t = b2[k], g = G[k];
      a[k & 3] += g.x * t.x + g.y * t.y;
    }
    if (lane < ndx) WD[i * ndx + lane] = h - ((a[0] + a[1]) + (a[2] + a[3]));
    wsync();
  };

  if (wv == 0 && lane < ndx) A2[lane] = 0.0;  // a2_{-1}
#ifndef RCX_NOP0
  for (int i = wv; i <= N; i += W) pnode(i, 0, false);
#endif
  __syncthreads();
  for (int it = 0; it < niter; ++it) {
#ifndef RCX_NOC1
    if (wv == 0) chain_fwd();
#endif
    __syncthreads();
#ifndef RCX_NOP2
    for (int i = wv; i <= N; i += W) p2node(i);
#endif
    __syncthreads();
#ifndef RCX_NOC2
    if (wv == 0) chain_bwd();
#endif
    __syncthreads();
    const bool lastit = it == niter - 1;
#ifndef RCX_NOP3
    for (int i = wv; i <= N; i += W) pnode(i, lastit ? 2 : 1, check && lastit);
#endif
    __syncthreads();
  }
  // the complete rhs for the next launch / kernel: rhs_i[dx] += a2_{i-1}
  for (int i = wv; i <= N; i += W) {
    if (i >= 1 && lane < ndx) {
      const int c = an[i].x_off + lane;
      rhs[c] = rhs[c] + A2[i * ndx + lane];
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
  int cap = ((budget - lm.prog_dbl) / w - o) & ~1;
  cap = std::max(0, std::min(up2(std::max(h->nent_max, 1)), cap));
  lm.asb_cap = cap;
  lm.per_wave = o + cap;
  c.lds = (size_t)(lm.prog_dbl + w * lm.per_wave) * sizeof(double);
  return c;
}

template <int W, int X>
void launch_rc_t(PlOcpHandle* h, int niter, int check, const RcCfg& c) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)k_admm_rc<W, X>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL((k_admm_rc<W, X>), dim3(h->B), dim3(64 * W), c.lds, h->stream, h->d, h->N, h->n, h->m, h->nnz,
                     h->S_stride, std::max(h->ncpl_max, 1), h->ch_stride, h->chv_stride, c.lm, niter, check,
                     h->set.sigma, h->set.alpha);
}

}  // namespace

long long rc_ch_stride(int N, int ndx) { return (long long)(N + 1) * 3 * ndx * ndx; }
int rc_chv_stride(int N, int ndx) { return 6 * (N + 2) * ndx; }

bool admm_rc_supported(const PlOcpHandle* h) {
  return (h->ndx == 24 || h->ndx == 36 || h->ndx == 48) && (h->rc_waves == 4 || h->rc_waves == 8) && h->nw_max <= 64 * MV && h->nrow_max <= 64 * MR && h->ncpl_max <= 64 &&
         rc_config(h, h->rc_waves).lds <= 160 * 1024;
}

void launch_fred(PlOcpHandle* h) {
  const size_t lds = (size_t)h->nw_max * h->ndx * sizeof(double);
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute((const void*)k_fred, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    attr = true;
  }
  hipLaunchKernelGGL(k_fred, dim3(h->B * (h->N + 1)), dim3(256), lds, h->stream, h->d, h->N, h->nnz, h->ndx,
                     h->S_stride, std::max(h->ncpl_max, 1), h->ch_stride);
}

void launch_admm_rc(PlOcpHandle* h, int niter, int check) {
  const RcCfg c = rc_config(h, h->rc_waves);
  switch (h->ndx * 16 + h->rc_waves) {
    case 24 * 16 + 4: launch_rc_t<4, 24>(h, niter, check, c); break;
    case 36 * 16 + 4: launch_rc_t<4, 36>(h, niter, check, c); break;
    case 48 * 16 + 4: launch_rc_t<4, 48>(h, niter, check, c); break;
    case 24 * 16 + 8: launch_rc_t<8, 24>(h, niter, check, c); break;
    case 36 * 16 + 8: launch_rc_t<8, 36>(h, niter, check, c); break;
    case 48 * 16 + 8: launch_rc_t<8, 48>(h, niter, check, c); break;
    default: break;
  }
}
