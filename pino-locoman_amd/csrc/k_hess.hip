// Lagrangian Hessian of the interior-point branch: the curvature of lam^T g that CasADi's
// exact Hessian gives the reference's Fatrop solve (optimization/ocp.py:248-263, Opti with
// expand=True).  The rows of node i depend on w_i = [dx_i, u_i] and linearly on dx_{i+1}
// (the integration rows dx_{i+1} - (dx_i + f dt), rows.h), so
//     H_L = diag(objective Hessian) + sum_i H_i,   H_i = sum_{rows r of node i} lam_r d^2 g_r / dw_i^2
// is block diagonal over the w_i: the same sparsity as the factor's diagonal blocks Kt_ii.
//
// The work list d.hlist holds the (node i, column pair j <= k of w_i) pairs (api.hip
// build_hess_list; pairs with an rnea tau_j column are structurally zero and not listed).  A
// pair's node rows are evaluated in hyper-dual numbers seeded on columns j and k (ad.h HDual)
// and the e1 e2 parts contracted with lam: H_i[k][j] = sum_r lam_r g_r.c, written packed lower
// (k (k + 1) / 2 + j from the node's offset d.hoff[i]), the layout k_fnode assembles Kt_ii in.
#include "dyn.h"
#include "eval_common.h"
#include "hess_tree.h"

using pl::VecIn;

namespace {

struct HessEmit {
  const double* lam;  // the node's rows
  double acc;
  int r;
  __device__ void operator()(const HDual& v, double, double) {
    acc = fma(lam[r], v.c, acc);
    ++r;
  }
};

}  // namespace

// k_lag_hess_pb: one pair per wave and one PROBLEM per lane (grid: pairs x problem groups of
// 64): the seeds are wave-uniform, so the row code's seed tests (tree passes a pair does not
// depend on are skipped) are scalar branches and every lane runs the same path.  (Until r04 a
// kernel with one pair per lane ran beside it, 298 against 254 ms per evaluation at the
// headline: removed.)
template <int DYN>
__global__ __launch_bounds__(64) void k_lag_hess_pb(PlDev d, int B, int N, int n, int m, int np, long long hl_stride) {
  const int qa = blockIdx.y * 64 + threadIdx.x;  // the active problems, compacted (k_ip_compact)
  if (qa >= d.ip_act[B]) return;
  const int b = d.ip_act[qa];
  const PlOcpConst& O = *d.oc;
  const PlModel& M = *d.model;
  const double* x = d.x + (size_t)b * n;
  const double* p = d.p + (size_t)b * np;
  const double* lam = d.ip_lam + (size_t)b * m;
  double* H = d.Hlag + (size_t)b * hl_stride;
  const int ndx = O.ndx;
  HDual kst[PL_KIN_STORE];
  const int2 w = d.hlist[blockIdx.x];
  const int wx = __builtin_amdgcn_readfirstlane(w.x);
  const int i = wx & 0xffff, only_ch = (wx >> 16) - 1;  // the pair's chain (api.hip set_solver)
  const int jk = __builtin_amdgcn_readfirstlane(w.y);
  const int j = jk & 0xffff, k = jk >> 16;
  const PlNode nd = d.nodes[i];
  const PlNode nn = d.nodes[i + 1];
  VecIn<HDual> dx{x + nd.x_off, nullptr, 0.0, j, k};
  VecIn<HDual> u{x + nd.x_off + ndx, nullptr, 0.0, j - ndx, k - ndx};
  VecIn<HDual> dxn{x + nn.x_off, nullptr, 0.0, j - nd.nw, k - nd.nw};
  HessEmit e{lam + nd.row_off, 0.0, 0};
  pl::node_rows<HDual, DYN>(M, O, i, p, dx, u, dxn, e, kst, 1, nullptr, nullptr, nullptr, only_ch);
  H[d.hoff[i] + k * (k + 1) / 2 + j] = e.acc;
}

// whole_body_rnea (u = [a | f | tau_j]): the rows are linear in a and in the contact forces,
// and only the RNEA rows (base rows and, on the tau nodes, the joint-torque rows; lambda_tau =
// their multipliers as a vector over v) couple them to q, through tau = M(q) a - sum_e J_e(q)^T f_e
// + ... (the DYNV rows are linear in a with constant coefficients, the force rows do not read
// q).  So for a dq column k
//     d^2 L / dq_k da   = d/dq_k [M(q) lambda_tau]        (one RNEA pass at v = 0, a = lambda_tau,
//                                                          f = 0 on the zero-gravity model)
//     d^2 L / dq_k df_e = -d/dq_k [J_e(q) lambda_tau]     (the foot velocities at v = lambda_tau)
// two dual tree passes seeded on dq_k give the whole (dq_k, a) and (dq_k, f_feet) rows of the
// node's block (k_lag_hess_pb would run one hyper-dual pass per pair: ~400 of a B2G node's
// ~1000).  One dq column per wave, one problem per lane.
namespace {
struct ZeroIn {
  PL_HD Dual operator[](int) const { return Dual(0.0, 0.0); }
};
struct LamIn {  // lambda_tau over v: the base rows' multipliers, then the joint-torque rows' (or 0)
  const double* lb;
  const double* lt;
  PL_HD Dual operator[](int k) const { return Dual(k < 6 ? lb[k] : (lt ? lt[k - 6] : 0.0), 0.0); }
};
}  // namespace

__global__ __launch_bounds__(64) void k_lag_hess_lin(PlDev d, int B, int n, int m, int np, long long hl_stride,
                                                     int3 rb_base, int3 rb_tau) {
  const int qa = blockIdx.y * 64 + threadIdx.x;  // the active problems, compacted (k_ip_compact)
  if (qa >= d.ip_act[B]) return;
  const int b = d.ip_act[qa];
  const PlOcpConst& O = *d.oc;
  const int2 w = d.hlin[blockIdx.x];
  const int i = __builtin_amdgcn_readfirstlane(w.x);
  const int wy = __builtin_amdgcn_readfirstlane(w.y);
  const int k = wy & 0xffff, only_ch = (wy >> 16) - 1;  // dq_k's chain (-1: a base coordinate)
  const PlNode nd = d.nodes[i];
  const double* p = d.p + (size_t)b * np;
  const double* lam = d.ip_lam + (size_t)b * m + nd.row_off;
  double* H = d.Hlag + (size_t)b * hl_stride + d.hoff[i];
  const int type = pl::node_type(O, i);
  const int rbb = type == 0 ? rb_base.x : (type == 1 ? rb_base.y : rb_base.z);
  const int rbt = type == 0 ? rb_tau.x : (type == 1 ? rb_tau.y : rb_tau.z);
  const LamIn lt{lam + rbb, rbt >= 0 ? lam + rbt : nullptr};
  const double* xi = p + O.P.x_init;
  const pl::VecIn<Dual> dq{d.x + (size_t)b * n + nd.x_off, nullptr, 0.0, k};
  Dual qb[7];
  pl::integrate_ff<Dual>(xi, dq, qb);
  const pl::RevQ<Dual, pl::VecIn<Dual>> qrev{xi, dq};
  Dual kst[PL_KIN_STORE];
  pl::NodeKin<Dual> kin;
  kin.vst = reinterpret_cast<double*>(kst);
  kin.dst = kin.vst + 1;
  kin.vstride = kin.dstride = 2;
  const int ndx = O.ndx, nv = O.nv;
  const auto slot = [&](int col) { return (size_t)col * (col + 1) / 2 + k; };  // (k, col) with k < col
  // (dq_k, a_j) = d/dq_k [M(q) lambda_tau]_j
  pl::tree_pass<Dual>(*d.model0, O, qb, qrev, ZeroIn{}, lt, ZeroIn{}, true, false, kin, nullptr, std::false_type{},
                      only_ch);
  for (int j = 0; j < nv; ++j) {
    const double t = j < 6 ? kin.tau[j].d : Dual(kin.tau_j(j - 6)).d;
    H[slot(ndx + j)] = t;
  }
  // (dq_k, f_e) = -d/dq_k [J_e(q) lambda_tau]   (feet)
  pl::tree_pass<Dual>(*d.model, O, qb, qrev, lt, ZeroIn{}, ZeroIn{}, false, true, kin, nullptr, std::false_type{},
                      only_ch);
  const int f0 = ndx + O.na;
  for (int e = 0; e < O.nfeet; ++e)
    for (int c = 0; c < 3; ++c) H[slot(f0 + 3 * e + c)] = -Dual(kin.foot_vel(e, c)).d;
}

// whole_body_rnea / whole_body_acc, the (dq, dq) and (dq, dv) pairs: of the node's rows only those that read
// the tree pass's outputs are nonlinear in the state (the RNEA base and joint-torque rows, the
// foot-velocity rows, the arm-velocity rows; every other row is linear in dx, rows.h node_rows), so
// the pair's curvature is that of
//     phi = lambda_tau^T tau(q, v, a, f) + sum_e mu_e . v_foot,e(q, v) + lambda_arm^T v_arm(q, v)
// (the last term in k_lag_hess_arm, launched after this kernel)
// (mu_e: the foot-velocity rows' multipliers times their coefficients, world axes).  By virtual work
// the first two terms are one forward sweep with no backward accumulation:
//     lambda_tau^T tau = sum_bodies L_b . f_b,   L_b = X_b,parent L_parent + S_b lambda_b   (L_root = lambda_base)
// with f_b the body's net wrench (I a + v x* I v - contact forces, body axes), and
//     mu_e . v_foot,e = (v_lin + w x p_e) . (oR_b^T mu_e)
// so a pair costs one hyper-dual sweep whose carried state is v, a, L and the world rotation of the
// current body (k_lag_hess_pb's node_rows<HDual> carries the world-frame force prefix, the joint
// subspaces and every row block as well, and spills).  The arm rows (relative to the base,
// dynamics/dynamics.py:86-113) keep the velocity-only tree pass, for the pairs on the base or the
// arm's chain.  d.htr packs pairs as d.hlist; one pair per wave, one problem per lane.
using namespace hess;

// whole_body_rnea / whole_body_acc, the (dv, dv) block: the only rows with curvature in v are the RNEA rows,
// and at a = 0, f = 0 without gravity the RNEA torque is the bias term C(q, v) v, a quadratic form
// in v.  With Q(v) = lambda_tau^T C(q, v) v the block is d^2 L / dv_j dv_k = d^2 Q / dv_j dv_k, and
// because Q is quadratic
//     Q(e_j + eps e_k) = Q(e_j) + eps d^2 Q / dv_j dv_k + eps^2 Q(e_k)
// so one dual sweep at v = e_j with tangent e_k gives the entry exactly (j = k: v = (1 + eps) e_j,
// the tangent is 2 Q(e_j)), with no cancellation.  Q by virtual work as in k_lag_hess_tree below:
// q is a constant here, so the joint rotations and the virtual velocities L_b are plain doubles and
// only v, a and the body wrenches carry a tangent.  d.hvv packs pairs as d.hlist (chain
// confinement included); one pair per wave, one problem per lane.
__global__ __launch_bounds__(64) void k_lag_hess_vv(PlDev d, int B, int n, int m, int np, long long hl_stride,
                                                    int3 rb_base, int3 rb_tau) {
  const int qa = blockIdx.y * 64 + threadIdx.x;  // the active problems, compacted (k_ip_compact)
  if (qa >= d.ip_act[B]) return;
  const int b = d.ip_act[qa];
  const PlOcpConst& O = *d.oc;
  const PlModel& M = *d.model;
  const int2 w = d.hvv[blockIdx.x];
  const int wx = __builtin_amdgcn_readfirstlane(w.x);
  const int i = wx & 0xffff, only_ch = (wx >> 16) - 1;
  const int jk = __builtin_amdgcn_readfirstlane(w.y);
  const int j = jk & 0xffff, k = jk >> 16;  // w_i columns nv + (velocity index)
  const PlNode nd = d.nodes[i];
  const double* x = d.x + (size_t)b * n + nd.x_off;
  const double* p = d.p + (size_t)b * np;
  const double* lam = d.ip_lam + (size_t)b * m + nd.row_off;
  const int type = pl::node_type(O, i);
  const int rbb = type == 0 ? rb_base.x : (type == 1 ? rb_base.y : rb_base.z);
  const int rbt = type == 0 ? rb_tau.x : (type == 1 ? rb_tau.y : rb_tau.z);
  const double* xi = p + O.P.x_init;
  const int nv = O.nv, vj_ = j - nv, vk_ = k - nv;
  const auto vin = [&](int q) { return Dual(q == vj_ ? 1.0 : 0.0, q == vk_ ? 1.0 : 0.0); };
  Dual phi(0.0, 0.0);
  if (only_ch < 0 && rbb >= 0) {  // the root body: f = v x* I v
    Dual v1[6], a1[6], f1[6];
    for (int c = 0; c < 6; ++c) { v1[c] = vin(c); a1[c] = Dual(0.0, 0.0); }
    body_wrench(M.mass[1], M.lever[1], M.Ic[1], a1, v1, f1);
    for (int c = 0; c < 6; ++c) phi += lam[rbb + c] * f1[c];
  }
  for (int ch = 0; ch < M.nchains; ++ch) {
    if (only_ch >= 0 && ch != only_ch) continue;
    const int first = M.chain_first[ch], L = M.chain_len[ch];
    Dual pv[6], pa[6];
    double pL[6];
    for (int c = 0; c < 6; ++c) { pv[c] = vin(c); pa[c] = Dual(0.0, 0.0); pL[c] = rbb >= 0 ? lam[rbb + c] : 0.0; }
    for (int kk = 0; kk < L; ++kk) {
      const int jt = first + kk;
      double s, c;
      sincos(xi[M.idx_q[jt]] + x[M.idx_q[jt] - 1], &s, &c);  // q_j = x_init + dq (rbd.h RevQ)
      const double* ax = M.axis[jt];
      const int iv = M.idx_v[jt];
      const Dual qd = vin(iv);
      Dual vj[6], aj[6], t[3];
      act_inv_j(M, jt, s, c, pv, vj);
      for (int q = 0; q < 3; ++q) vj[3 + q] += ax[q] * qd;
      act_inv_j(M, jt, s, c, pa, aj);
      crossd(ax, vj, t);
      for (int q = 0; q < 3; ++q) aj[q] -= t[q] * qd;
      crossd(ax, vj + 3, t);
      for (int q = 0; q < 3; ++q) aj[3 + q] -= t[q] * qd;
      double Lj[6];
      act_inv_j(M, jt, s, c, pL, Lj);
      const double lj = rbt >= 0 ? lam[rbt + iv - 6] : 0.0;
      for (int q = 0; q < 3; ++q) Lj[3 + q] += ax[q] * lj;
      Dual fj[6];
      body_wrench(M.mass[jt], M.lever[jt], M.Ic[jt], aj, vj, fj);
      for (int q = 0; q < 6; ++q) { phi += Lj[q] * fj[q]; pv[q] = vj[q]; pa[q] = aj[q]; pL[q] = Lj[q]; }
    }
  }
  d.Hlag[(size_t)b * hl_stride + d.hoff[i] + k * (k + 1) / 2 + j] = phi.d;
}

// SF: the (dq, f_ext) pairs (an external force frame, O.ext: the RNEA rows are linear in its force but
// it moves with q, so those pairs are this sweep with the force seeded); d.htrf
template <bool SF>
__global__ __launch_bounds__(64) void k_lag_hess_tree(PlDev d, int B, int n, int m, int np, long long hl_stride) {
  const int qa = blockIdx.y * 64 + threadIdx.x;  // the active problems, compacted (k_ip_compact)
  if (qa >= d.ip_act[B]) return;
  const int b = d.ip_act[qa];
  const int2 w = (SF ? d.htrf : d.htr)[blockIdx.x];
  const int wx = __builtin_amdgcn_readfirstlane(w.x);
  const int i = wx & 0xffff, only_ch = (wx >> 16) - 1;
  const int jk = __builtin_amdgcn_readfirstlane(w.y);
  const int j = jk & 0xffff, k = jk >> 16;
  const PlNode nd = d.nodes[i];
  d.Hlag[(size_t)b * hl_stride + d.hoff[i] + k * (k + 1) / 2 + j] =
      tree_pair<SF>(*d.model, *d.oc, i, only_ch, j, k, d.x + (size_t)b * n + nd.x_off, d.p + (size_t)b * np,
                    d.ip_lam + (size_t)b * m + nd.row_off);
}

// r06: the (dq, dq) and (dq, dv) pairs by forward-over-reverse columns (hess_tree.h tree_col): one work
// item per (node, chain, dq column j) with the mask of its pairs' other coordinates (api.hip
// set_solver groups d.htr that way: every pair is written by the item of its smaller index j), one item
// per wave, one problem per lane.  PL_PATH_HESS_PAIRS keeps k_lag_hess_tree<false> per pair.
template <bool WHOLE>
__global__ __launch_bounds__(64) void k_lag_hess_col(PlDev d, int B, int n, int m, int np, long long hl_stride,
                                                     int item0) {
  const int qa = blockIdx.y * 64 + threadIdx.x;
  if (qa >= d.ip_act[B]) return;
  const int b = d.ip_act[qa];
  const int4 w = d.hcol[item0 + blockIdx.x];
  const int wx = __builtin_amdgcn_readfirstlane(w.x);
  const int i = wx & 0xffff, only_ch = (wx >> 16) - 1;
  const int j = __builtin_amdgcn_readfirstlane(w.y);
  const uint32_t mask = (uint32_t)__builtin_amdgcn_readfirstlane(w.z);
  const PlNode nd = d.nodes[i];
  double* H = d.Hlag + (size_t)b * hl_stride + d.hoff[i];
  tree_col<WHOLE>(*d.model, *d.oc, i, only_ch, j, mask, d.x + (size_t)b * n + nd.x_off, d.p + (size_t)b * np,
           d.ip_lam + (size_t)b * m + nd.row_off, [&](int k, double v) {
             const int hi = k > j ? k : j, lo = k > j ? j : k;
             H[hi * (hi + 1) / 2 + lo] = v;
           });
}


// The arm rows of the (dq, dq) / (dq, dv) pairs, added to k_lag_hess_tree<false>'s entries (a
// kernel of their own: inside the sweep they pushed it past the register file).  Same pair list
// and lane mapping; the pairs on another chain exit at once.
__global__ __launch_bounds__(64) void k_lag_hess_arm(PlDev d, int B, int n, int m, int np, long long hl_stride) {
  const int qa = blockIdx.y * 64 + threadIdx.x;
  if (qa >= d.ip_act[B]) return;
  const int b = d.ip_act[qa];
  const PlOcpConst& O = *d.oc;
  const PlModel& M = *d.model;
  const int2 w = d.harm[blockIdx.x];  // the pairs on the base or the arm's chain (r06; d.htr until r05)
  const int wx = __builtin_amdgcn_readfirstlane(w.x);
  const int i = wx & 0xffff, only_ch = (wx >> 16) - 1;
  const int jk = __builtin_amdgcn_readfirstlane(w.y);
  const int j = jk & 0xffff, k = jk >> 16;
  if (j < 3) return;  // (k_lag_hess_tree wrote 0)
  const int type = pl::node_type(O, i);
  const PlNode nd = d.nodes[i];
  const double* x = d.x + (size_t)b * n + nd.x_off;
  const double* p = d.p + (size_t)b * np;
  const double* lam = d.ip_lam + (size_t)b * m + nd.row_off;
  const double* xi = p + O.P.x_init;
  const VecIn<HDual> dx{x, nullptr, 0.0, j, k};
  HDual qb[7];
  base_pose(xi, dx, qb);
  const pl::RevQ<HDual, VecIn<HDual>> qrev{xi, dx};
  const pl::VelAcc<HDual, VecIn<HDual>> vel{xi + O.nq, pl::sub_in(dx, O.nv)};
  double acc = 0.0;
  // ---- the arm rows (Dynamics.get_frame_velocity relative to the base, dynamics/dynamics.py:86-113;
  // rbd.h tree_pass): with l = [lam_0, lam_1, 0], l_b = R_base l (the base frame's placement on
  // the root) and mu_b = R0 l_b,
  //     lam_arm . v_arm = (mu_b + lam_2 e_z) . v_ee - mu_b . v_basept - l_b . (w1 x rel0)
  // where v_ee is the arm frame's world velocity, v_basept the base point's (linear in v_base with
  // constant coefficients: no curvature) and rel0 the arm frame's position relative to the base
  // point in root axes, which reads the arm joints only.  So the curvature is that of
  //     c_J . (v_J,lin - p x w_J)  -  sum_k pl_k . m_(k-1)  -  p . m_J
  // with c = R_chain^T (l_b + lam_2 R0^T e_z) and m = R_chain^T (l_b x w1) carried joint by joint
  // (pl_k the joint placements): one short sweep over the arm chain, for the pairs on the base or it.
  const int ra = O.arm.valid ? block_row(O, type, PL_RB_ARM, -1) : -1;
  if (ra >= 0) {
    int arm_ch = -1;
    for (int ch = 0; ch < M.nchains; ++ch)
      if (O.arm.joint >= M.chain_first[ch] && O.arm.joint < M.chain_first[ch] + M.chain_len[ch]) arm_ch = ch;
    if (arm_ch >= 0 && (only_ch < 0 || only_ch == arm_ch)) {
      const double l3[3] = {lam[ra], lam[ra + 1], 0.0};
      double lb[3];
      pl::matvec(O.base.R, l3, lb);
      HDual cm[3], mm[3], pv[6], psi(0.0);
      {
        HDual R0[9];
        pl::quat_to_R(qb + 3, R0);
        for (int q = 0; q < 3; ++q) cm[q] = lb[q] + lam[ra + 2] * R0[6 + q];  // R0^T e_z = row 3 of R0
      }
      for (int q = 0; q < 6; ++q) pv[q] = vel[q];
      crossd(lb, pv + 3, mm);
      const int first = M.chain_first[arm_ch];
      for (int jt = first; jt <= O.arm.joint; ++jt) {
        HDual s, c, t3[3], vj[6];
        sincos_s(qrev(M.idx_q[jt]), &s, &c);
        const double* pj = M.jp[jt];
        psi -= pj[0] * mm[0] + pj[1] * mm[1] + pj[2] * mm[2];
        rot_t(M, jt, s, c, mm, t3);
        for (int q = 0; q < 3; ++q) mm[q] = t3[q];
        rot_t(M, jt, s, c, cm, t3);
        for (int q = 0; q < 3; ++q) cm[q] = t3[q];
        act_inv_j(M, jt, s, c, pv, vj);
        const HDual qd = vel[M.idx_v[jt]];
        const double* ax = M.axis[jt];
        for (int q = 0; q < 3; ++q) { pv[q] = vj[q]; pv[3 + q] = vj[3 + q] + ax[q] * qd; }
      }
      const double* pf = O.arm.p;
      HDual pxw[3];
      crossd(pf, pv + 3, pxw);
      psi -= pf[0] * mm[0] + pf[1] * mm[1] + pf[2] * mm[2];
      for (int q = 0; q < 3; ++q) psi += (pv[q] - pxw[q]) * cm[q];
      acc += psi.c;
    }
  }
  if (acc != 0.0) d.Hlag[(size_t)b * hl_stride + d.hoff[i] + k * (k + 1) / 2 + j] += acc;
}

// whole_body_rnea / whole_body_acc, the (f, f) pairs: of the rows only the friction cones
// c (f_x^2 + f_y^2) - c mu^2 f_z^2 (rows.h PL_RB_CONE) are nonlinear in a foot force, so the
// block is diagonal with 2 c lambda and -2 c mu^2 lambda.  d.hcone: (node, w_i column); one entry
// per lane.
__global__ __launch_bounds__(64) void k_lag_hess_cone(PlDev d, int B, int m, int np, long long hl_stride, int len) {
  const int q = blockIdx.x * 64 + threadIdx.x;
  const int b = blockIdx.y;
  if (q >= len || !d.ipinfo[b].active) return;
  const PlOcpConst& O = *d.oc;
  const int2 w = d.hcone[q];
  const int i = w.x, col = w.y;
  const int e = (col - O.ndx - O.na) / 3, comp = (col - O.ndx - O.na) % 3;
  const int type = pl::node_type(O, i);
  const int r = block_row(O, type, PL_RB_CONE, e);
  const double c = d.p[(size_t)b * np + O.P.contact + 4 * i + e];
  const double h = comp < 2 ? c * 2.0 : -(c * O.mu * O.mu) * 2.0;
  const double lam = r >= 0 ? d.ip_lam[(size_t)b * m + d.nodes[i].row_off + r] : 0.0;
  d.Hlag[(size_t)b * hl_stride + d.hoff[i] + col * (col + 1) / 2 + col] = lam * h;
}

#define PL_DISPATCH_DYN(dyn, KERNEL, ...)                                            \
  switch (dyn) {                                                                      \
    case PL_DYN_RNEA: hipLaunchKernelGGL(KERNEL<PL_DYN_RNEA>, __VA_ARGS__); break;   \
    case PL_DYN_ACC: hipLaunchKernelGGL(KERNEL<PL_DYN_ACC>, __VA_ARGS__); break;     \
    case PL_DYN_CV: hipLaunchKernelGGL(KERNEL<PL_DYN_CV>, __VA_ARGS__); break;       \
    case PL_DYN_CA: hipLaunchKernelGGL(KERNEL<PL_DYN_CA>, __VA_ARGS__); break;       \
    case PL_DYN_ACCNB: hipLaunchKernelGGL(KERNEL<PL_DYN_ACCNB>, __VA_ARGS__); break; \
    case PL_DYN_CVNB: hipLaunchKernelGGL(KERNEL<PL_DYN_CVNB>, __VA_ARGS__); break;   \
    default: hipLaunchKernelGGL(KERNEL<PL_DYN_ABA>, __VA_ARGS__); break;             \
  }

// The active problems of this interior-point iteration in ascending order (one 256-thread
// block; a ballot prefix per wave, wave offsets in LDS): the Hessian kernels map lanes to
// d.ip_act, so the waves past the active count exit at once when most problems have
// terminated (a warm-started MPC step's line-search failures).  Lanes write only their own
// problem's entries, so the results do not depend on the mapping.
__global__ __launch_bounds__(256) void k_ip_compact(PlDev d, int B, int count_lanes) {
  __shared__ int s_wave[4], s_base;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (threadIdx.x == 0) s_base = 0;
  __syncthreads();
  for (int c0 = 0; c0 < B; c0 += 256) {
    const int b = c0 + threadIdx.x;
    const bool act = b < B && d.ipinfo[b].active;
    const unsigned long long m = __ballot(act);
    const int before = __popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) s_wave[w] = __popcll(m);
    __syncthreads();
    int off = s_base;
    for (int k = 0; k < w; ++k) off += s_wave[k];
    if (act) d.ip_act[off + before] = b;
    __syncthreads();
    if (threadIdx.x == 0) s_base += s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    d.ip_act[B] = s_base;
    // lanes of the Hessian waves that will run, for the launches that get a profiling event
    // slot only (pl_ocp_profile_read_hess averages over those)
    if (count_lanes) d.ip_act[B + 1] += (s_base + 63) / 64 * 64;
  }
}

void launch_lag_hess(PlOcpHandle* h) {
  const bool prof = h->profile && h->prof_hn < 16;  // pl_mpc_step collects the slots before every step
  if (prof) hipEventRecord(h->prof_hev[h->prof_hn][0], h->stream);
  hipLaunchKernelGGL(k_ip_compact, dim3(1), dim3(256), 0, h->stream, h->d, h->B, prof ? 1 : 0);
  if (h->hlin_len > 0)
    hipLaunchKernelGGL(k_lag_hess_lin, dim3(h->hlin_len, (h->B + 63) / 64), dim3(64), 0, h->stream, h->d, h->B, h->n,
                       h->m, h->np, h->hl_stride, make_int3(h->hl_rb_base[0], h->hl_rb_base[1], h->hl_rb_base[2]),
                       make_int3(h->hl_rb_tau[0], h->hl_rb_tau[1], h->hl_rb_tau[2]));
  if (h->hvv_len > 0)
    hipLaunchKernelGGL(k_lag_hess_vv, dim3(h->hvv_len, (h->B + 63) / 64), dim3(64), 0, h->stream, h->d, h->B, h->n,
                       h->m, h->np, h->hl_stride, make_int3(h->hl_rb_base[0], h->hl_rb_base[1], h->hl_rb_base[2]),
                       make_int3(h->hl_rb_tau[0], h->hl_rb_tau[1], h->hl_rb_tau[2]));
  if (h->hcol_len > 0) {  // the whole-tree base columns first, then the chain columns
    if (h->hcol_nbase > 0)
      hipLaunchKernelGGL(k_lag_hess_col<true>, dim3(h->hcol_nbase, (h->B + 63) / 64), dim3(64), 0, h->stream, h->d,
                         h->B, h->n, h->m, h->np, h->hl_stride, 0);
    if (h->hcol_len > h->hcol_nbase)
      hipLaunchKernelGGL(k_lag_hess_col<false>, dim3(h->hcol_len - h->hcol_nbase, (h->B + 63) / 64), dim3(64), 0,
                         h->stream, h->d, h->B, h->n, h->m, h->np, h->hl_stride, h->hcol_nbase);
  } else if (h->htr_len > 0)
    hipLaunchKernelGGL(k_lag_hess_tree<false>, dim3(h->htr_len, (h->B + 63) / 64), dim3(64), 0, h->stream, h->d, h->B,
                       h->n, h->m, h->np, h->hl_stride);
  if (h->harm_len > 0 && h->oc.arm.valid)
    hipLaunchKernelGGL(k_lag_hess_arm, dim3(h->harm_len, (h->B + 63) / 64), dim3(64), 0, h->stream, h->d, h->B, h->n,
                       h->m, h->np, h->hl_stride);
  if (h->htrf_len > 0)
    hipLaunchKernelGGL(k_lag_hess_tree<true>, dim3(h->htrf_len, (h->B + 63) / 64), dim3(64), 0, h->stream, h->d, h->B,
                       h->n, h->m, h->np, h->hl_stride);
  if (h->hcone_len > 0)
    hipLaunchKernelGGL(k_lag_hess_cone, dim3((h->hcone_len + 63) / 64, h->B), dim3(64), 0, h->stream, h->d, h->B, h->m,
                       h->np, h->hl_stride, h->hcone_len);
  if (h->hl_len > 0)
    PL_DISPATCH_DYN(h->oc.dyn, k_lag_hess_pb, dim3(h->hl_len, (h->B + 63) / 64), dim3(64), 0, h->stream, h->d, h->B, h->N,
                  h->n, h->m, h->np, h->hl_stride);
  if (prof) {
    hipEventRecord(h->prof_hev[h->prof_hn][1], h->stream);
    h->prof_hn++;
  }
}
