// C-ABI of the batched MPC inner loop (include/pinoloco.h).
//
// Host side of the drop-in boundary: builds the variable / row / sparsity layout
// the reference gets from CasADi Opti (optimization/ocp.py:38-44, 103-198, 283,
// 305), owns the device buffers of a batch, and sequences the kernels of one SQP
// iteration exactly as OCP.solve() sequences sqp_data -> osqp.update ->
// osqp.solve -> line search (ocp.py:375-414).
#include <stdarg.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <cmath>
#include <string>
#include <mutex>
#include <vector>

#include "../../include/pinoloco.h"
#include "dyn.h"
#include "handles.h"
#include "rows.h"
#include "state.h"

static thread_local char g_err[1024] = "";

void pl_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}


struct pl_ocp {
  PlOcpHandle h;
  bool on_device;
  std::vector<PlNode> nodes;
  std::vector<int> colptr, rowidx, entcol, rowptr, rowent, cplrow, rownode, colnode;
  std::vector<int> gr_ptr, gc_ptr;    // global CSR / CSC of the whole A (k_check)
  std::vector<int2> gr_ec, gc_er;     // (entry, global column) / (entry, global row)
  std::vector<PlAdmmNode> anodes;
  std::vector<uint16_t> aprog, fprog;
  std::vector<uint32_t> ttab;
  std::vector<PlFacNode> fnodes;
  std::vector<uint32_t> kasm, kcpl;
  std::vector<uint16_t> kfl;
  std::vector<double> h_params;  // host copy of the parameters (B x np)
  std::vector<void*> allocs;
  hipEvent_t ev[5];
  // pl_mpc_step replay: the launches of one OSQP-SQP MPC step after k_mpc_prepare, captured
  // once into a HIP graph and replayed while the handle's host state is unchanged
  hipGraphExec_t mpc_graph = nullptr;
  std::vector<unsigned char> mpc_key;  // bytes of `h` the graph was captured with (or last seen)
  int mpc_graph_off = 0;               // 1: capture failed or PL_MPC_GRAPH=0: launch eagerly
  long long mpc_captures = 0;
};

extern "C" const char* pl_last_error(void) { return g_err; }
extern "C" int pl_version(void) { return 1; }

// ---------------------------------------------------------------------------
// model
extern "C" int pl_model_create(const pl_model_desc* d, pl_model** out) {
  if (!d || !out) { pl_set_error("null argument"); return -1; }
  if (d->njoints > PL_MAXJ || d->nq > PL_MAXQ || d->nv > PL_MAXV) {
    pl_set_error("model too large (njoints=%d nq=%d nv=%d)", d->njoints, d->nq, d->nv);
    return -1;
  }
  pl_model* M = new pl_model();
  PlModel& m = M->m;
  memset(&m, 0, sizeof(m));
  m.njoints = d->njoints;
  m.nq = d->nq;
  m.nv = d->nv;
  int iq = 0, iv = 0;
  m.total_mass = 0.0;
  for (int j = 0; j < d->njoints; ++j) {
    m.parent[j] = d->parent[j];
    m.jtype[j] = d->jtype[j];
    for (int k = 0; k < 3; ++k) m.axis[j][k] = d->axis[3 * j + k];
    for (int k = 0; k < 9; ++k) m.jR[j][k] = d->placement_R[9 * j + k];
    for (int k = 0; k < 3; ++k) m.jp[j][k] = d->placement_p[3 * j + k];
    m.mass[j] = d->mass[j];
    for (int k = 0; k < 3; ++k) m.lever[j][k] = d->lever[3 * j + k];
    for (int k = 0; k < 9; ++k) m.Ic[j][k] = d->inertia[9 * j + k];
    m.total_mass += d->mass[j];
    if (j == 0) continue;
    m.idx_q[j] = iq;
    m.idx_v[j] = iv;
    if (m.jtype[j] == PL_JT_FREEFLYER) {
      if (j != 1) { pl_set_error("free-flyer must be joint 1"); delete M; return -1; }
      iq += 7;
      iv += 6;
    } else if (m.jtype[j] == PL_JT_REVOLUTE) {
      iq += 1;
      iv += 1;
      const double* a = m.axis[j];
      if (a[0] == 1.0 && a[1] == 0.0 && a[2] == 0.0) m.axis_kind[j] = PL_AX_X;
      else if (a[0] == 0.0 && a[1] == 1.0 && a[2] == 0.0) m.axis_kind[j] = PL_AX_Y;
      else if (a[0] == 0.0 && a[1] == 0.0 && a[2] == 1.0) m.axis_kind[j] = PL_AX_Z;
      else m.axis_kind[j] = PL_AX_GEN;
    } else {
      pl_set_error("unsupported joint type %d at joint %d", m.jtype[j], j);
      delete M;
      return -1;
    }
  }
  if (iq != d->nq || iv != d->nv || d->jtype[1] != PL_JT_FREEFLYER) {
    pl_set_error("inconsistent nq/nv or missing free-flyer root");
    delete M;
    return -1;
  }
  for (int k = 0; k < 3; ++k) m.gravity[k] = d->gravity[k];
  // chains: every non-root joint's parent is the root or the previous joint, and
  // only the root branches (utils/robot.py robots: 4 legs + optional arm)
  std::vector<int> nchild(d->njoints, 0);
  for (int j = 2; j < d->njoints; ++j) nchild[m.parent[j]]++;
  m.nchains = 0;
  for (int j = 2; j < d->njoints; ++j) {
    const int p = m.parent[j];
    if (p == 1) {
      if (m.nchains >= PL_MAXCHAIN) { pl_set_error("too many chains"); delete M; return -1; }
      m.chain_first[m.nchains] = j;
      m.chain_len[m.nchains] = 1;
      m.nchains++;
    } else if (p == j - 1 && nchild[p] == 1 && m.nchains > 0) {
      m.chain_len[m.nchains - 1]++;
      if (m.chain_len[m.nchains - 1] > PL_MAXCL) { pl_set_error("chain too long"); delete M; return -1; }
    } else {
      pl_set_error("joint %d breaks the root+chains tree shape", j);
      delete M;
      return -1;
    }
  }
  M->nframes = d->nframes;
  M->frame_parent.assign(d->frame_parent, d->frame_parent + d->nframes);
  M->frame_R.assign(d->frame_R, d->frame_R + 9 * d->nframes);
  M->frame_p.assign(d->frame_p, d->frame_p + 3 * d->nframes);
  *out = M;
  return 0;
}

extern "C" void pl_model_destroy(pl_model* m) { delete m; }

// ---------------------------------------------------------------------------
// layout
namespace {

void add_block(PlOcpConst& O, int type, int kind, int count, int arg = 0) {
  PlRowBlock& B = O.blk[type][O.nblk[type]++];
  B.kind = kind;
  B.count = count;
  B.arg = arg;
  B.pad = 0;
}

// Row blocks per node type in the reference's subject_to order.
void build_blocks(PlOcpConst& O, bool has_ext, bool has_arm) {
  for (int type = 0; type < 3; ++type) {
    O.nblk[type] = 0;
    const bool first = (type == 0);
    const bool tau = PL_IS_RNEA(O.dyn) && (type == 1 || (type == 0 && O.tau_nodes > 0));
    const bool cv = PL_IS_CV(O.dyn);
    // centroidal_vel keeps the state rows at node 0 (ocp.py:137-140, 170-173)
    const bool state = !first || cv;
    if (first) add_block(O, type, PL_RB_INIT, O.ndx);
    if (cv) {  // setup_dynamics_constraints (ocp_centroidal_vel.py:85-107)
      add_block(O, type, PL_RB_CV_DYNH, 6);
      add_block(O, type, PL_RB_CV_DYNQ, O.nv);
      if (O.dyn == PL_DYN_CV) add_block(O, type, PL_RB_CV_GAP, 6);  // include_base only
    } else {
      add_block(O, type, PL_RB_DYNQ, O.nv);
      // include_acc = False: "a inherently uses this finite difference" (ocp_whole_body_rnea.py:157-159)
      if (O.dyn != PL_DYN_RNEAFD) add_block(O, type, PL_RB_DYNV, O.nv);
    }
    if (PL_IS_RNEA(O.dyn) || O.dyn == PL_DYN_ACC) add_block(O, type, PL_RB_RNEA_BASE, 6);
    if (O.dyn == PL_DYN_CA) add_block(O, type, PL_RB_CA_GAP, 6);
    if (tau) {
      add_block(O, type, PL_RB_TAU_EQ, O.nj);
      add_block(O, type, PL_RB_TAU_BND, O.nj);
    }
    for (int k = 0; k < O.nfeet; ++k) {
      add_block(O, type, PL_RB_FZ, 1, k);
      add_block(O, type, PL_RB_CONE, 1, k);
      add_block(O, type, PL_RB_SWINGF, 3, k);
      if (state) {
        add_block(O, type, PL_RB_FVXY, 2, k);
        add_block(O, type, PL_RB_FVZ, 1, k);
      }
    }
    if (has_ext) add_block(O, type, PL_RB_EXT, 3);
    if (state) {
      if (has_arm) add_block(O, type, PL_RB_ARM, 3);
      add_block(O, type, PL_RB_QJ, O.nj);
      add_block(O, type, PL_RB_VJ, O.nj);
    }
    int rows = 0;
    for (int b = 0; b < O.nblk[type]; ++b) rows += O.blk[type][b].count;
    O.rows_of_type[type] = rows;
  }
}

// velocity-index support of a frame on joint j (joints from j up to the root, root excluded)
std::vector<int> support_v(const PlModel& M, int j) {
  std::vector<int> s;
  while (j > 1) {
    s.push_back(M.idx_v[j]);
    j = M.parent[j];
  }
  return s;
}

// Local-column dependency set of every row of node i (superset of the true
// nonzeros; values of structurally-irrelevant entries evaluate to 0).
std::vector<std::vector<int>> node_row_deps(const PlModel& M, const PlOcpConst& O, int i, int nu) {
  const int type = pl::node_type(O, i);
  const int nv = O.nv, nj = O.nj, nf = O.nf, ndx = O.ndx;
  const int nw = ndx + nu;
  const bool cv = PL_IS_CV(O.dyn), cvnb = O.dyn == PL_DYN_CVNB;
  // dx = [dq, dv] (whole body) or [dh, dq] with v = u[:nv] (centroidal_vel); without the
  // base, v = [v_b(h, q, v_j), v_j] with u = [v_j | f]
  auto DQ = [&](int k) { return cv ? 6 + k : k; };
  auto U = [&](int k) { return ndx + k; };
  auto DV = [&](int k) { return cv ? ndx + k : nv + k; };
  auto add_v = [&](std::vector<int>& s, int k) {
    if (!cvnb) { s.push_back(DV(k)); return; }
    if (k >= 6) { s.push_back(U(k - 6)); return; }
    for (int c = 0; c < 6; ++c) s.push_back(c);
    for (int c = 3; c < nv; ++c) s.push_back(DQ(c));
    for (int c = 0; c < nj; ++c) s.push_back(U(c));
  };
  auto DXN = [&](int k) { return nw + k; };
  const bool accf = O.dyn == PL_DYN_ACC || O.dyn == PL_DYN_CA || O.dyn == PL_DYN_ACCNB;
  const int f_off = (PL_IS_RNEA(O.dyn) || accf) ? O.na : (O.dyn == PL_DYN_CV ? nv : nj);
  auto F = [&](int k) { return U(f_off + k); };
  std::vector<int> dynset;  // dependency set of the RNEA / ABA / base-solve outputs
  for (int k = 3; k < nv; ++k) dynset.push_back(DQ(k));
  for (int k = 0; k < nv; ++k) dynset.push_back(DV(k));
  if (O.dyn == PL_DYN_ABA || O.dyn == PL_DYN_ACCNB) {
    for (int k = 0; k < nj; ++k) dynset.push_back(U(k));
  } else if (O.dyn == PL_DYN_RNEAFD) {  // a = (v_{i+1} - v_i) / dt
    for (int k = 0; k < nv; ++k) dynset.push_back(DXN(nv + k));
  } else {
    for (int k = 0; k < nv; ++k) dynset.push_back(U(k));
  }
  for (int k = 0; k < nf; ++k) dynset.push_back(F(k));
  auto frame_deps = [&](const PlFrameRef& fr) {
    std::vector<int> s;
    for (int k = 3; k < 6; ++k) s.push_back(DQ(k));
    for (int v : support_v(M, fr.joint)) s.push_back(DQ(v));
    for (int k = 0; k < 6; ++k) add_v(s, k);
    for (int v : support_v(M, fr.joint)) add_v(s, v);
    return s;
  };
  std::vector<std::vector<int>> rows;
  for (int b = 0; b < O.nblk[type]; ++b) {
    const PlRowBlock& B = O.blk[type][b];
    const int k = B.arg;
    for (int r = 0; r < B.count; ++r) {
      std::vector<int> s;
      switch (B.kind) {
        case PL_RB_INIT: s = {r}; break;
        case PL_RB_DYNQ: s = {DQ(r), DV(r), DXN(r)}; break;
        case PL_RB_DYNV:
          if (O.dyn == PL_DYN_ABA || (O.dyn == PL_DYN_ACCNB && r < 6)) {
            s = dynset;
            s.push_back(DV(r));
            s.push_back(DXN(nv + r));
          } else if (O.dyn == PL_DYN_ACCNB) {
            s = {DV(r), U(r - 6), DXN(nv + r)};
          } else {
            s = {DV(r), U(r), DXN(nv + r)};
          }
          break;
        case PL_RB_RNEA_BASE: s = dynset; break;
        case PL_RB_CA_GAP: s = dynset; break;
        case PL_RB_TAU_EQ: s = dynset; s.push_back(U(O.na + nf + r)); break;
        case PL_RB_TAU_BND: s = {U(O.na + nf + r)}; break;
        case PL_RB_FZ: s = {F(3 * k + 2)}; break;
        case PL_RB_CONE: s = {F(3 * k), F(3 * k + 1), F(3 * k + 2)}; break;
        case PL_RB_SWINGF: s = {F(3 * k + r)}; break;
        case PL_RB_FVXY:
        case PL_RB_FVZ: s = frame_deps(O.feet[k]); break;
        case PL_RB_EXT: s = {F(3 * O.nfeet + r)}; break;
        case PL_RB_ARM: s = frame_deps(O.arm); break;
        case PL_RB_QJ: s = {DQ(6 + r)}; break;
        case PL_RB_VJ: add_v(s, 6 + r); break;
        case PL_RB_CV_DYNH:  // h_dot(q, forces): orientation + joints, every force
          s = {r, DXN(r)};
          for (int k = 3; k < nv; ++k) s.push_back(DQ(k));
          for (int k = 0; k < nf; ++k) s.push_back(F(k));
          break;
        case PL_RB_CV_DYNQ: s = {DQ(r), DXN(6 + r)}; add_v(s, r); break;
        case PL_RB_CV_GAP:  // A(q) v - m h
          s = {r};
          for (int k = 3; k < nv; ++k) s.push_back(DQ(k));
          for (int k = 0; k < nv; ++k) s.push_back(DV(k));
          break;
      }
      std::sort(s.begin(), s.end());
      s.erase(std::unique(s.begin(), s.end()), s.end());
      rows.push_back(s);
    }
  }
  return rows;
}

int build_layout(pl_ocp* o) {
  PlOcpHandle& h = o->h;
  const PlOcpConst& O = h.oc;
  const PlModel& M = h.model;
  const int N = O.N, ndx = O.ndx;
  o->nodes.assign(N + 1, PlNode());
  o->colptr.clear();
  o->rowidx.clear();
  o->entcol.clear();
  o->rowptr.clear();
  o->rowent.clear();
  o->cplrow.clear();
  int x_off = 0, row_off = 0, ent_off = 0, s_off = 0;
  h.nw_max = 0;
  h.ncol_max = 0;
  h.nrow_max = 0;
  h.nunit_max = 0;
  h.ntile_max = 0;
  for (int i = 0; i <= N; ++i) {
    PlNode& nd = o->nodes[i];
    memset(&nd, 0, sizeof(nd));
    const int nu = (i < N) ? pl::node_nu(O, i) : 0;
    nd.nu = nu;
    nd.nw = ndx + nu;
    nd.x_off = x_off;
    nd.row_off = row_off;
    nd.ent_off = ent_off;
    nd.colptr_off = (int)o->colptr.size();
    nd.rowptr_off = (int)o->rowptr.size();
    nd.csr_off = (int)o->rowent.size();
    nd.cpl_off = (int)o->cplrow.size();
    if (i < N) {
      auto deps = node_row_deps(M, O, i, nu);
      nd.nrow = (int)deps.size();
      nd.ncol = nd.nw + ndx;
      std::vector<std::vector<int>> cols(nd.ncol);
      for (int r = 0; r < nd.nrow; ++r)
        for (int c : deps[r]) cols[c].push_back(r);
      int e = 0;
      std::vector<std::vector<int>> rowents(nd.nrow);
      for (int c = 0; c < nd.ncol; ++c) {
        o->colptr.push_back(e);
        for (int r : cols[c]) {
          o->rowidx.push_back(r);
          o->entcol.push_back(c);
          rowents[r].push_back(e);
          ++e;
        }
      }
      o->colptr.push_back(e);
      nd.nent = e;
      int s = 0;
      for (int r = 0; r < nd.nrow; ++r) {
        o->rowptr.push_back(s);
        bool cpl = false;
        for (int ee : rowents[r]) {
          o->rowent.push_back(ee);
          if (o->entcol[ent_off + ee] >= nd.nw) cpl = true;
          ++s;
        }
        if (cpl) o->cplrow.push_back(r);
      }
      o->rowptr.push_back(s);
      nd.ncpl = (int)o->cplrow.size() - nd.cpl_off;
    }
    // factor block: lower triangle in 4x4 tiles, K tile slots per lane of a wave
    nd.ntile = (nd.nw + 3) / 4;
    nd.nunit = (nd.ntile * (nd.ntile + 1) / 2 + 63) / 64;
    nd.s_off = s_off;
    s_off += nd.nunit * 64 * 16;
    x_off += nd.nw;
    row_off += nd.nrow;
    ent_off += nd.nent;
    h.nw_max = std::max(h.nw_max, nd.nw);
    h.ncol_max = std::max(h.ncol_max, nd.ncol);
    h.nrow_max = std::max(h.nrow_max, nd.nrow);
    h.nunit_max = std::max(h.nunit_max, nd.nunit);
    h.ntile_max = std::max(h.ntile_max, nd.ntile);
  }
  h.n = x_off;
  h.m = row_off;
  h.nnz = ent_off;
  h.S_stride = s_off;
  if (h.nw_max > 112) {
    pl_set_error("node block %d > 112 variables is not supported by the factor kernel", h.nw_max);
    return -1;
  }
  o->rownode.assign(h.m, 0);
  o->colnode.assign(h.n, 0);
  for (int i = 0; i <= N; ++i) {
    const PlNode& nd = o->nodes[i];
    for (int r = 0; r < nd.nrow; ++r) o->rownode[nd.row_off + r] = i;
    for (int c = 0; c < nd.nw; ++c) o->colnode[nd.x_off + c] = i;
  }
  // global CSR and CSC with flattened (entry, index) pairs: entries of a column in the
  // order of its own node, then of the previous node (dx_{i+1} part)
  o->gr_ptr.assign(1, 0);
  o->gr_ec.clear();
  for (int i = 0; i <= N; ++i) {
    const PlNode& nd = o->nodes[i];
    for (int r = 0; r < nd.nrow; ++r) {
      for (int q = o->rowptr[nd.rowptr_off + r]; q < o->rowptr[nd.rowptr_off + r + 1]; ++q) {
        const int e = o->rowent[nd.csr_off + q];
        const int lc = o->entcol[nd.ent_off + e];
        const int j = lc < nd.nw ? nd.x_off + lc : o->nodes[i + 1].x_off + (lc - nd.nw);
        o->gr_ec.push_back(make_int2(nd.ent_off + e, j));
      }
      o->gr_ptr.push_back((int)o->gr_ec.size());
    }
  }
  o->gc_ptr.assign(1, 0);
  o->gc_er.clear();
  for (int i = 0; i <= N; ++i) {
    const PlNode& nd = o->nodes[i];
    for (int lc = 0; lc < nd.nw; ++lc) {
      if (i < N) {
        const int* cp = o->colptr.data() + nd.colptr_off;
        for (int e = cp[lc]; e < cp[lc + 1]; ++e)
          o->gc_er.push_back(make_int2(nd.ent_off + e, nd.row_off + o->rowidx[nd.ent_off + e]));
      }
      if (i > 0 && lc < ndx) {
        const PlNode& np_ = o->nodes[i - 1];
        const int* cp = o->colptr.data() + np_.colptr_off;
        const int c = np_.nw + lc;
        for (int e = cp[c]; e < cp[c + 1]; ++e)
          o->gc_er.push_back(make_int2(np_.ent_off + e, np_.row_off + o->rowidx[np_.ent_off + e]));
      }
      o->gc_ptr.push_back((int)o->gc_er.size());
    }
  }
  return 0;
}

// Node programs of the factor and ADMM kernels (PlAdmmNode, state.h), one per
// distinct local structure.
int build_admm_prog(pl_ocp* o) {
  PlOcpHandle& h = o->h;
  const int N = h.oc.N, ndx = h.oc.ndx;
  o->anodes.assign(N + 1, PlAdmmNode());
  o->aprog.clear();
  o->fprog.clear();
  std::vector<std::vector<uint16_t>> aprogs, fprogs;
  std::vector<int> aoff, foff;
  h.ncpl_max = 0;
  h.nent_max = 0;
  h.chunk_max = 1;
  h.flen_max = 2;
  h.admm_fwd_asb = 0;
  auto intern = [](std::vector<std::vector<uint16_t>>& progs, std::vector<int>& off, std::vector<uint16_t>& all,
                   std::vector<uint16_t>& P) {
    while (P.size() % 4) P.push_back(0);  // 8-byte aligned programs
    for (size_t k = 0; k < progs.size(); ++k)
      if (progs[k] == P) return off[k];
    progs.push_back(P);
    off.push_back((int)all.size());
    all.insert(all.end(), P.begin(), P.end());
    return off.back();
  };
  for (int i = 0; i <= N; ++i) {
    const PlNode& nd = o->nodes[i];
    PlAdmmNode& a = o->anodes[i];
    memset(&a, 0, sizeof(a));
    a.nw = nd.nw; a.nrow = nd.nrow; a.ncol = nd.ncol; a.ncpl = nd.ncpl; a.nent = nd.nent;
    a.nunit = nd.nunit; a.ntile = nd.ntile; a.ntl = nd.ntile * (nd.ntile + 1) / 2;
    a.kmagic = (unsigned)((0x100000000ull + nd.nunit - 1) / nd.nunit);
    a.x_off = nd.x_off; a.row_off = nd.row_off; a.ent_off = nd.ent_off; a.s_off = nd.s_off;
    if (nd.nent > 65535 || nd.ncol > 65535) { pl_set_error("node too large for u16 programs"); return -1; }
    const int* cp = o->colptr.data() + nd.colptr_off;
    const int* rp = o->rowptr.data() + nd.rowptr_off;
    const int* re = o->rowent.data() + nd.csr_off;
    const int* rid = o->rowidx.data() + nd.ent_off;
    const int* ecol = o->entcol.data() + nd.ent_off;
    const int* cpl = o->cplrow.data() + nd.cpl_off;
    std::vector<uint16_t> P;
    auto mark = [&](int& field) { field = (int)P.size(); };
    auto mark2 = [&](int& field) {  // pair lists start on a 32-bit boundary
      if (P.size() & 1) P.push_back(0);
      field = (int)P.size();
    };
    auto pair = [&](int e, int c) {
      P.push_back((uint16_t)e);
      P.push_back((uint16_t)c);
    };
    // ---- factor program: rowptr, cplr, rowp
    mark(a.f_rowptr);
    for (int r = 0; r <= nd.nrow; ++r) P.push_back((uint16_t)(nd.nrow ? rp[r] : 0));
    mark(a.f_cplr);
    for (int s = 0; s < nd.ncpl; ++s) P.push_back((uint16_t)cpl[s]);
    mark2(a.f_rowp);
    for (int q = 0; nd.nrow && q < rp[nd.nrow]; ++q) pair(re[q], ecol[re[q]]);
    {  // coupling lists: w part / dx_{i+1} part of each coupling row, coupling rows of each dx_{i+1} column
      std::vector<int> cpl_idx(nd.nrow, -1);
      for (int s = 0; s < nd.ncpl; ++s) cpl_idx[cpl[s]] = s;
      std::vector<int> wp{0}, xp{0};
      std::vector<std::pair<int, int>> wl, xl;
      for (int s = 0; s < nd.ncpl; ++s) {
        const int r = cpl[s];
        for (int q = rp[r]; q < rp[r + 1]; ++q) {
          const int e = re[q], c = ecol[e];
          if (c < nd.nw) wl.push_back({e, c});
          else xl.push_back({e, c - nd.nw});
        }
        wp.push_back((int)wl.size());
        xp.push_back((int)xl.size());
      }
      std::vector<int> cp2{0};
      std::vector<std::pair<int, int>> cl;
      for (int c = 0; c < ndx && nd.ncol; ++c) {
        for (int e = cp[nd.nw + c]; e < cp[nd.nw + c + 1]; ++e)
          if (cpl_idx[rid[e]] >= 0) cl.push_back({e, cpl_idx[rid[e]]});
        cp2.push_back((int)cl.size());
      }
      if (!nd.ncol) cp2.assign(ndx + 1, 0);
      mark(a.f_cwptr);
      for (int x : wp) P.push_back((uint16_t)x);
      mark2(a.f_cwp);
      for (auto& pr : wl) pair(pr.first, pr.second);
      mark(a.f_xcptr);
      for (int x : cp2) P.push_back((uint16_t)x);
      mark2(a.f_xcp);
      for (auto& pr : cl) pair(pr.first, pr.second);
      mark(a.f_cxptr);
      for (int x : xp) P.push_back((uint16_t)x);
      mark2(a.f_cxp);
      for (auto& pr : xl) pair(pr.first, pr.second);
    }
    a.fprog = intern(fprogs, foff, o->fprog, P);
    a.flen = (int)P.size();
    h.flen_max = std::max(h.flen_max, a.flen);
    // ---- ADMM program
    P.clear();
    std::vector<int> cpl_index(nd.nrow, -1);
    for (int s = 0; s < nd.ncpl; ++s) cpl_index[cpl[s]] = s;
    // rows: entry (u16) and local column (u8) of every CSR slot; cols: local row (u8)
    // of every entry.  u8 lists are packed two per u16 word.
    if (nd.ncol > 255 || nd.nrow > 255) { pl_set_error("node with > 255 local rows / columns"); return -1; }
    auto bytes = [&](int& field, int count, auto get) {
      field = (int)P.size();
      for (int k = 0; k < count; k += 2)
        P.push_back((uint16_t)(get(k) | ((k + 1 < count ? get(k + 1) : 0) << 8)));
    };
    const int nq = nd.nrow ? rp[nd.nrow] : 0;
    mark(a.rowe);
    for (int q = 0; q < nq; ++q) P.push_back((uint16_t)re[q]);
    bytes(a.rowc, nq, [&](int q) { return ecol[re[q]]; });
    bytes(a.colr, nd.nent, [&](int e) { return rid[e]; });
    // coupling rows split into their w part and their dx_{i+1} part
    std::vector<int> cwp{0}, cxp{0};
    std::vector<std::pair<int, int>> cw, cx;
    for (int s = 0; s < nd.ncpl; ++s) {
      const int r = cpl[s];
      for (int q = rp[r]; q < rp[r + 1]; ++q) {
        const int e = re[q], c = ecol[e];
        if (c < nd.nw) cw.push_back({e, c});
        else cx.push_back({e, c - nd.nw});
      }
      cwp.push_back((int)cw.size());
      cxp.push_back((int)cx.size());
      if (cwp[s + 1] - cwp[s] > PL_ADMM_CWM) h.admm_fwd_asb = 1;
    }
    mark(a.cwptr);
    for (int x : cwp) P.push_back((uint16_t)x);
    mark2(a.cwp);
    for (auto& pr : cw) pair(pr.first, pr.second);
    mark(a.cxptr);
    for (int x : cxp) P.push_back((uint16_t)x);
    mark2(a.cxp);
    for (auto& pr : cx) pair(pr.first, pr.second);
    // per column: entries in coupling rows, as (entry, coupling index)
    std::vector<int> ccp{0}, xcp{0};
    std::vector<std::pair<int, int>> cc, xc;
    for (int c = 0; c < nd.nw && nd.ncol; ++c) {
      for (int e = cp[c]; e < cp[c + 1]; ++e)
        if (cpl_index[rid[e]] >= 0) cc.push_back({e, cpl_index[rid[e]]});
      ccp.push_back((int)cc.size());
    }
    for (int c = 0; c < ndx && nd.ncol; ++c) {
      for (int e = cp[nd.nw + c]; e < cp[nd.nw + c + 1]; ++e) {
        if (cpl_index[rid[e]] < 0) { pl_set_error("dx_{i+1} entry outside a coupling row"); return -1; }
        xc.push_back({e, cpl_index[rid[e]]});
      }
      xcp.push_back((int)xc.size());
      if (xcp[c + 1] - xcp[c] > PL_ADMM_XCM) h.admm_fwd_asb = 1;
    }
    mark(a.ccptr);
    for (int x : ccp) P.push_back((uint16_t)x);
    mark2(a.ccp);
    for (auto& pr : cc) pair(pr.first, pr.second);
    mark(a.xcptr);
    for (int x : xcp) P.push_back((uint16_t)x);
    mark2(a.xcp);
    for (auto& pr : xc) pair(pr.first, pr.second);
    // balanced chunks of <= PL_CHUNK entries for the row and column gathers
    {
      std::vector<std::pair<int, int>> ch;
      std::vector<int> ptr{0};
      for (int r = 0; r < nd.nrow; ++r) {
        for (int q = rp[r]; q < rp[r + 1]; q += PL_CHUNK) ch.push_back({q, std::min(q + PL_CHUNK, rp[r + 1])});
        ptr.push_back((int)ch.size());
      }
      a.rchn = (int)ch.size();
      mark2(a.rch);
      for (auto& c : ch) pair(c.first, c.second);
      mark(a.rchptr);
      for (int x : ptr) P.push_back((uint16_t)x);
      std::vector<int> own;
      for (int r = 0; r < nd.nrow; ++r)
        for (int k = ptr[r]; k < ptr[r + 1]; ++k) own.push_back(r);
      bytes(a.rchr, a.rchn, [&](int k) { return own[k]; });
      ch.clear();
      ptr.assign(1, 0);
      for (int c = 0; c < nd.ncol; ++c) {
        for (int e = cp[c]; e < cp[c + 1]; e += PL_CHUNK) ch.push_back({e, std::min(e + PL_CHUNK, cp[c + 1])});
        ptr.push_back((int)ch.size());
      }
      a.cchn = (int)ch.size();
      mark2(a.cch);
      for (auto& c : ch) pair(c.first, c.second);
      mark(a.cchptr);
      for (int x : ptr) P.push_back((uint16_t)x);
      own.clear();
      for (int c = 0; c < nd.ncol; ++c)
        for (int k = ptr[c]; k < ptr[c + 1]; ++k) own.push_back(c);
      bytes(a.cchc, a.cchn, [&](int k) { return own[k]; });
      h.chunk_max = std::max(h.chunk_max, std::max(a.rchn, a.cchn));
    }
    a.prog = intern(aprogs, aoff, o->aprog, P);
    a.prog_len = (int)P.size();
    h.ncpl_max = std::max(h.ncpl_max, nd.ncpl);
    h.nent_max = std::max(h.nent_max, nd.nent);
  }
  // lane-tile tables of the ADMM mat-vec: slot k of lane l holds 4x4 tile t = K l + k,
  // (I, J) its tile row / column and cidx its column-major off-diagonal index
  o->ttab.clear();
  {
    std::vector<std::pair<int, int>> keys;
    std::vector<int> offs;
    for (int i = 0; i <= N; ++i) {
      PlAdmmNode& a = o->anodes[i];
      const int T = a.ntile, K = a.nunit;
      if (K > PL_ADMM_KM) { a.ttab = -1; continue; }
      size_t k = 0;
      while (k < keys.size() && keys[k] != std::make_pair(T, K)) ++k;
      if (k == keys.size()) {
        keys.push_back({T, K});
        offs.push_back((int)o->ttab.size());
        for (int l = 0; l < 64; ++l)
          for (int s = 0; s < PL_ADMM_KM; ++s) {
            const int t = K * l + s;
            uint32_t w = 0xff000000u;  // invalid slot
            if (s < K && t < a.ntl) {
              int I = 0;
              while ((I + 1) * (I + 2) / 2 <= t) ++I;
              const int J = t - I * (I + 1) / 2;
              const int cidx = I > J ? (J * (2 * T - J - 1)) / 2 + I - J - 1 : 0;
              w = ((uint32_t)I << 24) | ((uint32_t)J << 16) | (uint32_t)cidx;
            }
            o->ttab.push_back(w);
          }
      }
      a.ttab = offs[k];
    }
    if (o->ttab.empty()) o->ttab.assign(64 * PL_ADMM_KM, 0xff000000u);
  }
  h.aprog_len = (int)o->aprog.size();
  h.prog_len_max = 0;
  for (int i = 0; i <= N; ++i) h.prog_len_max = std::max(h.prog_len_max, o->anodes[i].prog_len);
  {  // A values staged through registers: enough for the most frequent node program
    std::vector<int> cnt;
    std::vector<int> nmax;
    std::vector<int> keys;
    for (int i = 0; i <= N; ++i) {
      const int key = o->anodes[i].prog;
      size_t k = 0;
      while (k < keys.size() && keys[k] != key) ++k;
      if (k == keys.size()) { keys.push_back(key); cnt.push_back(0); nmax.push_back(0); }
      cnt[k]++;
      nmax[k] = std::max(nmax[k], o->anodes[i].nent);
    }
    size_t dom = 0;
    for (size_t k = 0; k < keys.size(); ++k)
      if (cnt[k] > cnt[dom]) dom = k;
    h.admm_asr = nmax[dom] <= 16 * 64 ? 16 : PL_ADMM_ASR_MAX;
  }
  if (!factor_supports_ndx(ndx)) {
    pl_set_error("state dimension ndx = %d is not supported by the factor kernel (24, 30, 36, 48)", ndx);
    return -1;
  }
  if (h.nrow_max > 64 * PL_ADMM_MR || h.nw_max > 64 * PL_ADMM_MV || h.ncpl_max > 64) {
    pl_set_error("ADMM kernel needs <= %d rows, <= %d columns and <= 64 coupling rows per node", 64 * PL_ADMM_MR,
                 64 * PL_ADMM_MV);
    return -1;
  }
  const PlNode& last = o->nodes[N];
  if (last.nrow != 0 || last.nw != ndx) {
    pl_set_error("terminal node must own exactly dx_N and no rows");
    return -1;
  }
  return 0;
}


// Programs of the two-stage factor (PlFacNode, state.h): the slot-owner assembly
// streams of Kt_ii and the coupling program of the Schur chain, one per distinct
// local structure, plus the launch groups of k_fnode.
int build_factor_prog(pl_ocp* o) {
  PlOcpHandle& h = o->h;
  const int N = h.oc.N, X = h.oc.ndx;
  const int NT = PL_FAC_NT;
  o->fnodes.assign(N + 1, PlFacNode());
  o->kasm.clear();
  o->kfl.clear();
  o->kcpl.clear();
  std::vector<std::vector<uint32_t>> asms, cpls;
  std::vector<std::vector<uint16_t>> fls;
  std::vector<int> asm_offs, fl_offs, cpl_offs;
  auto intern32 = [](std::vector<std::vector<uint32_t>>& progs, std::vector<int>& offs, std::vector<uint32_t>& all,
                     const std::vector<uint32_t>& P) {
    for (size_t k = 0; k < progs.size(); ++k)
      if (progs[k] == P) return offs[k];
    progs.push_back(P);
    offs.push_back((int)all.size());
    all.insert(all.end(), P.begin(), P.end());
    return offs.back();
  };
  long long fs = 0;
  std::vector<int> lds_of(N + 1), um_of(N + 1);
  int npc_max = 1, ncw_max = 2, nc_max = 1, nxc_max = 2, cwlen_max = 0;
  // General coupling (h.fac_gc) when some node's rows touch a dx_{i+1} column more than once
  // or one row touches several (whole_body_rnea include_acc = False: the RNEA rows read
  // a = (v_{i+1} - v_i) / dt); otherwise every dx_{i+1} column has exactly one coupling row.
  h.fac_gc = 0;
  for (int i = 0; i < N; ++i) {
    const PlNode& nd = o->nodes[i];
    const int* cp = o->colptr.data() + nd.colptr_off;
    const int* rid = o->rowidx.data() + nd.ent_off;
    std::vector<int> seen(nd.nrow, 0);
    for (int a = 0; a < X; ++a) {
      const int c = nd.nw + a;
      if (cp[c + 1] - cp[c] != 1 || seen[rid[cp[c]]]++) h.fac_gc = 1;
    }
  }
  for (int i = 0; i <= N; ++i) {
    const PlNode& nd = o->nodes[i];
    PlFacNode& f = o->fnodes[i];
    memset(&f, 0, sizeof(f));
    const int nw = nd.nw, U = nd.nu;
    f.nw = nw; f.nu = U; f.nrow = nd.nrow; f.nent = nd.nent; f.ent_off = nd.ent_off; f.row_off = nd.row_off;
    f.x_off = nd.x_off; f.s_off = nd.s_off; f.nunit = nd.nunit; f.ntl = nd.ntile * (nd.ntile + 1) / 2;
    if (U > 64) { pl_set_error("factor kernel: node with %d > 64 inputs", U); return -1; }
    if (nd.nent >= 0x7fff) { pl_set_error("factor kernel: node with %d entries", nd.nent); return -1; }
    const int* cp = o->colptr.data() + nd.colptr_off;
    const int* rp = o->rowptr.data() + nd.rowptr_off;
    const int* re = o->rowent.data() + nd.csr_off;
    const int* rid = o->rowidx.data() + nd.ent_off;
    const int* ecol = o->entcol.data() + nd.ent_off;
    // ---- assembly: triples (rho_r a_e1, a_e2) of every lower slot of Kt_ii, rows in order
    const int nslot = nw * (nw + 1) / 2;
    std::vector<std::vector<uint32_t>> trip(nslot);
    for (int r = 0; r < nd.nrow; ++r) {
      for (int q1 = rp[r]; q1 < rp[r + 1]; ++q1) {
        const int e1 = re[q1], c1 = ecol[e1];
        if (c1 >= nw) continue;
        for (int q2 = rp[r]; q2 < rp[r + 1]; ++q2) {
          const int e2 = re[q2], c2 = ecol[e2];
          if (c2 > c1) continue;
          trip[c1 * (c1 + 1) / 2 + c2].push_back((uint32_t)e1 | ((uint32_t)e2 << 16));
        }
      }
    }
    std::vector<int> order;
    for (int sl = 0; sl < nslot; ++sl)
      if (!trip[sl].empty()) order.push_back(sl);
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return trip[a].size() > trip[b].size(); });
    std::vector<std::vector<uint32_t>> lane_w(NT);
    std::vector<std::vector<uint16_t>> lane_f(NT);
    std::vector<int> load(NT, 0);
    for (int sl : order) {
      int best = 0;
      for (int t = 1; t < NT; ++t)
        if (load[t] < load[best]) best = t;
      for (size_t k = 0; k < trip[sl].size(); ++k)
        lane_w[best].push_back(trip[sl][k] | (k + 1 == trip[sl].size() ? 0x8000u : 0u));
      lane_f[best].push_back((uint16_t)sl);
      load[best] += (int)trip[sl].size();
    }
    int L = 0, F = 0;
    for (int t = 0; t < NT; ++t) {
      L = std::max(L, (int)lane_w[t].size());
      F = std::max(F, (int)lane_f[t].size());
    }
    const uint32_t zero = (uint32_t)nd.nent | ((uint32_t)nd.nent << 16);
    std::vector<uint32_t> A((size_t)L * NT, zero);
    std::vector<uint16_t> Fl((size_t)std::max(F, 1) * NT, 0);
    for (int t = 0; t < NT; ++t) {
      for (size_t k = 0; k < lane_w[t].size(); ++k) A[k * NT + t] = lane_w[t][k];
      for (size_t k = 0; k < lane_f[t].size(); ++k) Fl[k * NT + t] = lane_f[t][k];
    }
    if (nslot > 65535) { pl_set_error("factor kernel: node block too large"); return -1; }
    f.asm_len = L;
    f.fl_len = F;
    f.asm_off = A.empty() ? 0 : intern32(asms, asm_offs, o->kasm, A);
    {
      size_t k = 0;
      for (; k < fls.size(); ++k)
        if (fls[k] == Fl) break;
      if (k == fls.size()) {
        fls.push_back(Fl);
        fl_offs.push_back((int)o->kfl.size());
        o->kfl.insert(o->kfl.end(), Fl.begin(), Fl.end());
      }
      f.fl_off = fl_offs[k];
    }
    // ---- coupling program (i < N)
    std::vector<uint32_t> C;
    if (i < N && h.fac_gc) {
      // general form: coupling rows s (rows with a dx_{i+1} entry), Z = R - R Vc S Vc^T R over
      // them and E_{i+1} = Wc^T Z Wc.  Words: crow[nc] | cwptr[nc + 1] | pcl[npc] |
      // cw (e | col << 16 | pc << 24)[ncw] | xcptr[X + 1] | xc (e | s << 16)[nxc]
      const int* cpl = o->cplrow.data() + nd.cpl_off;
      const int nc = nd.ncpl;
      std::vector<int> sidx_of(nd.nrow, -1);
      for (int q = 0; q < nc; ++q) sidx_of[cpl[q]] = q;
      std::vector<int> used(nw, 0);
      std::vector<std::vector<std::pair<int, int>>> cw(nc);
      for (int q = 0; q < nc; ++q)
        for (int t = rp[cpl[q]]; t < rp[cpl[q] + 1]; ++t) {
          const int e = re[t], c = ecol[e];
          if (c < nw) { cw[q].push_back({e, c}); used[c] = 1; }
        }
      std::vector<int> pcl, pcof(nw, -1);
      for (int c = 0; c < nw; ++c)
        if (used[c]) { pcof[c] = (int)pcl.size(); pcl.push_back(c); }
      if (nw > 255 || pcl.size() > 255 || nc > 64) { pl_set_error("factor kernel: node too wide"); return -1; }
      for (int q = 0; q < nc; ++q) C.push_back((uint32_t)cpl[q]);
      uint32_t acc = 0;
      for (int q = 0; q <= nc; ++q) {
        C.push_back(acc);
        if (q < nc) acc += (uint32_t)cw[q].size();
      }
      for (int c : pcl) C.push_back((uint32_t)c);
      for (int q = 0; q < nc; ++q)
        for (auto& pr : cw[q])
          C.push_back((uint32_t)pr.first | ((uint32_t)pr.second << 16) | ((uint32_t)pcof[pr.second] << 24));
      uint32_t nx = 0;
      std::vector<uint32_t> xl;
      for (int a = 0; a <= X; ++a) {
        C.push_back(nx);
        if (a == X) break;
        for (int e = cp[nw + a]; e < cp[nw + a + 1]; ++e) {
          if (sidx_of[rid[e]] < 0) { pl_set_error("factor kernel: dx_{i+1} entry outside a coupling row"); return -1; }
          xl.push_back((uint32_t)e | ((uint32_t)sidx_of[rid[e]] << 16));
          ++nx;
        }
      }
      C.insert(C.end(), xl.begin(), xl.end());
      f.npc = (int)pcl.size();
      f.nc = nc;
      npc_max = std::max(npc_max, f.npc);
      ncw_max = std::max(ncw_max, (int)acc);
      nc_max = std::max(nc_max, nc);
      nxc_max = std::max(nxc_max, (int)nx);
      f.cp_off = intern32(cpls, cpl_offs, o->kcpl, C);
    } else if (i < N) {
      std::vector<int> crow(X), cent(X);
      std::vector<int> owner(nd.nrow, -1);
      for (int a = 0; a < X; ++a) {
        const int c = nw + a;
        if (cp[c + 1] - cp[c] != 1) {
          pl_set_error("factor kernel: dx_{i+1} column %d of node %d is not owned by exactly one row", a, i);
          return -1;
        }
        const int e = cp[c];
        crow[a] = rid[e];
        cent[a] = e;
        if (owner[crow[a]] >= 0) {
          pl_set_error("factor kernel: row %d of node %d couples more than one dx_{i+1} column", crow[a], i);
          return -1;
        }
        owner[crow[a]] = a;
      }
      std::vector<int> used(nw, 0);
      std::vector<std::vector<std::pair<int, int>>> cw(X);
      for (int a = 0; a < X; ++a) {
        const int r = crow[a];
        for (int q = rp[r]; q < rp[r + 1]; ++q) {
          const int e = re[q], c = ecol[e];
          if (c < nw) { cw[a].push_back({e, c}); used[c] = 1; }
        }
      }
      std::vector<int> pcl, pcof(nw, -1);
      for (int c = 0; c < nw; ++c)
        if (used[c]) { pcof[c] = (int)pcl.size(); pcl.push_back(c); }
      if (nw > 255 || pcl.size() > 255) { pl_set_error("factor kernel: node too wide"); return -1; }
      for (int a = 0; a < X; ++a) C.push_back((uint32_t)crow[a]);
      for (int a = 0; a < X; ++a) C.push_back((uint32_t)cent[a]);
      uint32_t q = 0;
      for (int a = 0; a <= X; ++a) {
        C.push_back(q);
        if (a < X) q += (uint32_t)cw[a].size();
      }
      for (int c : pcl) C.push_back((uint32_t)c);
      for (int a = 0; a < X; ++a)
        for (auto& pr : cw[a])
          C.push_back((uint32_t)pr.first | ((uint32_t)pr.second << 16) | ((uint32_t)pcof[pr.second] << 24));
      f.npc = (int)pcl.size();
      npc_max = std::max(npc_max, f.npc);
      ncw_max = std::max(ncw_max, (int)q);
      for (int a = 0; a < X; ++a) cwlen_max = std::max(cwlen_max, (int)cw[a].size());
      f.cp_off = intern32(cpls, cpl_offs, o->kcpl, C);
    }
    f.fs_off = fs;
    fs += (long long)X * X + (long long)U * X + (long long)U * U;
    fs = (fs + 31) & ~31LL;
    // k_fnode LDS: packed lower Kt (even) | A values x 2 (assembly), then the pivot buffer
    // [2][512] (sweep), then G (after the sweep): the three share one region
    const int nK = (nslot + 1) & ~1;
    const int r2 = (std::max(std::max(2 * (nd.nent + 1), U * X), 1024) + 1) & ~1;
    lds_of[i] = (nK + r2) * 8;
    um_of[i] = U <= 40 ? 40 : 64;
  }
  h.fs_stride = std::max(fs, 32LL);
  // launch groups: maximal runs of consecutive nodes with the same LDS size and register class
  h.nfgroup = 0;
  for (int i = 0; i <= N;) {
    int j = i + 1;
    while (j <= N && lds_of[j] == lds_of[i] && um_of[j] == um_of[i]) ++j;
    if (h.nfgroup == PL_FAC_MAXGROUPS) { pl_set_error("factor kernel: too many node groups"); return -1; }
    h.fg_i0[h.nfgroup] = i;
    h.fg_n[h.nfgroup] = j - i;
    h.fg_lds[h.nfgroup] = lds_of[i];
    h.fg_um[h.nfgroup] = um_of[i];
    ++h.nfgroup;
    i = j;
  }
  for (int g = 0; g < h.nfgroup; ++g)
    if (h.fg_lds[g] > 160 * 1024) { pl_set_error("factor kernel: node needs %d bytes of LDS", h.fg_lds[g]); return -1; }
  // k_fchain LDS: packed lower S (even) | Y / transpose buffer, the pivot buffer during the
  // sweep | E (packed lower) | staged coupling values (ncw + 2 X) | timing stamps (74 KB for
  // B2G rnea: two chains per CU, which the latency-bound chain needs)
  // (general coupling: Y [npc][nc], then T = Z Wc [nc][X] in the Y buffer, and behind the
  // stamps Z [nc][nc], the staged dx_{i+1} values [nxc] and rho of the coupling rows [nc])
  const int nS = (h.nw_max * (h.nw_max + 1) / 2 + 1) & ~1;
  int ny = std::max(std::max((npc_max + 1) / 2 * X, X * (X + 1)), 1024);  // Y in two halves (k_fchain)
  if (h.fac_gc) ny = std::max(ny, std::max(npc_max, X) * nc_max);
  ny = (ny + 1) & ~1;
  const int nE = (X * (X + 1) / 2 + 1) & ~1;
  h.fchain_ny = ny;
  // short coupling-row lists (the integration rows of rnea / acc: 2 entries): E_{i+1} straight
  // from S (4 products per entry) instead of through Y
  h.fchain_short = !h.fac_gc && cwlen_max <= 4;
  h.fchain_ncw = (ncw_max + 1) & ~1;
  h.fchain_nc = h.fac_gc ? nc_max : 0;
  h.fchain_nxc = h.fac_gc ? (nxc_max + 1) & ~1 : 0;
  const int ngc = h.fac_gc ? ((nc_max * nc_max + h.fchain_nxc + nc_max + 1) & ~1) : 0;
  h.fchain_lds = (nS + ny + nE + h.fchain_ncw + 2 * X + 10 + ngc) * 8;  // + timing stamps
  if (h.fchain_lds > 160 * 1024) { pl_set_error("factor kernel: chain needs %d bytes of LDS", h.fchain_lds); return -1; }
  if (o->kasm.empty()) o->kasm.assign(NT, 0);
  if (o->kcpl.empty()) o->kcpl.assign(4, 0);
  return 0;
}

template <class T>
int dalloc(pl_ocp* o, T** p, size_t count) {
  void* q = nullptr;
  count += 256;  // slack: kernels issue clamped, unconditional loads up to one row past the end
  hipError_t e = hipMalloc(&q, count * sizeof(T));
  if (e != hipSuccess) {
    pl_set_error("hipMalloc(%zu bytes): %s", count * sizeof(T), hipGetErrorString(e));
    return -2;
  }
  (void)hipMemset(q, 0, count * sizeof(T));
  o->allocs.push_back(q);
  *p = (T*)q;
  return 0;
}

// Work list of the Jacobian kernel (k_eval_jac): one lane per non-empty local column.
// Columns whose dual pass runs the tree / ABA / centroidal recursion come first, packed
// 64 per wave ACROSS node boundaries and padded to whole waves; then the columns that
// skip it (dx_{i+1}; rnea tau_j; centroidal h), which are cheap.  The classification
// mirrors node_rows' skip logic (rows.h); it only affects the schedule.
int build_jac_list(pl_ocp* o, std::vector<int2>& list) {
  const PlOcpConst& O = o->h.oc;
  std::vector<int2> ex, ch;
  for (int i = 0; i < o->h.N; ++i) {
    const PlNode& nd = o->nodes[i];
    const int* cp = o->colptr.data() + nd.colptr_off;
    for (int lc = 0; lc < nd.ncol; ++lc) {
      if (cp[lc] == cp[lc + 1]) continue;
      bool cheap;
      if (lc >= nd.nw) {
        cheap = !(O.dyn == PL_DYN_RNEAFD && lc - nd.nw >= O.nv);  // FD: dv_{i+1} enters the RNEA
      } else if (lc < O.ndx) {
        cheap = O.dyn == PL_DYN_CV && lc < 6;  // (without the base, h enters v_b: not cheap)
      } else {
        const int k = lc - O.ndx;
        cheap = PL_IS_RNEA(O.dyn) && k >= O.na + O.nf;
      }
      (cheap ? ch : ex).push_back(make_int2(i, lc));
    }
  }
  while (ex.size() % 64) ex.push_back(make_int2(-1, -1));
  // a wave's lanes hold at most PL_JAC_SLOTS consecutive nodes (shared-value slots)
  for (size_t w = 0; w < ex.size(); w += 64) {
    int last = ex[w].x;
    for (size_t q = w; q < w + 64; ++q) last = std::max(last, ex[q].x);
    if (last - ex[w].x >= PL_JAC_SLOTS) {
      pl_set_error("Jacobian wave spans more than %d nodes", PL_JAC_SLOTS);
      return -1;
    }
  }
  list = ex;
  list.insert(list.end(), ch.begin(), ch.end());
  return 0;
}

template <class T>
int upload(pl_ocp* o, T** p, const std::vector<T>& v) {
  if (dalloc(o, p, v.size())) return -2;
  if (!v.empty()) PL_CHECK_HIP(hipMemcpy(*p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return 0;
}

}  // namespace

// ADMM kernel selection (the three give the same iterates to round-off):
//   sweep   k_admm: one wave per problem, node-by-node block sweeps (HBM-bound at B >= 1024)
//   sweep2  k_admm2: two waves per problem
//   chain   k_admm_rc: reduced chain, one workgroup of 8 waves per problem (small batches)
// AUTO: chain up to PL_ADMM_CHAIN_MAX_B problems when supported, else sweep2 up to 512
// problems (idle SIMDs below 4 x 256), else sweep.  The chain
// buffers are allocated on first selection.
#define PL_ADMM_CHAIN_MAX_B 256  // measured: profiles/r03b (B2 aba B=256 13.8 -> 5.3 ms per launch; B2G at 512 the sweep2 wins)
int admm_select(pl_ocp* o, int kind) {
  PlOcpHandle& h = o->h;
  if (kind == PL_ADMM_AUTO) {
    if (h.B <= PL_ADMM_CHAIN_MAX_B && admm_rc_supported(&h)) kind = PL_ADMM_CHAIN;
    else kind = (h.B <= 512 && admm2_supported(&h)) ? PL_ADMM_SWEEP2 : PL_ADMM_SWEEP;
  }
  if (kind == PL_ADMM_SWEEP2 && !admm2_supported(&h)) { pl_set_error("sweep2 ADMM kernel does not support this OCP"); return -1; }
  if (kind == PL_ADMM_CHAIN && !admm_rc_supported(&h)) { pl_set_error("chain ADMM kernel does not support this OCP"); return -1; }
  if (kind == PL_ADMM_CHAIN && o->on_device && !h.d.CH) {
    if (dalloc(o, &h.d.CH, (size_t)h.B * h.ch_stride) || dalloc(o, &h.d.chv, (size_t)h.B * h.chv_stride)) return -2;
  }
  h.admm_rc = kind == PL_ADMM_CHAIN ? 1 : 0;
  h.admm_waves = kind == PL_ADMM_SWEEP2 ? 2 : 1;
  return 0;
}

extern "C" int pl_ocp_create(const pl_model* model, const pl_ocp_desc* d, int batch, int device, pl_ocp** out) {
  if (!model || !d || !out || batch <= 0) { pl_set_error("bad arguments"); return -1; }
  if (d->dynamics < 0 || d->dynamics > 4) { pl_set_error("Unknown dynamics type: %d", d->dynamics); return -1; }
  if (d->nodes < 2 || d->n_feet != 4) { pl_set_error("need nodes >= 2 and 4 feet"); return -1; }
  pl_ocp* o = new pl_ocp();
  PlOcpHandle& h = o->h;
  memset(&h, 0, sizeof(h));
  h.model = model->m;
  PlOcpConst& O = h.oc;
  memset(&O, 0, sizeof(O));
  const PlModel& M = h.model;
  O.dyn = d->dynamics;
  // whole_body_acc / centroidal_acc without the base in u share the ACCNB rows
  if ((O.dyn == PL_DYN_ACC || O.dyn == PL_DYN_CA) && !d->include_base) O.dyn = PL_DYN_ACCNB;
  // centroidal_vel without the base velocity in u (the class default, ocp_centroidal_vel.py:9-23)
  if (O.dyn == PL_DYN_CV && !d->include_base) O.dyn = PL_DYN_CVNB;
  // whole_body_rnea with finite-difference accelerations (include_acc = False,
  // ocp_whole_body_rnea.py:21-26, 183-191): u = [f | tau_j], no dv_{i+1} rows; the RNEA rows
  // of node i read dv_{i+1}, so the factor takes the general coupling program (fac_gc)
  if (O.dyn == PL_DYN_RNEA && !d->include_acc) O.dyn = PL_DYN_RNEAFD;
  O.N = d->nodes;
  O.nq = M.nq;
  O.nv = M.nv;
  O.nj = M.nq - 7;
  O.nfeet = 4;
  const bool has_ext = d->ext_force_frame >= 0;
  const bool has_arm = d->arm_ee_frame >= 0;
  O.nf = 12 + (has_ext ? 3 : 0);
  O.nee = 4 + (has_ext ? 1 : 0);
  const bool cv = PL_IS_CV(O.dyn);
  O.nx = cv ? 6 + M.nq : M.nq + M.nv;   // centroidal_vel: x = [h, q] (ocp_centroidal_vel.py:50-52)
  O.ndx = cv ? 6 + M.nv : 2 * M.nv;
  O.na = (O.dyn == PL_DYN_RNEA || O.dyn == PL_DYN_ACC || O.dyn == PL_DYN_CA) ? M.nv
         : (O.dyn == PL_DYN_ACCNB ? M.nq - 7 : 0);
  O.tau_nodes = PL_IS_RNEA(O.dyn) ? d->tau_nodes : 0;
  O.mu = d->mu;
  for (int k = 0; k < 4; ++k) O.feet[k] = frame_ref(model, d->foot_frames[k]);
  O.ext = frame_ref(model, d->ext_force_frame);
  O.arm = frame_ref(model, d->arm_ee_frame);
  O.base = frame_ref(model, d->base_frame);
  if (has_arm && !O.base.valid) { pl_set_error("arm velocity needs the base_link frame"); delete o; return -1; }
  for (int k = 0; k < M.nq; ++k) O.q0[k] = d->q0[k];
  for (int k = 0; k < O.nj; ++k) {
    O.pos_min[k] = d->joint_pos_min[k];
    O.pos_max[k] = d->joint_pos_max[k];
    O.vel_max[k] = d->joint_vel_max[k];
    O.tau_max[k] = d->joint_torque_max[k];
  }
  build_blocks(O, has_ext, has_arm);
  // parameter layout (Opti declaration order)
  int off = 0;
  auto take = [&](int len) { int r = off; off += len; return r; };
  const int nu0 = pl::node_nu(O, 0);
  O.P.x_init = take(O.nx);
  O.P.dt_min = take(1);
  O.P.dt_max = take(1);
  O.P.contact = take(4 * O.N);
  O.P.swing = take(4 * O.N);
  O.P.n_contacts = take(1);
  O.P.swing_period = take(1);
  O.P.swing_height = take(1);
  O.P.swing_vel_limits = take(2);
  O.P.Q_diag = take(O.ndx);
  O.P.R_diag = take(nu0);
  O.P.base_vel_des = take(6);
  O.P.ext_force_des = take(3);
  O.P.arm_vel_des = take(3);
  if (PL_IS_RNEA(O.dyn)) {
    O.P.tau_prev = take(O.nj);
    O.P.W_diag = take(O.nj);
  } else {
    O.P.tau_prev = O.P.W_diag = -1;
  }
  O.P.np = off;
  if (build_layout(o) || build_admm_prog(o) || build_factor_prog(o)) { delete o; return -1; }
  O.n = h.n;
  O.m = h.m;
  h.B = batch;
  h.N = O.N;
  h.np = O.P.np;
  h.nx = O.nx;
  h.ndx = O.ndx;
  h.set.rho = d->rho;
  h.set.sigma = d->sigma;
  h.set.alpha = d->alpha;
  h.set.eps_abs = d->eps_abs;
  h.set.eps_rel = d->eps_rel;
  h.set.eps_prim_inf = d->eps_prim_inf;
  h.set.eps_dual_inf = d->eps_dual_inf;
  h.set.max_iter = d->max_iter;
  h.set.scaling = d->scaling;
  h.set.check_termination = d->check_termination;
  h.set.warm_start = d->warm_start;
  h.sqp_iters = 1;
  h.solver = PL_SOLVER_OSQP;
  // Fatrop settings of the reference (ocp.py:254-262) + the restatement's constants
  // (oracle/ip_ref.py IP_SETTINGS)
  h.ip = PlIpSettings{1e-3, 1e-4, 1e-7, 1e-2, 1e-8, 1e-4, 10, 12, 8, 0, 1e-7};
  h.ip_hess = PL_IP_HESS_EXACT;  // the Lagrangian Hessian (pl_ip_settings.hessian)
  // ADMM kernel (admm_select below): PL_ADMM_KERNEL = sweep | sweep2 | chain | auto overrides
  // the batch-size rule at creation, pl_ocp_set_admm_kernel afterwards.
  h.admm_waves = 1;
  h.admm_rc = 0;
  h.rc_waves = 8;
  h.ruiz_fused = !(getenv("PL_RUIZ_FUSED") && atoi(getenv("PL_RUIZ_FUSED")) == 0);
  h.ch_stride = rc_ch_stride(h.N, h.ndx);
  h.chv_stride = rc_chv_stride(h.N, h.ndx);
  h.gait_type = d->gait_type;
  h.gait_period = d->gait_period;
  h.swing_period = d->gait_type == 0 ? 0.5 * d->gait_period : (d->gait_type == 1 ? 0.25 * d->gait_period : d->gait_period);
  o->h_params.assign((size_t)batch * h.np, 0.0);
  o->on_device = device >= 0;
  h.device = device;
  if (!o->on_device) { *out = o; return 0; }

  if (hipSetDevice(device) != hipSuccess) {
    (void)hipGetLastError();  // do not leave the failure as the thread's sticky last error
    pl_set_error("hipSetDevice(%d) failed", device);
    delete o;
    return -2;
  }
  if (hipStreamCreateWithFlags(&h.stream, hipStreamNonBlocking) != hipSuccess) {
    pl_set_error("hipStreamCreate failed");
    delete o;
    return -2;
  }
  for (int k = 0; k < 5; ++k) hipEventCreate(&o->ev[k]);
  PlDev& D = h.d;
  const size_t B = batch;
  int rc = 0;
  rc |= dalloc(o, &D.model, 1);
  rc |= dalloc(o, &D.oc, 1);
  rc |= upload(o, &D.nodes, o->nodes);
  rc |= upload(o, &D.colptr, o->colptr);
  rc |= upload(o, &D.rowidx, o->rowidx);
  rc |= upload(o, &D.entcol, o->entcol);
  rc |= upload(o, &D.rowptr, o->rowptr);
  rc |= upload(o, &D.rowent, o->rowent);
  rc |= upload(o, &D.cplrow, o->cplrow);
  rc |= upload(o, &D.rownode, o->rownode);
  rc |= upload(o, &D.colnode, o->colnode);
  rc |= upload(o, &D.gr_ptr, o->gr_ptr);
  rc |= upload(o, &D.gr_ec, o->gr_ec);
  rc |= upload(o, &D.gc_ptr, o->gc_ptr);
  rc |= upload(o, &D.gc_er, o->gc_er);
  if (h.n < 65536 && h.m < 65536) {  // entry coordinates of the fused Ruiz kernel (k_qp.hip)
    std::vector<uint32_t> erc(h.nnz);
    for (int i = 0; i < h.N; ++i) {
      const PlNode& nd = o->nodes[i];
      for (int e = 0; e < nd.nent; ++e) {
        const int lc = o->entcol[nd.ent_off + e];
        const int r = nd.row_off + o->rowidx[nd.ent_off + e];
        const int j = lc < nd.nw ? nd.x_off + lc : o->nodes[i + 1].x_off + (lc - nd.nw);
        erc[nd.ent_off + e] = ((uint32_t)r << 16) | (uint32_t)j;
      }
    }
    rc |= upload(o, &D.erc, erc);
  }
  rc |= upload(o, &D.anodes, o->anodes);
  rc |= upload(o, &D.aprog, o->aprog);
  rc |= upload(o, &D.fprog, o->fprog);
  rc |= upload(o, &D.ttab, o->ttab);
  rc |= upload(o, &D.fnodes, o->fnodes);
  rc |= upload(o, &D.kasm, o->kasm);
  rc |= upload(o, &D.kfl, o->kfl);
  rc |= upload(o, &D.kcpl, o->kcpl);
  {
    std::vector<int2> jl;
    if (build_jac_list(o, jl)) {
      pl_ocp_destroy(o);
      return -1;
    }
    h.jl_len = (int)jl.size();
    rc |= upload(o, &D.jlist, jl);
  }
  const size_t n = h.n, m = h.m, nnz = h.nnz;
  rc |= dalloc(o, &D.p, B * h.np);
  rc |= dalloc(o, &D.x, B * n);
  rc |= dalloc(o, &D.x0, B * n);
  rc |= dalloc(o, &D.g, B * m);
  rc |= dalloc(o, &D.lbg, B * m);
  rc |= dalloc(o, &D.ubg, B * m);
  rc |= dalloc(o, &D.grad, B * n);
  rc |= dalloc(o, &D.Araw, B * nnz);
  rc |= dalloc(o, &D.P, B * n);
  rc |= dalloc(o, &D.As, B * nnz);
  rc |= dalloc(o, &D.qs, B * n);
  rc |= dalloc(o, &D.ls, B * m);
  rc |= dalloc(o, &D.us, B * m);
  rc |= dalloc(o, &D.rho, B * m);
  rc |= dalloc(o, &D.rhoc, B * (size_t)(h.N + 1) * std::max(h.ncpl_max, 1));
  rc |= dalloc(o, &D.Acpl, B * (size_t)(h.N + 1) * PL_ACPL);
  rc |= dalloc(o, &D.D, B * n);
  rc |= dalloc(o, &D.E, B * m);
  rc |= dalloc(o, &D.cs, B);
  rc |= dalloc(o, &D.Ps, B * n);
  rc |= dalloc(o, &D.xa, B * n);
  rc |= dalloc(o, &D.za, B * m);
  rc |= dalloc(o, &D.ya, B * m);
  rc |= dalloc(o, &D.rhs, B * n);
  rc |= dalloc(o, &D.bt, B * n);
  rc |= dalloc(o, &D.dxs, B * n);
  rc |= dalloc(o, &D.dys, B * m);
  rc |= dalloc(o, &D.aty, B * n);
  rc |= dalloc(o, &D.step, B * n);
  rc |= dalloc(o, &D.S, B * (size_t)h.S_stride);
  rc |= dalloc(o, &D.FS, B * (size_t)h.fs_stride);
  rc |= dalloc(o, &D.work, B * 8);
  rc |= dalloc(o, &D.chk, B * (size_t)(h.N + 1) * 8);
  rc |= dalloc(o, &D.info, B);
  rc |= dalloc(o, &D.t0, B);
  rc |= dalloc(o, &D.xstate, B * (size_t)h.nx);
  D.dbg = nullptr;
  if (getenv("PL_ADMM_TIMING") && atoi(getenv("PL_ADMM_TIMING")) > 0) rc |= dalloc(o, &D.dbg, B * 32);
  if (rc) { pl_ocp_destroy(o); return -2; }
  {
    int kind = PL_ADMM_AUTO;
    if (const char* k = getenv("PL_ADMM_KERNEL")) {
      if (!strcmp(k, "sweep")) kind = PL_ADMM_SWEEP;
      else if (!strcmp(k, "sweep2")) kind = PL_ADMM_SWEEP2;
      else if (!strcmp(k, "chain")) kind = PL_ADMM_CHAIN;
    }
    if (admm_select(o, kind)) { pl_ocp_destroy(o); return -2; }
  }
  o->mpc_graph_off = getenv("PL_MPC_GRAPH") && atoi(getenv("PL_MPC_GRAPH")) == 0;
  if (hipMemcpy(D.model, &h.model, sizeof(PlModel), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(D.oc, &h.oc, sizeof(PlOcpConst), hipMemcpyHostToDevice) != hipSuccess) {
    pl_set_error("upload of model tables failed");
    pl_ocp_destroy(o);
    return -2;
  }
  *out = o;
  return 0;
}

static void cas_forget(const pl_ocp* o);

extern "C" void pl_ocp_destroy(pl_ocp* o) {
  if (!o) return;
  cas_forget(o);  // a bound CasADi handle must not outlive its OCP
  if (o->on_device) {
    hipSetDevice(o->h.device);
    hipStreamSynchronize(o->h.stream);
    for (void* p : o->allocs) hipFree(p);
    for (int k = 0; k < 5; ++k) hipEventDestroy(o->ev[k]);
    if (o->mpc_graph) hipGraphExecDestroy(o->mpc_graph);
    hipStreamDestroy(o->h.stream);
  }
  delete o;
}

extern "C" int pl_ocp_dims(const pl_ocp* o, int* n, int* m, int* np, int* nnz) {
  if (!o) { pl_set_error("null handle"); return -1; }
  if (n) *n = o->h.n;
  if (m) *m = o->h.m;
  if (np) *np = o->h.np;
  if (nnz) *nnz = o->h.nnz;
  return 0;
}

extern "C" int pl_ocp_pattern(const pl_ocp* o, int* rows, int* cols) {
  if (!o || !rows || !cols) { pl_set_error("null argument"); return -1; }
  const int N = o->h.N;
  for (int i = 0; i < N; ++i) {
    const PlNode& nd = o->nodes[i];
    for (int e = 0; e < nd.nent; ++e) {
      const int lc = o->entcol[nd.ent_off + e];
      rows[nd.ent_off + e] = nd.row_off + o->rowidx[nd.ent_off + e];
      cols[nd.ent_off + e] = lc < nd.nw ? nd.x_off + lc : o->nodes[i + 1].x_off + (lc - nd.nw);
    }
  }
  return 0;
}

static void prof_collect(PlOcpHandle* h);

#define REQUIRE_DEVICE(o)                                              \
  do {                                                                 \
    if (!(o) || !(o)->on_device) {                                     \
      pl_set_error("handle has no device (created with device = -1)"); \
      return -1;                                                       \
    }                                                                  \
    (void)hipSetDevice((o)->h.device);                                 \
    (void)hipGetLastError(); /* errors of earlier calls were reported there */ \
  } while (0)

extern "C" int pl_ocp_set_params(pl_ocp* o, const double* P) {
  REQUIRE_DEVICE(o);
  const size_t len = (size_t)o->h.B * o->h.np;
  memcpy(o->h_params.data(), P, len * sizeof(double));
  PL_CHECK_HIP(hipMemcpyAsync(o->h.d.p, P, len * sizeof(double), hipMemcpyHostToDevice, o->h.stream));
  PL_CHECK_HIP(hipStreamSynchronize(o->h.stream));
  return 0;
}

extern "C" int pl_ocp_get_params(pl_ocp* o, double* P) {
  REQUIRE_DEVICE(o);
  PL_CHECK_HIP(hipMemcpyAsync(P, o->h.d.p, (size_t)o->h.B * o->h.np * sizeof(double), hipMemcpyDeviceToHost,
                              o->h.stream));
  PL_CHECK_HIP(hipStreamSynchronize(o->h.stream));
  return 0;
}

extern "C" int pl_ocp_set_x(pl_ocp* o, const double* X) {
  REQUIRE_DEVICE(o);
  PL_CHECK_HIP(hipMemcpyAsync(o->h.d.x, X, (size_t)o->h.B * o->h.n * sizeof(double), hipMemcpyHostToDevice,
                              o->h.stream));
  PL_CHECK_HIP(hipStreamSynchronize(o->h.stream));
  return 0;
}

extern "C" int pl_ocp_get_x(pl_ocp* o, double* X) {
  REQUIRE_DEVICE(o);
  PL_CHECK_HIP(hipMemcpyAsync(X, o->h.d.x, (size_t)o->h.B * o->h.n * sizeof(double), hipMemcpyDeviceToHost,
                              o->h.stream));
  PL_CHECK_HIP(hipStreamSynchronize(o->h.stream));
  return 0;
}

extern "C" int pl_ocp_get_step(pl_ocp* o, double* dx) {
  REQUIRE_DEVICE(o);
  PL_CHECK_HIP(hipMemcpyAsync(dx, o->h.d.step, (size_t)o->h.B * o->h.n * sizeof(double), hipMemcpyDeviceToHost,
                              o->h.stream));
  PL_CHECK_HIP(hipStreamSynchronize(o->h.stream));
  return 0;
}

extern "C" int pl_ocp_init_solver(pl_ocp* o) {
  REQUIRE_DEVICE(o);
  launch_hess(&o->h);
  launch_reset_iterates(&o->h);
  launch_reset_info(&o->h);
  PL_CHECK_HIP(hipGetLastError());
  PL_CHECK_HIP(hipStreamSynchronize(o->h.stream));
  return 0;
}

static int enqueue_solve(pl_ocp* o, bool timed) {
  PlOcpHandle* h = &o->h;
  if (timed) hipEventRecord(o->ev[0], h->stream);
  // sqp_data(x, p): grad_f, J_g, g, lbg, ubg (ocp.py:386)
  launch_eval_values(h, h->d.x);
  launch_eval_jac(h);
  launch_objective(h);
  if (timed) hipEventRecord(o->ev[1], h->stream);
  // osqp.update(q, Ax, l, u): rescale + refactor (ocp.py:391-395)
  launch_qp_setup(h);
  launch_factor(h);
  if (timed) hipEventRecord(o->ev[2], h->stream);
  // osqp.solve() (ocp.py:401)
  launch_reset_info(h);
  if (!h->set.warm_start) launch_reset_iterates(h);
  launch_admm_init(h);
  const int ct = h->set.check_termination > 0 ? h->set.check_termination : h->set.max_iter;
  int it = 0;
  while (it < h->set.max_iter) {
    const int nit = std::min(ct, h->set.max_iter - it);
    it += nit;
    const bool final = it >= h->set.max_iter;
    const bool at_check = (h->set.check_termination > 0 && it % h->set.check_termination == 0);
    launch_admm(h, nit, (at_check || final) ? 1 : 0, it - nit);
    if (at_check || final) launch_check(h, it, final ? 1 : 0);
  }
  launch_unscale(h);
  if (timed) hipEventRecord(o->ev[3], h->stream);
  // _armijo_line_search (ocp.py:406, 430-480)
  launch_line_search(h);
  if (timed) hipEventRecord(o->ev[4], h->stream);
  return 0;
}

static int fetch_stats(pl_ocp* o, pl_stats* stats) {
  if (!stats) return 0;
  std::vector<PlProbInfo> info(o->h.B);
  PL_CHECK_HIP(hipMemcpyAsync(info.data(), o->h.d.info, o->h.B * sizeof(PlProbInfo), hipMemcpyDeviceToHost,
                              o->h.stream));
  PL_CHECK_HIP(hipStreamSynchronize(o->h.stream));
  for (int b = 0; b < o->h.B; ++b) {
    pl_stats& s = stats[b];
    memset(&s, 0, sizeof(s));
    s.status = info[b].status;
    s.admm_iters = info[b].iter;
    s.ls_accepted = info[b].ls_accepted;
    s.ls_branch = info[b].ls_branch;
    s.ls_trials = info[b].ls_trials;
    s.ls_alpha = info[b].ls_alpha;
    s.viol_max = info[b].viol_max;
    s.pri_res = info[b].pri_res;
    s.dua_res = info[b].dua_res;
    s.f = info[b].f;
  }
  return 0;
}

// SQP iterations per solve.  The reference runs one (`for _ in range(1)` with a TODO,
// optimization/ocp.py:382-383); k > 1 repeats eval -> osqp.update -> warm-started
// osqp.solve -> line search from the accepted point.  Phase times are those of the
// last iteration.
extern "C" int pl_ocp_set_admm_kernel(pl_ocp* o, int kind) {
  REQUIRE_DEVICE(o);
  if (kind < PL_ADMM_AUTO || kind > PL_ADMM_CHAIN) { pl_set_error("ADMM kernel %d unknown", kind); return -1; }
  PL_CHECK_HIP(hipStreamSynchronize(o->h.stream));
  return admm_select(o, kind);
}

extern "C" int pl_ocp_get_admm_kernel(const pl_ocp* o) {
  if (!o) { pl_set_error("null handle"); return -1; }
  return o->h.admm_rc ? PL_ADMM_CHAIN : (o->h.admm_waves == 2 ? PL_ADMM_SWEEP2 : PL_ADMM_SWEEP);
}

extern "C" int pl_ocp_set_sqp_iters(pl_ocp* o, int sqp_iters) {
  if (!o) { pl_set_error("null handle"); return -1; }
  if (sqp_iters < 1 || sqp_iters > 1000) { pl_set_error("sqp_iters %d outside [1, 1000]", sqp_iters); return -1; }
  o->h.sqp_iters = sqp_iters;
  return 0;
}

// Solver selection (ocp.py:248 / :265 dispatch on the solver string).  The interior
// point's per-problem state (slacks and multipliers, 7 x m doubles per problem) is
// allocated on first selection.
// ---- structurally non-zero pairs of the Lagrangian Hessian blocks (k_lag_hess work list)
// Probed once on the host with the same hyper-dual row code (rows.h) at a generic point:
// random x, parameters and multipliers, contact c = 0.5 so that stance and swing rows are
// both active.  A column pair whose contracted second derivative is exactly 0 there is
// identically 0 (RNEA is linear in a and f, the velocity rows in v, the integration rows in
// everything, the base position never enters): about half of the pairs of a whole-body node.
namespace {
struct HostHessEmit {
  const double* lam;
  double acc;
  int r;
  void operator()(const HDual& v, double, double) {
    acc += lam[r] * v.c;
    ++r;
  }
};

template <int DYN>
void probe_hess(const PlModel& M, const PlOcpConst& O, int i, const double* p, const double* xw, int nw,
                const double* lam, std::vector<uint8_t>& nz) {
  std::vector<HDual> kst(PL_KIN_STORE);
  const int ndx = O.ndx;
  nz.assign((size_t)nw * (nw + 1) / 2, 0);
  for (int k = 0; k < nw; ++k)
    for (int j = 0; j <= k; ++j) {
      pl::VecIn<HDual> dx{xw, nullptr, 0.0, j, k};
      pl::VecIn<HDual> u{xw + ndx, nullptr, 0.0, j - ndx, k - ndx};
      pl::VecIn<HDual> dxn{xw + nw, nullptr, 0.0, j - nw, k - nw};
      HostHessEmit e{lam, 0.0, 0};
      pl::node_rows<HDual, DYN>(M, O, i, p, dx, u, dxn, e, kst.data(), 1);
      nz[(size_t)k * (k + 1) / 2 + j] = e.acc != 0.0;
    }
}

void hess_pattern(const PlOcpHandle& h, const std::vector<PlNode>& nodes, int i, std::vector<uint8_t>& nz) {
  const PlOcpConst& O = h.oc;
  uint64_t st = 0x9e3779b97f4a7c15ull ^ (uint64_t)(i + 1);
  auto rnd = [&]() {  // uniform in (0.5, 1.5)
    st = st * 6364136223846793005ull + 1442695040888963407ull;
    return 0.5 + (double)(st >> 11) / 9007199254740992.0;
  };
  std::vector<double> p(O.P.np);
  for (double& v : p) v = rnd();
  p[O.P.dt_min] = 0.02;
  p[O.P.dt_max] = 0.05;
  for (int k = 0; k < 4 * O.N; ++k) {
    p[O.P.contact + k] = 0.5;
    p[O.P.swing + k] = 0.3;
  }
  p[O.P.n_contacts] = 2.0;
  p[O.P.swing_period] = 0.4;
  p[O.P.swing_vel_limits + 1] = -0.2;
  const int qo = PL_IS_CV(O.dyn) ? 9 : 3;  // quaternion of x_init
  double qn = 0.0;
  for (int k = 0; k < 4; ++k) qn += p[O.P.x_init + qo + k] * p[O.P.x_init + qo + k];
  for (int k = 0; k < 4; ++k) p[O.P.x_init + qo + k] /= sqrt(qn);
  const int nw = nodes[i].nw;
  std::vector<double> xw(nw + O.ndx), lam(nodes[i].nrow);
  for (double& v : xw) v = 0.2 * (rnd() - 1.0);
  for (size_t r = 0; r < lam.size(); ++r) lam[r] = (r & 1) ? rnd() : -rnd();
  const PlModel& M = h.model;
  switch (O.dyn) {
    case PL_DYN_RNEA: probe_hess<PL_DYN_RNEA>(M, O, i, p.data(), xw.data(), nw, lam.data(), nz); break;
    case PL_DYN_ACC: probe_hess<PL_DYN_ACC>(M, O, i, p.data(), xw.data(), nw, lam.data(), nz); break;
    case PL_DYN_CV: probe_hess<PL_DYN_CV>(M, O, i, p.data(), xw.data(), nw, lam.data(), nz); break;
    case PL_DYN_CA: probe_hess<PL_DYN_CA>(M, O, i, p.data(), xw.data(), nw, lam.data(), nz); break;
    case PL_DYN_ACCNB: probe_hess<PL_DYN_ACCNB>(M, O, i, p.data(), xw.data(), nw, lam.data(), nz); break;
    case PL_DYN_CVNB: probe_hess<PL_DYN_CVNB>(M, O, i, p.data(), xw.data(), nw, lam.data(), nz); break;
    default: probe_hess<PL_DYN_ABA>(M, O, i, p.data(), xw.data(), nw, lam.data(), nz); break;
  }
}
}  // namespace

extern "C" int pl_ocp_set_solver(pl_ocp* o, int solver) {
  REQUIRE_DEVICE(o);
  if (solver != PL_SOLVER_OSQP && solver != PL_SOLVER_IP) {
    pl_set_error("Solver %d not supported (PL_SOLVER_OSQP = 0, PL_SOLVER_IP = 1)", solver);
    return -1;
  }
  PlOcpHandle* h = &o->h;
  if (solver == PL_SOLVER_IP && h->oc.dyn == PL_DYN_RNEAFD) {
    // the reference keeps the accelerations in u for its Fatrop branch ("necessary for Fatrop
    // solver", ocp_whole_body_rnea.py:21); the Lagrangian Hessian here is block diagonal over w_i
    pl_set_error("the interior-point solver needs include_acc=True (ocp_whole_body_rnea.py:21)");
    return -1;
  }
  if (solver == PL_SOLVER_IP && !h->d.ipinfo) {
    const size_t Bm = (size_t)h->B * h->m;
    if (dalloc(o, &h->d.ip_s, Bm) || dalloc(o, &h->d.ip_lam, Bm) || dalloc(o, &h->d.ip_lam0, Bm) ||
        dalloc(o, &h->d.ip_zl, Bm) ||
        dalloc(o, &h->d.ip_zu, Bm) || dalloc(o, &h->d.ip_rh, Bm) || dalloc(o, &h->d.ip_dl, Bm) ||
        dalloc(o, &h->d.ip_ds, Bm) || dalloc(o, &h->d.ip_jdx, Bm) || dalloc(o, &h->d.ip_dx, (size_t)h->B * h->n) ||
        dalloc(o, &h->d.ipinfo, (size_t)h->B) || dalloc(o, &h->d.ip_dwi, (size_t)2 * h->B) ||
        dalloc(o, &h->d.ip_iflag, (size_t)4 * h->B))
      return -2;
    // Lagrangian Hessian work list (k_hess.hip): the structurally non-zero column pairs
    // j <= k of every w_i block (hess_pattern, one probe per node type); node blocks packed
    // lower, the pairs not listed stay 0
    std::vector<int2> hl;
    std::vector<int> hoff;
    long long off = 0;
    const PlOcpConst& O = h->oc;
    std::vector<uint8_t> pat[3];
    for (int i = 0; i <= h->N; ++i) {
      const int nw = o->nodes[i].nw;
      hoff.push_back((int)off);
      off += (long long)nw * (nw + 1) / 2;
      if (i == h->N) break;  // no rows on the last node
      const int type = pl::node_type(O, i);
      if (pat[type].empty()) hess_pattern(*h, o->nodes, i, pat[type]);
      for (int k = 0; k < nw; ++k)
        for (int j = 0; j <= k; ++j)
          if (pat[type][(size_t)k * (k + 1) / 2 + j]) hl.push_back(make_int2(i, j | (k << 16)));
    }
    h->hl_len = (int)hl.size();
    h->hl_stride = (off + 1) & ~1LL;
    if (upload(o, &h->d.hlist, hl) || upload(o, &h->d.hoff, hoff) ||
        dalloc(o, &h->d.Hlag, (size_t)h->B * h->hl_stride))
      return -2;
  }
  h->solver = solver;
  return 0;
}

extern "C" int pl_ocp_set_ip_settings(pl_ocp* o, const pl_ip_settings* s) {
  if (!o || !s) { pl_set_error("null argument"); return -1; }
  if (s->max_iter < 0 || s->max_iter > PL_IP_MAXFILT) {
    pl_set_error("ip max_iter %d outside [0, %d]", s->max_iter, PL_IP_MAXFILT);
    return -1;
  }
  if (s->ls_max < 1 || s->ls_max > 60 || !(s->tol > 0) || !(s->mu_init > 0) || !(s->bound_push > 0) ||
      !(s->bound_frac > 0) || !(s->delta_w >= 0) || !(s->delta_c > 0) || s->n_refine < 0 || s->n_refine > 8) {
    pl_set_error("invalid interior-point settings");
    return -1;
  }
  if (s->hessian != PL_IP_HESS_EXACT && s->hessian != PL_IP_HESS_GN) {
    pl_set_error("ip hessian %d unknown (PL_IP_HESS_EXACT = 0, PL_IP_HESS_GN = 1)", s->hessian);
    return -1;
  }
  o->h.ip = PlIpSettings{s->tol, s->mu_init, s->bound_push, s->bound_frac, s->delta_w, s->delta_c, s->max_iter,
                         s->ls_max, s->n_refine, 0, 1e-7};
  o->h.ip_hess = s->hessian;
  return 0;
}

// lam_g warm start of the interior-point branch (opti.set_initial(opti.lam_g, lam_g),
// ocp_whole_body_rnea.py:234-235 and the other OCPs' warm_start): lam = NULL returns to the
// cold start (lam = 0).  Kept until changed, like an Opti initial value.
extern "C" int pl_ocp_set_lam(pl_ocp* o, const double* lam) {
  REQUIRE_DEVICE(o);
  PlOcpHandle* h = &o->h;
  if (!h->d.ip_lam0) { pl_set_error("no interior-point state (pl_ocp_set_solver(o, PL_SOLVER_IP) first)"); return -1; }
  if (!lam) {
    h->ip_lam_warm = 0;
    return 0;
  }
  PL_CHECK_HIP(hipMemcpyAsync(h->d.ip_lam0, lam, (size_t)h->B * h->m * 8, hipMemcpyHostToDevice, h->stream));
  PL_CHECK_HIP(hipStreamSynchronize(h->stream));
  h->ip_lam_warm = 1;
  return 0;
}

extern "C" int pl_ocp_get_lam(pl_ocp* o, double* lam) {
  REQUIRE_DEVICE(o);
  PlOcpHandle* h = &o->h;
  if (!h->d.ip_lam) { pl_set_error("no interior-point state (pl_ocp_set_solver(o, PL_SOLVER_IP) first)"); return -1; }
  PL_CHECK_HIP(hipMemcpyAsync(lam, h->d.ip_lam, (size_t)h->B * h->m * 8, hipMemcpyDeviceToHost, h->stream));
  PL_CHECK_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

extern "C" int pl_ocp_ip_stats(pl_ocp* o, pl_ip_stats* out) {
  REQUIRE_DEVICE(o);
  PlOcpHandle* h = &o->h;
  if (!h->d.ipinfo) { pl_set_error("no interior-point state (pl_ocp_set_solver(o, PL_SOLVER_IP) first)"); return -1; }
  std::vector<PlIpInfo> info(h->B);
  PL_CHECK_HIP(hipMemcpyAsync(info.data(), h->d.ipinfo, h->B * sizeof(PlIpInfo), hipMemcpyDeviceToHost, h->stream));
  PL_CHECK_HIP(hipStreamSynchronize(h->stream));
  for (int b = 0; b < h->B; ++b) {
    pl_ip_stats& s = out[b];
    memset(&s, 0, sizeof(s));
    s.status = info[b].status;
    s.iter = info[b].iter;
    s.ls_trials = info[b].trials;
    s.nfilter = info[b].nfilt;
    s.err = info[b].err;
    s.mu = info[b].mu;
    s.alpha = info[b].alpha;
    s.alpha_z = info[b].alpha_z;
    s.f = info[b].f;
    s.viol_max = info[b].viol_max;
    for (int q = 0; q < PL_IP_MAXFILT; ++q) s.alphas[q] = info[b].alphas[q];
  }
  return 0;
}

extern "C" int pl_debug_ip_direction(pl_ocp* o, const double* S, const double* LAM, const double* ZL,
                                     const double* ZU, const double* MU) {
  REQUIRE_DEVICE(o);
  PlOcpHandle* h = &o->h;
  if (!h->d.ipinfo) { pl_set_error("no interior-point state (pl_ocp_set_solver(o, PL_SOLVER_IP) first)"); return -1; }
  const size_t Bm = (size_t)h->B * h->m * 8;
  PL_CHECK_HIP(hipMemcpyAsync(h->d.ip_s, S, Bm, hipMemcpyHostToDevice, h->stream));
  PL_CHECK_HIP(hipMemcpyAsync(h->d.ip_lam, LAM, Bm, hipMemcpyHostToDevice, h->stream));
  PL_CHECK_HIP(hipMemcpyAsync(h->d.ip_zl, ZL, Bm, hipMemcpyHostToDevice, h->stream));
  PL_CHECK_HIP(hipMemcpyAsync(h->d.ip_zu, ZU, Bm, hipMemcpyHostToDevice, h->stream));
  std::vector<PlIpInfo> info(h->B);
  for (int b = 0; b < h->B; ++b) {
    memset(&info[b], 0, sizeof(PlIpInfo));
    info[b].mu = MU[b];
    info[b].active = 1;
  }
  PL_CHECK_HIP(hipMemcpyAsync(h->d.ipinfo, info.data(), h->B * sizeof(PlIpInfo), hipMemcpyHostToDevice, h->stream));
  launch_reset_info(h);
  enqueue_ip_direction(h);
  PL_CHECK_HIP(hipGetLastError());
  PL_CHECK_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

extern "C" int pl_ocp_solve(pl_ocp* o, pl_stats* stats, double* phase_ms) {
  REQUIRE_DEVICE(o);
  if (o->h.solver == PL_SOLVER_IP) {
    enqueue_ip(&o->h);
    PL_CHECK_HIP(hipGetLastError());
    PL_CHECK_HIP(hipStreamSynchronize(o->h.stream));
    if (phase_ms)
      for (int k = 0; k < 4; ++k) phase_ms[k] = 0.0;
    return fetch_stats(o, stats);
  }
  for (int k = 0; k < o->h.sqp_iters; ++k) enqueue_solve(o, phase_ms != nullptr);
  PL_CHECK_HIP(hipGetLastError());
  PL_CHECK_HIP(hipStreamSynchronize(o->h.stream));
  if (phase_ms) {
    for (int k = 0; k < 4; ++k) {
      float ms = 0.f;
      hipEventElapsedTime(&ms, o->ev[k], o->ev[k + 1]);
      phase_ms[k] = ms;
    }
  }
  return fetch_stats(o, stats);
}

extern "C" int pl_eval_sqp_data(pl_ocp* o, double* grad, double* Jvals, double* g, double* lbg, double* ubg) {
  REQUIRE_DEVICE(o);
  PlOcpHandle* h = &o->h;
  launch_eval_values(h, h->d.x);
  launch_eval_jac(h);
  launch_objective(h);
  PL_CHECK_HIP(hipGetLastError());
  const size_t B = h->B;
  if (grad) PL_CHECK_HIP(hipMemcpyAsync(grad, h->d.grad, B * h->n * 8, hipMemcpyDeviceToHost, h->stream));
  if (Jvals) PL_CHECK_HIP(hipMemcpyAsync(Jvals, h->d.Araw, B * h->nnz * 8, hipMemcpyDeviceToHost, h->stream));
  if (g) PL_CHECK_HIP(hipMemcpyAsync(g, h->d.g, B * h->m * 8, hipMemcpyDeviceToHost, h->stream));
  if (lbg) PL_CHECK_HIP(hipMemcpyAsync(lbg, h->d.lbg, B * h->m * 8, hipMemcpyDeviceToHost, h->stream));
  if (ubg) PL_CHECK_HIP(hipMemcpyAsync(ubg, h->d.ubg, B * h->m * 8, hipMemcpyDeviceToHost, h->stream));
  PL_CHECK_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

extern "C" int pl_eval_f(pl_ocp* o, double* f) {
  REQUIRE_DEVICE(o);
  PlOcpHandle* h = &o->h;
  launch_objective(h);
  std::vector<double> w((size_t)h->B * 8);
  PL_CHECK_HIP(hipMemcpyAsync(w.data(), h->d.work, w.size() * 8, hipMemcpyDeviceToHost, h->stream));
  PL_CHECK_HIP(hipStreamSynchronize(h->stream));
  for (int b = 0; b < h->B; ++b) f[b] = w[(size_t)b * 8];
  return 0;
}

extern "C" int pl_mpc_setup(pl_ocp* o, const double* x_state, const double* t0) {
  REQUIRE_DEVICE(o);
  PlOcpHandle* h = &o->h;
  PL_CHECK_HIP(hipMemcpyAsync(h->d.xstate, x_state, (size_t)h->B * h->nx * 8, hipMemcpyHostToDevice, h->stream));
  PL_CHECK_HIP(hipMemcpyAsync(h->d.t0, t0, (size_t)h->B * 8, hipMemcpyHostToDevice, h->stream));
  PL_CHECK_HIP(hipStreamSynchronize(h->stream));
  h->ip_lam_warm = 0;  // the loop's first solve has no lam_g yet (ocp.py:198)
  return 0;
}

// The OSQP-SQP part of an MPC step (every launch after k_mpc_prepare) as one HIP graph.
// The sequence is fixed by the handle's host state (sizes, settings, kernel choice,
// device pointers): it is captured on the second step that sees the same bytes of `h`
// (the first runs eagerly, so every one-time kernel attribute is set outside a capture)
// and replayed while they stay the same; any change (a setter, another kernel choice)
// runs eagerly once and re-captures.  Per-call data lives in device memory, so a replay
// is the eager sequence.  Profiling runs (per-launch events) and PL_MPC_GRAPH=0 stay eager.
static void enqueue_mpc_sqp(pl_ocp* o) {
  for (int it = 0; it < o->h.sqp_iters; ++it) enqueue_solve(o, false);
  launch_mpc_finish(&o->h);
}

static int mpc_sqp_graph(pl_ocp* o) {
  PlOcpHandle* h = &o->h;
  const unsigned char* hb = reinterpret_cast<const unsigned char*>(h);
  const bool same = o->mpc_key.size() == sizeof(PlOcpHandle) && !memcmp(o->mpc_key.data(), hb, sizeof(PlOcpHandle));
  if (same && o->mpc_graph) return hipGraphLaunch(o->mpc_graph, h->stream) == hipSuccess ? 0 : -1;
  if (o->mpc_graph) {
    hipGraphExecDestroy(o->mpc_graph);
    o->mpc_graph = nullptr;
  }
  if (!same) {  // first sighting of this state: eager, remember it
    o->mpc_key.assign(hb, hb + sizeof(PlOcpHandle));
    enqueue_mpc_sqp(o);
    return 0;
  }
  hipGraph_t g = nullptr;
  if (hipStreamBeginCapture(h->stream, hipStreamCaptureModeThreadLocal) != hipSuccess) return -1;
  enqueue_mpc_sqp(o);
  const hipError_t ec = hipStreamEndCapture(h->stream, &g);
  if (ec != hipSuccess || !g) {
    (void)hipGetLastError();
    if (g) hipGraphDestroy(g);
    return -1;
  }
  const hipError_t ei = hipGraphInstantiate(&o->mpc_graph, g, nullptr, nullptr, 0);
  hipGraphDestroy(g);
  if (ei != hipSuccess) {
    o->mpc_graph = nullptr;
    return -1;
  }
  ++o->mpc_captures;
  return hipGraphLaunch(o->mpc_graph, h->stream) == hipSuccess ? 0 : -1;
}

extern "C" int pl_mpc_step(pl_ocp* o, int k) {
  REQUIRE_DEVICE(o);
  if (o->h.profile && o->h.prof_n > 48) prof_collect(&o->h);
  launch_mpc_prepare(&o->h, k);
  if (o->h.solver != PL_SOLVER_IP && !o->h.profile && !o->mpc_graph_off) {
    if (mpc_sqp_graph(o)) {
      // capture or replay refused: nothing of the step ran; from now on launch eagerly
      (void)hipGetLastError();
      o->mpc_graph_off = 1;
      enqueue_mpc_sqp(o);
    }
    PL_CHECK_HIP(hipGetLastError());
    return 0;
  }
  if (o->h.solver == PL_SOLVER_IP) {
    enqueue_ip(&o->h);
    // warm_start() of the next step passes this solve's lam_g back (ocp.py:373, ocp_*.py warm_start)
    PlOcpHandle* h = &o->h;
    PL_CHECK_HIP(hipMemcpyAsync(h->d.ip_lam0, h->d.ip_lam, (size_t)h->B * h->m * 8, hipMemcpyDeviceToDevice, h->stream));
    h->ip_lam_warm = 1;
    launch_mpc_finish(&o->h);
  } else
    enqueue_mpc_sqp(o);
  PL_CHECK_HIP(hipGetLastError());
  return 0;
}

extern "C" int pl_mpc_get_state(pl_ocp* o, double* x_state) {
  REQUIRE_DEVICE(o);
  PlOcpHandle* h = &o->h;
  PL_CHECK_HIP(hipMemcpyAsync(x_state, h->d.xstate, (size_t)h->B * h->nx * 8, hipMemcpyDeviceToHost, h->stream));
  PL_CHECK_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

extern "C" int pl_mpc_get_stats(pl_ocp* o, pl_stats* stats) {
  REQUIRE_DEVICE(o);
  return fetch_stats(o, stats);
}

extern "C" int pl_mpc_export(pl_ocp* o, void* device_dst) {
  REQUIRE_DEVICE(o);
  PlOcpHandle* h = &o->h;
  const int nu0 = o->nodes[0].nu;
  const size_t row = (size_t)nu0 + h->nx;
  char* dst = (char*)device_dst;
  // two strided copies on the handle's stream: u_0 of every problem, then x_state
  PL_CHECK_HIP(hipMemcpy2DAsync(dst, row * 8, h->d.x + h->ndx, (size_t)h->n * 8, (size_t)nu0 * 8, h->B,
                                hipMemcpyDeviceToDevice, h->stream));
  PL_CHECK_HIP(hipMemcpy2DAsync(dst + (size_t)nu0 * 8, row * 8, h->d.xstate, (size_t)h->nx * 8, (size_t)h->nx * 8,
                                h->B, hipMemcpyDeviceToDevice, h->stream));
  PL_CHECK_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

static void prof_collect(PlOcpHandle* h) {
  if (!h->profile || h->prof_n == 0) return;
  hipStreamSynchronize(h->stream);
  for (int k = 0; k < h->prof_n; ++k) {
    float ms = 0.f;
    hipEventElapsedTime(&ms, h->prof_ev[k][0], h->prof_ev[k][1]);
    h->prof_admm_ms += ms;
    h->prof_admm_launches++;
  }
  h->prof_n = 0;
}

extern "C" int pl_ocp_sync(pl_ocp* o) {
  REQUIRE_DEVICE(o);
  PL_CHECK_HIP(hipStreamSynchronize(o->h.stream));
  prof_collect(&o->h);
  return 0;
}

// Per-launch timing of the dominant kernel (k_admm) with HIP events recorded on
// the handle's stream around every launch.  enable=1 starts (and clears),
// enable=0 stops.  out: [total_ms, launches, problem_iterations].
extern "C" int pl_ocp_profile(pl_ocp* o, int enable) {
  REQUIRE_DEVICE(o);
  PlOcpHandle* h = &o->h;
  prof_collect(h);
  if (enable && !h->profile) {
    for (int k = 0; k < 64; ++k) {
      hipEventCreate(&h->prof_ev[k][0]);
      hipEventCreate(&h->prof_ev[k][1]);
    }
  }
  h->profile = enable;
  h->prof_n = 0;
  h->prof_admm_ms = 0.0;
  h->prof_admm_launches = 0;
  h->prof_admm_iters = 0;
  if (enable) {
    launch_reset_prof(h);
    PL_CHECK_HIP(hipStreamSynchronize(h->stream));
  }
  return 0;
}

extern "C" int pl_ocp_profile_read(pl_ocp* o, double* out) {
  REQUIRE_DEVICE(o);
  PlOcpHandle* h = &o->h;
  prof_collect(h);
  // problem-iterations the ADMM launches actually executed: per-problem counters
  // (terminated problems skip later launches, so B * niter would over-count)
  std::vector<PlProbInfo> info(h->B);
  PL_CHECK_HIP(hipMemcpyAsync(info.data(), h->d.info, h->B * sizeof(PlProbInfo), hipMemcpyDeviceToHost, h->stream));
  PL_CHECK_HIP(hipStreamSynchronize(h->stream));
  long long it = 0;
  for (int b = 0; b < h->B; ++b) it += info[b].iter_prof;
  h->prof_admm_iters = it;
  out[0] = h->prof_admm_ms;
  out[1] = (double)h->prof_admm_launches;
  out[2] = (double)h->prof_admm_iters;
  return 0;
}

int admm_lds_bytes(const PlOcpHandle* h);
int admm_ppw(const PlOcpHandle* h);
int admm_asb_cap(const PlOcpHandle* h);

// Sizes: [n, m, nnz, S_stride (doubles), nw_max, N, ADMM programs (u16, LDS-resident),
// problems per ADMM workgroup, ADMM LDS bytes per workgroup, A values per lane / 64,
// A values per problem staged in LDS by the one-wave sweep, largest node's A count].
extern "C" int pl_ocp_sizes(const pl_ocp* o, long long* out) {
  if (!o) { pl_set_error("null handle"); return -1; }
  out[0] = o->h.n; out[1] = o->h.m; out[2] = o->h.nnz; out[3] = o->h.S_stride; out[4] = o->h.nw_max; out[5] = o->h.N;
  out[6] = (long long)o->aprog.size(); out[7] = admm_ppw(&o->h); out[8] = admm_lds_bytes(&o->h); out[9] = o->h.admm_asr;
  out[10] = admm_asb_cap(&o->h); out[11] = o->h.nent_max;
  return 0;
}

// Debug / parity access to internal per-problem arrays (tests only).
static int debug_rw(pl_ocp* o, const char* name, double* out, const double* in, long long count) {
  PlOcpHandle* h = &o->h;
  const size_t B = h->B;
  struct Item { const char* n; double* p; size_t len; } items[] = {
      {"Hlag", h->d.Hlag, h->d.Hlag ? B * (size_t)h->hl_stride : 0},
      {"ip_dwi", h->d.ip_dwi, h->d.ip_dwi ? 2 * B : 0},
      {"As", h->d.As, B * h->nnz}, {"Araw", h->d.Araw, B * h->nnz}, {"qs", h->d.qs, B * h->n},
      {"ls", h->d.ls, B * h->m},   {"us", h->d.us, B * h->m},       {"rho", h->d.rho, B * h->m},
      {"D", h->d.D, B * h->n},     {"E", h->d.E, B * h->m},         {"cs", h->d.cs, B},
      {"admm_t", h->d.dbg, h->d.dbg ? B * 32 : 0}, {"Ps", h->d.Ps, B * h->n},   {"P", h->d.P, B * h->n},         {"xa", h->d.xa, B * h->n},
      {"za", h->d.za, B * h->m},   {"ya", h->d.ya, B * h->m},       {"S", h->d.S, B * (size_t)h->S_stride},
      {"rhs", h->d.rhs, B * h->n}, {"step", h->d.step, B * h->n},   {"grad", h->d.grad, B * h->n},
      {"g", h->d.g, B * h->m},     {"xstate", h->d.xstate, B * h->nx},
      {"ip_s", h->d.ip_s, h->d.ip_s ? B * h->m : 0},     {"ip_lam", h->d.ip_lam, h->d.ip_lam ? B * h->m : 0},
      {"ip_lam0", h->d.ip_lam0, h->d.ip_lam0 ? B * h->m : 0},
      {"ip_zl", h->d.ip_zl, h->d.ip_zl ? B * h->m : 0},  {"ip_zu", h->d.ip_zu, h->d.ip_zu ? B * h->m : 0},
      {"ip_rh", h->d.ip_rh, h->d.ip_rh ? B * h->m : 0},  {"ip_dl", h->d.ip_dl, h->d.ip_dl ? B * h->m : 0},
      {"ip_ds", h->d.ip_ds, h->d.ip_ds ? B * h->m : 0},  {"ip_dx", h->d.ip_dx, h->d.ip_dx ? B * h->n : 0},
      {"ip_jdx", h->d.ip_jdx, h->d.ip_jdx ? B * h->m : 0}};
  for (auto& it : items) {
    if (strcmp(it.n, name) == 0) {
      if ((size_t)count < it.len) { pl_set_error("buffer too small for %s (%zu)", name, it.len); return -1; }
      if (out) PL_CHECK_HIP(hipMemcpyAsync(out, it.p, it.len * 8, hipMemcpyDeviceToHost, h->stream));
      else PL_CHECK_HIP(hipMemcpyAsync(it.p, in, it.len * 8, hipMemcpyHostToDevice, h->stream));
      PL_CHECK_HIP(hipStreamSynchronize(h->stream));
      return (int)0;
    }
  }
  pl_set_error("unknown array %s", name);
  return -1;
}

extern "C" int pl_debug_get(pl_ocp* o, const char* name, double* out, long long count) {
  REQUIRE_DEVICE(o);
  if (!out) { pl_set_error("null argument"); return -1; }
  return debug_rw(o, name, out, nullptr, count);
}

// Overwrite an internal array (tests: e.g. "ip_dwi", the inertia state of a teacher-forced
// interior-point direction).
extern "C" int pl_debug_set(pl_ocp* o, const char* name, const double* in, long long count) {
  REQUIRE_DEVICE(o);
  if (!in) { pl_set_error("null argument"); return -1; }
  return debug_rw(o, name, nullptr, in, count);
}

// Node table (tests): per node [nw, nu, x_off, row_off, nrow, ncol, ent_off, nent, ntile, nunit, s_off, ncpl]
extern "C" int pl_debug_nodes(const pl_ocp* o, int* out) {
  for (size_t i = 0; i < o->nodes.size(); ++i) {
    const PlNode& nd = o->nodes[i];
    int* r = out + 12 * i;
    r[0] = nd.nw; r[1] = nd.nu; r[2] = nd.x_off; r[3] = nd.row_off; r[4] = nd.nrow; r[5] = nd.ncol;
    r[6] = nd.ent_off; r[7] = nd.nent; r[8] = nd.ntile; r[9] = nd.nunit; r[10] = nd.s_off; r[11] = nd.ncpl;
  }
  return 0;
}

// Host entry points of the Lie-group state maps (DynamicsWholeBodyTorque.state_integrate /
// state_difference, dynamics_whole_body_torque.py:11-40), same code as the kernels.
extern "C" int pl_state_integrate(const pl_model* model, const double* x, const double* dx, double* out) {
  if (!model || !x || !dx || !out) { pl_set_error("null argument"); return -1; }
  const PlModel& M = model->m;
  pl::VecIn<double> acc{dx, nullptr, 0.0, -1};
  double q[PL_MAXQ];
  pl::integrate_q<double>(M, x, acc, q);
  for (int k = 0; k < M.nq; ++k) out[k] = q[k];
  for (int k = 0; k < M.nv; ++k) out[M.nq + k] = x[M.nq + k] + dx[M.nv + k];
  return 0;
}

extern "C" int pl_state_difference(const pl_model* model, const double* x0, const double* x1, double* dx) {
  if (!model || !x0 || !x1 || !dx) { pl_set_error("null argument"); return -1; }
  const PlModel& M = model->m;
  pl::difference_q(M, x0, x1, dx);
  for (int k = 0; k < M.nv; ++k) dx[M.nv + k] = x1[M.nq + k] - x0[M.nq + k];
  return 0;
}

// Raw copies of the host-built descriptors (tests: host build of the device math).
extern "C" int pl_debug_consts(const pl_ocp* o, void* model_out, void* oc_out, int* sizes) {
  if (!o) { pl_set_error("null handle"); return -1; }
  if (sizes) { sizes[0] = (int)sizeof(PlModel); sizes[1] = (int)sizeof(PlOcpConst); }
  if (model_out) memcpy(model_out, &o->h.model, sizeof(PlModel));
  if (oc_out) memcpy(oc_out, &o->h.oc, sizeof(PlOcpConst));
  return 0;
}

// Tests: evaluate + scale + factor, then exactly `niter` ADMM iterations from the
// current iterates (no termination checks, no line search).
extern "C" int pl_debug_admm(pl_ocp* o, int niter, int reset) {
  REQUIRE_DEVICE(o);
  PlOcpHandle* h = &o->h;
  launch_eval_values(h, h->d.x);
  launch_eval_jac(h);
  launch_objective(h);
  launch_qp_setup(h);
  launch_factor(h);
  launch_reset_info(h);
  if (reset) launch_reset_iterates(h);
  launch_admm_init(h);
  if (niter > 0) launch_admm(h, niter, 0, 0);
  PL_CHECK_HIP(hipGetLastError());
  PL_CHECK_HIP(hipStreamSynchronize(h->stream));
  return 0;
}

// ---------------------------------------------------------------------------
// CasADi external-function ABI.  The reference builds
//   sqp_data(x, p) -> (grad_f, J_g, g, lbg, ubg), f_data(x, p) -> (f, grad_f),
//   g_data(x, p) -> (g, lbg, ubg), hess_data(x, p) -> hess_f   (optimization/ocp.py:287-290)
//   retract_solution(sol_x, x_init) -> (q, v, a, forces, tau)   (ocp_whole_body_rnea.py:326-366)
// and loads generated code with ca.external(NAME, lib) (ocp.py:299-302, run_mpc.py:53).
// These symbols give an unmodified ca.external consumer the same functions from this
// library: shapes and sparsity come from the OCP bound with pl_casadi_bind (same process:
// ca.external dlopens the already-loaded library).  Evaluations run on the bound handle's
// device (problem slot 0); J_g is returned in CasADi's compressed-column order.
// Every entry point takes one process-wide lock (CasADi may evaluate from several
// threads, e.g. a threaded map; the bound handle has one stream and one staging
// buffer), and each evaluation waits on its stream once, after all its copies.
namespace {
typedef long long casadi_int;
struct CasadiState {
  pl_ocp* o = nullptr;
  int steps = 3;
  std::vector<casadi_int> sp_x, sp_p, sp_n1, sp_J, sp_m1, sp_11, sp_H, sp_xinit, sp_q, sp_v, sp_a, sp_f, sp_tau;
  std::vector<int> J_perm;  // CCS position -> library entry
  std::vector<double> buf;
};
CasadiState g_cas;
std::mutex g_cas_mu;
#define PL_CAS_LOCK std::lock_guard<std::mutex> cas_lock_(g_cas_mu)

std::vector<casadi_int> dense_sp(int nrow, int ncol) {
  std::vector<casadi_int> s{nrow, ncol};
  for (int c = 0; c <= ncol; ++c) s.push_back((casadi_int)c * nrow);
  for (int c = 0; c < ncol; ++c)
    for (int r = 0; r < nrow; ++r) s.push_back(r);
  return s;
}

int cas_ready() {
  if (!g_cas.o) {
    pl_set_error("no OCP bound (pl_casadi_bind)");
    return 0;
  }
  return 1;
}

// retract_solution outputs of the bound OCP: inputs ahead of the forces (na), forces
// (nf), joint torques (nt: u's tau block for rnea, RNEA / u's tau_j for the others)
void cas_u_split(const pl_ocp* o, int& na, int& nf, int& nt) {
  const PlOcpConst& O = o->h.oc;
  if (PL_IS_RNEA(O.dyn)) { na = O.na; nf = O.nf; nt = O.nj; }
  else if (O.dyn == PL_DYN_ACC || O.dyn == PL_DYN_CA || O.dyn == PL_DYN_ACCNB) { na = O.na; nf = O.nf; nt = O.nj; }
  else if (O.dyn == PL_DYN_CV) { na = O.nv; nf = O.nf; nt = O.nj; }
  else if (O.dyn == PL_DYN_CVNB) { na = O.nj; nf = O.nf; nt = O.nj; }
  else { na = 0; nf = O.nf; nt = O.nj; }
}

int cas_eval(const double** arg, bool jac) {
  pl_ocp* o = g_cas.o;
  PlOcpHandle* h = &o->h;
  if (!o->on_device) { pl_set_error("bound OCP has no device"); return 1; }
  (void)hipSetDevice(h->device);
  (void)hipGetLastError();
  if (!arg[0] || !arg[1]) { pl_set_error("sqp/f/g_data: null input"); return 1; }
  if (hipMemcpyAsync(h->d.x, arg[0], h->n * 8, hipMemcpyHostToDevice, h->stream) != hipSuccess ||
      hipMemcpyAsync(h->d.p, arg[1], h->np * 8, hipMemcpyHostToDevice, h->stream) != hipSuccess)
    return 1;
  memcpy(o->h_params.data(), arg[1], h->np * 8);
  launch_eval_values(h, h->d.x);
  if (jac) launch_eval_jac(h);
  launch_objective(h);
  return hipGetLastError() != hipSuccess;
}

// enqueue one device -> host copy of an output (null outputs are skipped)
int cas_get(const double* dev, size_t count, double* host) {
  if (!host) return 0;
  PlOcpHandle* h = &g_cas.o->h;
  return hipMemcpyAsync(host, dev, count * 8, hipMemcpyDeviceToHost, h->stream) != hipSuccess;
}

int cas_wait() { return hipStreamSynchronize(g_cas.o->h.stream) != hipSuccess; }
}  // namespace

extern "C" int pl_casadi_bind(pl_ocp* o, int retract_steps) {
  if (!o) { pl_set_error("null handle"); return -1; }
  const PlOcpHandle& h = o->h;
  if (retract_steps < 1 || retract_steps > h.N) { pl_set_error("retract_steps %d outside [1, N]", retract_steps); return -1; }
  PL_CAS_LOCK;
  CasadiState& c = g_cas;
  c.o = o;
  c.steps = retract_steps;
  c.sp_x = dense_sp(h.n, 1);
  c.sp_p = dense_sp(h.np, 1);
  c.sp_n1 = dense_sp(h.n, 1);
  c.sp_m1 = dense_sp(h.m, 1);
  c.sp_11 = dense_sp(1, 1);
  c.sp_xinit = dense_sp(h.nx, 1);
  // J_g: compressed columns of the library pattern
  struct T { int col, row, e; };
  std::vector<T> t;
  t.reserve(h.nnz);
  for (int i = 0; i < h.N; ++i) {
    const PlNode& nd = o->nodes[i];
    const PlNode& nn = o->nodes[i + 1];
    const int* cp = o->colptr.data() + nd.colptr_off;
    for (int lc = 0; lc < nd.ncol; ++lc)
      for (int e = cp[lc]; e < cp[lc + 1]; ++e) {
        const int col = lc < nd.nw ? nd.x_off + lc : nn.x_off + (lc - nd.nw);
        t.push_back({col, nd.row_off + o->rowidx[nd.ent_off + e], nd.ent_off + e});
      }
  }
  std::sort(t.begin(), t.end(), [](const T& a, const T& b) { return a.col != b.col ? a.col < b.col : a.row < b.row; });
  c.sp_J.assign({h.m, h.n});
  std::vector<casadi_int> colind(h.n + 1, 0);
  for (const T& x : t) colind[x.col + 1]++;
  for (int j = 0; j < h.n; ++j) colind[j + 1] += colind[j];
  c.sp_J.insert(c.sp_J.end(), colind.begin(), colind.end());
  c.J_perm.resize(t.size());
  for (size_t k = 0; k < t.size(); ++k) {
    c.sp_J.push_back(t[k].row);
    c.J_perm[k] = t[k].e;
  }
  // hess_f: diagonal (ocp.py:293-296, P = diag)
  c.sp_H.assign({h.n, h.n});
  for (int j = 0; j <= h.n; ++j) c.sp_H.push_back(j);
  for (int j = 0; j < h.n; ++j) c.sp_H.push_back(j);
  int na, nf, nt;
  cas_u_split(o, na, nf, nt);
  if (PL_IS_CV(h.oc.dyn) && retract_steps >= h.N) {
    pl_set_error("centroidal_vel retract needs node i + 1's velocities: retract_steps < N");
    c.o = nullptr;
    return -1;
  }
  c.sp_q = dense_sp(retract_steps, h.oc.nq);
  c.sp_v = dense_sp(retract_steps, h.oc.nv);
  // a: inputs (rnea / acc; none for rnea include_acc = False, u_sol[:0]), ABA (aba), FD + dccrba (cv)
  c.sp_a = dense_sp(retract_steps, h.oc.dyn == PL_DYN_RNEAFD ? 0 : h.oc.nv);
  c.sp_f = dense_sp(retract_steps, nf);
  int ntau = nt;
  if (PL_IS_RNEA(h.oc.dyn))
    for (int i = 0; i < retract_steps; ++i)
      if (o->nodes[i].nu - na - nf < ntau) ntau = o->nodes[i].nu - na - nf;
  c.sp_tau = dense_sp(retract_steps, std::max(ntau, 0));
  return 0;
}

extern "C" void pl_casadi_unbind(void) {
  PL_CAS_LOCK;
  g_cas.o = nullptr;
}

static void cas_forget(const pl_ocp* o) {
  PL_CAS_LOCK;
  if (g_cas.o == o) g_cas.o = nullptr;
}

// ---- shared boilerplate of every external function
#define PL_CASADI_COMMON(NAME, NIN, NOUT)                                                          \
  extern "C" int NAME##_alloc_mem(void) { return 0; }                                              \
  extern "C" int NAME##_init_mem(int) { return 0; }                                                \
  extern "C" void NAME##_free_mem(int) {}                                                          \
  extern "C" int NAME##_checkout(void) { return 0; }                                               \
  extern "C" void NAME##_release(int) {}                                                           \
  extern "C" void NAME##_incref(void) {}                                                           \
  extern "C" void NAME##_decref(void) {}                                                           \
  extern "C" casadi_int NAME##_n_in(void) { return NIN; }                                          \
  extern "C" casadi_int NAME##_n_out(void) { return NOUT; }                                        \
  extern "C" double NAME##_default_in(casadi_int) { return 0.0; }                                  \
  extern "C" int NAME##_work(casadi_int* sz_arg, casadi_int* sz_res, casadi_int* sz_iw, casadi_int* sz_w) { \
    if (sz_arg) *sz_arg = NIN;                                                                     \
    if (sz_res) *sz_res = NOUT;                                                                    \
    if (sz_iw) *sz_iw = 0;                                                                         \
    if (sz_w) *sz_w = 0;                                                                           \
    return 0;                                                                                      \
  }

static const char* cas_name(const char* const* names, int count, casadi_int i) {
  return (i >= 0 && i < count) ? names[i] : nullptr;
}

// sqp_data(x, p) -> (grad_f, J_g, g, lbg, ubg)
PL_CASADI_COMMON(sqp_data, 2, 5)
extern "C" const char* sqp_data_name_in(casadi_int i) {
  static const char* n[] = {"i0", "i1"};
  return cas_name(n, 2, i);
}
extern "C" const char* sqp_data_name_out(casadi_int i) {
  static const char* n[] = {"o0", "o1", "o2", "o3", "o4"};
  return cas_name(n, 5, i);
}
extern "C" const casadi_int* sqp_data_sparsity_in(casadi_int i) {
  PL_CAS_LOCK;
  if (!cas_ready()) return nullptr;
  return i == 0 ? g_cas.sp_x.data() : (i == 1 ? g_cas.sp_p.data() : nullptr);
}
extern "C" const casadi_int* sqp_data_sparsity_out(casadi_int i) {
  PL_CAS_LOCK;
  if (!cas_ready()) return nullptr;
  switch (i) {
    case 0: return g_cas.sp_n1.data();
    case 1: return g_cas.sp_J.data();
    case 2: case 3: case 4: return g_cas.sp_m1.data();
    default: return nullptr;
  }
}
extern "C" int sqp_data(const double** arg, double** res, casadi_int*, double*, int) {
  PL_CAS_LOCK;
  if (!cas_ready() || cas_eval(arg, true)) return 1;
  PlOcpHandle* h = &g_cas.o->h;
  if (res[1]) g_cas.buf.resize(h->nnz);
  // every copy is enqueued (| does not short-circuit) and waited for before returning
  if (cas_get(h->d.grad, h->n, res[0]) | cas_get(h->d.Araw, h->nnz, res[1] ? g_cas.buf.data() : nullptr) |
      cas_get(h->d.g, h->m, res[2]) | cas_get(h->d.lbg, h->m, res[3]) | cas_get(h->d.ubg, h->m, res[4]) | cas_wait())
    return 1;
  if (res[1])
    for (size_t k = 0; k < g_cas.J_perm.size(); ++k) res[1][k] = g_cas.buf[g_cas.J_perm[k]];
  return 0;
}

// f_data(x, p) -> (f, grad_f)
PL_CASADI_COMMON(f_data, 2, 2)
extern "C" const char* f_data_name_in(casadi_int i) {
  static const char* n[] = {"i0", "i1"};
  return cas_name(n, 2, i);
}
extern "C" const char* f_data_name_out(casadi_int i) {
  static const char* n[] = {"o0", "o1"};
  return cas_name(n, 2, i);
}
extern "C" const casadi_int* f_data_sparsity_in(casadi_int i) { return sqp_data_sparsity_in(i); }
extern "C" const casadi_int* f_data_sparsity_out(casadi_int i) {
  PL_CAS_LOCK;
  if (!cas_ready()) return nullptr;
  return i == 0 ? g_cas.sp_11.data() : (i == 1 ? g_cas.sp_n1.data() : nullptr);
}
extern "C" int f_data(const double** arg, double** res, casadi_int*, double*, int) {
  PL_CAS_LOCK;
  if (!cas_ready() || cas_eval(arg, false)) return 1;
  PlOcpHandle* h = &g_cas.o->h;
  double w[8];
  if (cas_get(h->d.work, 8, w) | cas_get(h->d.grad, h->n, res[1]) | cas_wait()) return 1;
  if (res[0]) res[0][0] = w[0];
  return 0;
}

// g_data(x, p) -> (g, lbg, ubg)
PL_CASADI_COMMON(g_data, 2, 3)
extern "C" const char* g_data_name_in(casadi_int i) {
  static const char* n[] = {"i0", "i1"};
  return cas_name(n, 2, i);
}
extern "C" const char* g_data_name_out(casadi_int i) {
  static const char* n[] = {"o0", "o1", "o2"};
  return cas_name(n, 3, i);
}
extern "C" const casadi_int* g_data_sparsity_in(casadi_int i) { return sqp_data_sparsity_in(i); }
extern "C" const casadi_int* g_data_sparsity_out(casadi_int i) {
  PL_CAS_LOCK;
  if (!cas_ready()) return nullptr;
  return (i >= 0 && i < 3) ? g_cas.sp_m1.data() : nullptr;
}
extern "C" int g_data(const double** arg, double** res, casadi_int*, double*, int) {
  PL_CAS_LOCK;
  if (!cas_ready() || cas_eval(arg, false)) return 1;
  PlOcpHandle* h = &g_cas.o->h;
  return cas_get(h->d.g, h->m, res[0]) | cas_get(h->d.lbg, h->m, res[1]) | cas_get(h->d.ubg, h->m, res[2]) |
         cas_wait();
}

// hess_data(x, p) -> hess_f (diagonal pattern; constant, ocp.py:293-296)
PL_CASADI_COMMON(hess_data, 2, 1)
extern "C" const char* hess_data_name_in(casadi_int i) {
  static const char* n[] = {"i0", "i1"};
  return cas_name(n, 2, i);
}
extern "C" const char* hess_data_name_out(casadi_int i) { return i == 0 ? "o0" : nullptr; }
extern "C" const casadi_int* hess_data_sparsity_in(casadi_int i) { return sqp_data_sparsity_in(i); }
extern "C" const casadi_int* hess_data_sparsity_out(casadi_int i) {
  PL_CAS_LOCK;
  if (!cas_ready()) return nullptr;
  return i == 0 ? g_cas.sp_H.data() : nullptr;
}
extern "C" int hess_data(const double** arg, double** res, casadi_int*, double*, int) {
  PL_CAS_LOCK;
  if (!cas_ready()) return 1;
  pl_ocp* o = g_cas.o;
  PlOcpHandle* h = &o->h;
  if (!o->on_device) { pl_set_error("bound OCP has no device"); return 1; }
  (void)hipSetDevice(h->device);
  (void)hipGetLastError();
  if (!arg[1] || hipMemcpyAsync(h->d.p, arg[1], h->np * 8, hipMemcpyHostToDevice, h->stream) != hipSuccess) return 1;
  launch_hess(h);
  if (hipGetLastError() != hipSuccess) return 1;
  return cas_get(h->d.P, h->n, res[0]) | cas_wait();
}

// retract_solution(sol_x, x_init) -> (q, v, a, forces, tau), first `steps` nodes, node-major
// rows (ocp_whole_body_rnea.py:326-366).  Host computation (Lie-group integrate).
PL_CASADI_COMMON(retract_solution, 2, 5)
extern "C" const char* retract_solution_name_in(casadi_int i) {
  static const char* n[] = {"sol_x", "x_init"};
  return cas_name(n, 2, i);
}
extern "C" const char* retract_solution_name_out(casadi_int i) {
  static const char* n[] = {"q", "v", "a", "forces", "tau"};
  return cas_name(n, 5, i);
}
extern "C" const casadi_int* retract_solution_sparsity_in(casadi_int i) {
  PL_CAS_LOCK;
  if (!cas_ready()) return nullptr;
  return i == 0 ? g_cas.sp_x.data() : (i == 1 ? g_cas.sp_xinit.data() : nullptr);
}
extern "C" const casadi_int* retract_solution_sparsity_out(casadi_int i) {
  PL_CAS_LOCK;
  if (!cas_ready()) return nullptr;
  switch (i) {
    case 0: return g_cas.sp_q.data();
    case 1: return g_cas.sp_v.data();
    case 2: return g_cas.sp_a.data();
    case 3: return g_cas.sp_f.data();
    case 4: return g_cas.sp_tau.data();
    default: return nullptr;
  }
}
// compile_solution of each OCP (ocp_whole_body_rnea.py:326-366, ocp_whole_body_acc.py:236-288,
// ocp_whole_body_aba.py:216-264, ocp_centroidal_vel.py:262-324) on the host, with the
// library's own point functions (dyn.h): a = ABA (aba), tau = RNEA joints (acc, cv),
// cv: v from the inputs, a by forward difference with the base part from the
// centroidal base_acc_dynamics; the step sizes are the bound handle's (problem 0).
extern "C" int retract_solution(const double** arg, double** res, casadi_int*, double*, int) {
  PL_CAS_LOCK;
  if (!cas_ready() || !arg[0] || !arg[1]) return 1;
  const pl_ocp* o = g_cas.o;
  const PlModel& M = o->h.model;
  const PlOcpConst& O = o->h.oc;
  const int S = g_cas.steps, nq = M.nq, nv = M.nv, nj = O.nj;
  int na, nf, nt;
  cas_u_split(o, na, nf, nt);
  const int ntau = (int)g_cas.sp_tau[1];
  const bool cv = PL_IS_CV(O.dyn);
  std::vector<double> xs(O.nx), a(nv), tau(nv), vfull(nv), vnext(nv);
  PlFrameRef F0;
  memset(&F0, 0, sizeof(F0));
  const double* p = o->h_params.data();
  if (cv && !(p[O.P.dt_min] > 0.0 && p[O.P.dt_max] > 0.0)) {
    pl_set_error("retract_solution: the bound centroidal_vel OCP has no step sizes (pl_ocp_set_params)");
    return 1;
  }
  for (int i = 0; i < S; ++i) {
    const PlNode& nd = o->nodes[i];
    const double* dx = arg[0] + nd.x_off;
    const double* u = dx + o->h.ndx;
    pl::dyn_eval(M, O, F0, cv ? PL_FN_INTEGRATE_CV : PL_FN_INTEGRATE_WB, 0, arg[1], dx, nullptr, nullptr, xs.data());
    const double* q = cv ? xs.data() + 6 : xs.data();
    const double* v = cv ? u : xs.data() + nq;
    const double* f = u + (O.dyn == PL_DYN_ABA ? nj : na);
    if (O.dyn == PL_DYN_CVNB) {  // v = [base_vel_dynamics(h, q, v_j), v_j] (ocp_centroidal_vel.py:228-235)
      pl::dyn_eval(M, O, F0, PL_FN_BASE_VEL_CV, 0, xs.data(), q, u, nullptr, vfull.data());
      for (int k = 0; k < nj; ++k) vfull[6 + k] = u[k];
      v = vfull.data();
    }
    switch (O.dyn) {
      case PL_DYN_ABA:
        pl::dyn_eval(M, O, F0, PL_FN_ABA, 0, q, v, u, f, a.data());
        break;
      case PL_DYN_CV:
      case PL_DYN_CVNB: {
        const double dt = pl::node_dt(O, p, i);
        const double* un = arg[0] + o->nodes[i + 1].x_off + o->h.ndx;
        if (O.dyn == PL_DYN_CVNB) {  // v_next from this node's h, q (ocp_centroidal_vel.py:240-246)
          pl::dyn_eval(M, O, F0, PL_FN_BASE_VEL_CV, 0, xs.data(), q, un, nullptr, vnext.data());
          for (int k = 0; k < nj; ++k) vnext[6 + k] = un[k];
          un = vnext.data();
        }
        for (int k = 0; k < nv; ++k) a[k] = (un[k] - v[k]) / dt;
        pl::dyn_eval(M, O, F0, PL_FN_BASE_ACC_CV, 0, q, v, a.data() + 6, f, a.data());
      } break;
      case PL_DYN_ACCNB:  // a = [base_acc_dynamics(q, v, a_j, f), a_j] (ocp_whole_body_acc.py:124-135)
        for (int k = 0; k < nj; ++k) a[6 + k] = u[k];
        pl::dyn_eval(M, O, F0, PL_FN_BASE_ACC_WB, 0, q, v, u, f, a.data());
        break;
      default:
        for (int k = 0; k < nv; ++k) a[k] = u[k];
    }
    if (O.dyn == PL_DYN_ACC || O.dyn == PL_DYN_CA || O.dyn == PL_DYN_ACCNB || cv)
      pl::dyn_eval(M, O, F0, PL_FN_RNEA, 0, q, v, a.data(), f, tau.data());
    // CasADi dense matrices are column-major: element (row i, col k) at k * S + i
    if (res[0]) for (int k = 0; k < nq; ++k) res[0][k * S + i] = q[k];
    if (res[1]) for (int k = 0; k < nv; ++k) res[1][k * S + i] = v[k];
    if (res[2] && O.dyn != PL_DYN_RNEAFD) for (int k = 0; k < nv; ++k) res[2][k * S + i] = a[k];
    if (res[3]) for (int k = 0; k < nf; ++k) res[3][k * S + i] = f[k];
    if (res[4]) {
      for (int k = 0; k < ntau; ++k) {
        double t;
        if (PL_IS_RNEA(O.dyn)) t = u[na + nf + k];
        else if (O.dyn == PL_DYN_ABA) t = u[k];
        else t = tau[6 + k];
        res[4][k * S + i] = t;
      }
    }
  }
  return 0;
}
