// OCP layout and device programs (host side of the C-ABI, include/pinoloco.h): the
// variable / row / sparsity layout the reference gets from CasADi Opti
// (optimization/ocp.py:38-44, 103-198, 283, 305), the ADMM and factor node programs and
// the Jacobian work list.  Called by pl_ocp_create (api.hip).
#include <algorithm>
#include "api_internal.h"

// ---------------------------------------------------------------------------
// layout

static void add_block(PlOcpConst& O, int type, int kind, int count, int arg = 0) {
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
  // short coupling-row lists (the integration rows of rnea / acc: 2 entries): E_{i+1} straight
  // from S (4 products per entry, the lists staged per row in LDS: 4 values | 4 columns)
  // instead of through Y; longer lists (aba, centroidal): E_{i+1} = Wc S Wc^T on the f64 MFMA
  // with Wc and Y = Wc S dense in the Y buffer ([X16][NWS] each, r04; PL_FCHAIN_MF=0: the
  // list route)
  const bool is_short = !h.fac_gc && cwlen_max <= 4;
  const int X16 = (X + 15) & ~15, NWS = ((h.nw_max + 15) & ~15) + 1;
  h.fchain_ncw = ((is_short ? std::max(ncw_max, 6 * X) : ncw_max) + 1) & ~1;
  h.fchain_nc = h.fac_gc ? nc_max : 0;
  h.fchain_nxc = h.fac_gc ? (nxc_max + 1) & ~1 : 0;
  const int ngc = h.fac_gc ? ((nc_max * nc_max + h.fchain_nxc + nc_max + 1) & ~1) : 0;
  const auto chain_lds = [&](int ny_) { return (nS + ny_ + nE + h.fchain_ncw + 2 * X + 10 + ngc) * 8; };  // + stamps
  bool mf = !h.fac_gc && !is_short && !(h.debug_paths & PL_PATH_FCHAIN_LIST);
  // the MFMA route's dense Wc / Y buffers must fit beside S_i: a model too wide for them takes
  // the list route (which needs only the halves of Y)
  if (mf && chain_lds(std::max(ny, (2 * X16 * NWS + 1) & ~1)) > 160 * 1024) mf = false;
  if (mf) ny = std::max(ny, (2 * X16 * NWS + 1) & ~1);
  h.fchain_ny = ny;
  h.fchain_short = is_short ? (cwlen_max <= 2 ? 3 : 1) : (mf ? 2 : 0);
  h.fchain_lds = chain_lds(ny);
  if (h.fchain_lds > 160 * 1024) { pl_set_error("factor kernel: chain needs %d bytes of LDS", h.fchain_lds); return -1; }
  if (o->kasm.empty()) o->kasm.assign(NT, 0);
  if (o->kcpl.empty()) o->kcpl.assign(4, 0);
  return 0;
}


// Work list of the Jacobian kernel (k_eval_jac): one lane per non-empty local column.
// Columns whose dual pass runs the tree / ABA / centroidal recursion come first, packed
// 64 per wave ACROSS node boundaries and padded to whole waves; then the columns that
// skip it (dx_{i+1}; rnea tau_j; centroidal h), which are cheap.  The classification
// mirrors node_rows' skip logic (rows.h); it only affects the schedule.
int build_jac_list(pl_ocp* o, std::vector<int2>& list, std::vector<int2>& lin, bool use_lin, int* n_ex) {
  const PlOcpConst& O = o->h.oc;
  std::vector<int2> ex, ch;
  const PlModel& Mo = o->h.model;
  const auto chain_of = [&](int j) {
    for (int c = 0; c < Mo.nchains; ++c)
      if (j >= Mo.chain_first[c] && j < Mo.chain_first[c] + Mo.chain_len[c]) return c;
    return -1;
  };
  const auto vidx_chain = [&](int vi) {  // the chain of velocity index vi (-1: the base)
    if (vi < 6) return -1;
    for (int j = 2; j < Mo.njoints; ++j)
      if (Mo.idx_v[j] == vi) return chain_of(j);
    return -1;
  };
  // whole_body_rnea / _acc with the linear a / f columns: the dq / dv tree-pass columns run
  // confined to their chain (k_eval_jac only_ch); the r03 path (PL_PATH_JAC_DUAL_ALL) does not
  const bool confine = use_lin && (O.dyn == PL_DYN_RNEA || O.dyn == PL_DYN_ACC);
  const int slots = confine ? PL_JAC_SLOTS_CH : PL_JAC_SLOTS;
  lin.clear();
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
        // rnea / acc: the base position enters the integration rows only (rows.h seed_pos)
        if ((PL_IS_RNEA(O.dyn) || O.dyn == PL_DYN_ACC) && lc < 3) cheap = true;
      } else {
        const int k = lc - O.ndx;
        cheap = PL_IS_RNEA(O.dyn) && k >= O.na + O.nf;
        if (use_lin && (PL_IS_RNEA(O.dyn) || O.dyn == PL_DYN_ACC) && !cheap) {  // a / f: linear in the RNEA (k_eval_jac_lin)
          lin.push_back(make_int2(i, lc));
          continue;
        }
      }
      int tag = 0;
      if (confine && !cheap && lc < O.ndx) tag = (vidx_chain(lc < O.nv ? lc : lc - O.nv) + 1) << 16;
      (cheap ? ch : ex).push_back(make_int2(i, lc | tag));
    }
  }
  if (confine) {  // grouped by chain (the base columns first), each group padded to whole waves
    std::stable_sort(ex.begin(), ex.end(), [](const int2& a, const int2& b) { return (a.y >> 16) < (b.y >> 16); });
    std::vector<int2> g;
    for (size_t q = 0; q < ex.size(); ++q) {
      if (q > 0 && (ex[q].y >> 16) != (ex[q - 1].y >> 16))
        while (g.size() % 64) g.push_back(make_int2(-1, -1));
      g.push_back(ex[q]);
    }
    ex.swap(g);
  }
  while (ex.size() % 64) ex.push_back(make_int2(-1, -1));
  // a wave's lanes hold at most `slots` consecutive nodes (shared-value slots)
  for (size_t w = 0; w < ex.size(); w += 64) {
    int last = ex[w].x;
    for (size_t q = w; q < w + 64; ++q) last = std::max(last, ex[q].x);
    if (last - ex[w].x >= slots) {
      pl_set_error("Jacobian wave spans more than %d nodes", slots);
      return -1;
    }
  }
  *n_ex = (int)ex.size();
  list = ex;
  list.insert(list.end(), ch.begin(), ch.end());
  if (!lin.empty()) {
    // the chain a column's RNEA pass is confined to (k_eval_jac_lin: tree_pass only_ch; -1:
    // a base acceleration, which moves every chain); the list is grouped by chain so that a
    // wave's lanes walk the same chain.  .y = local column | (chain + 1) << 16.
    for (int2& w : lin) {
      const int k = w.y - O.ndx;
      int c = -1;
      if (k < O.na) {
        for (int j = 2; j < Mo.njoints; ++j)
          if (Mo.idx_v[j] == k) c = chain_of(j);
      } else {
        const int e = (k - O.na) / 3;
        c = chain_of(e < O.nfeet ? O.feet[e].joint : O.ext.joint);
      }
      w.y |= (c + 1) << 16;
    }
    std::stable_sort(lin.begin(), lin.end(), [](const int2& a, const int2& b) { return (a.y >> 16) < (b.y >> 16); });
  }
  while (lin.size() % 64) lin.push_back(make_int2(-1, -1));
  return 0;
}
