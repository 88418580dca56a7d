// C-ABI of the batched MPC inner loop (include/pinoloco.h).
//
// Host side of the drop-in boundary: owns the device buffers of a batch and sequences
// the kernels of one SQP iteration exactly as OCP.solve() sequences sqp_data ->
// osqp.update -> osqp.solve -> line search (ocp.py:375-414), the MPC loop and the
// interior-point branch.  The layout the reference gets from CasADi Opti
// (optimization/ocp.py:38-44, 103-198, 283, 305) and the device programs are built in
// api_build.hip; the CasADi external-function ABI is api_casadi.hip.
#include "api_internal.h"

#include <map>

static thread_local char g_err[1024] = "";

void pl_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}



extern "C" const char* pl_last_error(void) { return g_err; }
extern "C" int pl_version(void) { return 1; }

// Build provenance: build.py passes the sha256 of csrc/* + include/*.h (PL_SRC_SHA), so a
// caller can tell which sources a pushed binary was built from (bench.py prints it,
// __graft_entry__.smoke() asserts it against the tree).
#ifndef PL_SRC_SHA
#define PL_SRC_SHA "unknown"
#endif
extern "C" const char* pl_build_info(void) { return "pl_src_sha256=" PL_SRC_SHA " arch=gfx950"; }

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


// ADMM kernel selection (the three give the same iterates to round-off):
//   sweep   k_admm: one wave per problem, node-by-node block sweeps (HBM-bound at B >= 1024)
//   sweep2  k_admm2: two waves per problem
//   chain   k_admm_rc: reduced chain, 8 waves per problem (small batches); up to ceil((N + 1) / 8)
//           workgroups per problem while the batch's workgroups fit one per CU (rc_groups)
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
    if (dalloc(o, &h.d.CH, (size_t)h.B * h.ch_stride) || dalloc(o, &h.d.chv, (size_t)h.B * h.chv_stride) ||
        dalloc(o, &h.d.rcsync, (size_t)h.B * PL_RC_SYNC))
      return -2;
  }
  h.admm_rc = kind == PL_ADMM_CHAIN ? 1 : 0;
  h.admm_waves = kind == PL_ADMM_SWEEP2 ? 2 : 1;
  return 0;
}

extern "C" int pl_ocp_create(const pl_model* model, const pl_ocp_desc* d, int batch, int device, pl_ocp** out) {
  if (!model || !d || !out || batch <= 0) { pl_set_error("bad arguments"); return -1; }
  if (d->dynamics < 0 || d->dynamics > 4) { pl_set_error("Unknown dynamics type: %d", d->dynamics); return -1; }
  // nodes >= 2 is also what k_admm's software pipeline relies on (the prefetch / deferred-store
  // invariant in its header: steps q - 1 and q + 1 never meet at a node both touch)
  if (d->nodes < 2 || d->n_feet != 4) { pl_set_error("need nodes >= 2 and 4 feet"); return -1; }
  if (d->debug_paths & ~PL_PATH_ALL) {
    pl_set_error("debug_paths 0x%x has bits outside PL_PATH_* (0x%x): zero the pl_ocp_desc", d->debug_paths, PL_PATH_ALL);
    return -1;
  }
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
  // ADMM kernel (admm_select below): the batch-size rule at creation, pl_ocp_set_admm_kernel
  // afterwards.  No environment variable changes a kernel path: the reference paths of the
  // regression tests and the phase timing are pl_ocp_desc.debug_paths bits.
  h.debug_paths = d->debug_paths;
  h.admm_waves = 1;
  h.admm_rc = 0;
  h.rc_waves = 8;
  h.ruiz_fused = !(h.debug_paths & PL_PATH_RUIZ_PER_PASS);
  h.ch_stride = rc_ch_stride(h.N, h.ndx, h.rc_waves);
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
  if (hipDeviceGetAttribute(&h.num_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || h.num_cu <= 0)
    h.num_cu = 1;  // unknown: k_admm_rc then runs one workgroup per problem
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
  {  // node-local (row, column) of each entry: the entry-order residual gathers of k_check_part
    std::vector<uint32_t> erl(h.nnz);
    for (int e = 0; e < h.nnz; ++e) erl[e] = ((uint32_t)o->rowidx[e] << 16) | (uint32_t)o->entcol[e];
    rc |= upload(o, &D.erl, erl);
  }
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
    std::vector<int2> jl, jlin;
    // PL_PATH_JAC_DUAL_ALL keeps the rnea a / f columns as dual tree-pass lanes (the r03 path)
    const bool use_lin = !(h.debug_paths & PL_PATH_JAC_DUAL_ALL);
    if (build_jac_list(o, jl, jlin, use_lin, &h.jl_ex)) {
      pl_ocp_destroy(o);
      return -1;
    }
    h.jl_len = (int)jl.size();
    h.jlin_len = (int)jlin.size();
    rc |= upload(o, &D.jlist, jl);
    D.jlin = nullptr;
    D.model0 = nullptr;
    if (!jlin.empty()) {
      rc |= upload(o, &D.jlin, jlin);
      PlModel m0 = h.model;  // zero gravity: the primal RNEA pass is then linear in (a, f)
      for (int k = 0; k < 3; ++k) m0.gravity[k] = 0.0;
      rc |= dalloc(o, &D.model0, 1);
      if (!rc && hipMemcpy(D.model0, &m0, sizeof(PlModel), hipMemcpyHostToDevice) != hipSuccess) rc = 1;
    }
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
  if (h.debug_paths & PL_PATH_ADMM_TIMING) rc |= dalloc(o, &D.dbg, B * 40);
  if (rc) { pl_ocp_destroy(o); return -2; }
  if (admm_select(o, PL_ADMM_AUTO)) { pl_ocp_destroy(o); return -2; }
  o->mpc_graph_off = (h.debug_paths & PL_PATH_NO_MPC_GRAPH) != 0;
  // the cheap Jacobian columns (dx_{i+1}, rnea tau_j, centroidal_vel h) have constant entries
  // (+-1, -m): written by the first evaluation only (PL_PATH_JAC_CONST_EVERY: every evaluation)
  o->h.jac_cheap_every = (h.debug_paths & PL_PATH_JAC_CONST_EVERY) != 0;
  o->h.jac_cheap_ok = 0;
  if (hipMemcpy(D.model, &h.model, sizeof(PlModel), hipMemcpyHostToDevice) != hipSuccess ||
      hipMemcpy(D.oc, &h.oc, sizeof(PlOcpConst), hipMemcpyHostToDevice) != hipSuccess) {
    pl_set_error("upload of model tables failed");
    pl_ocp_destroy(o);
    return -2;
  }
  *out = o;
  return 0;
}


extern "C" void pl_ocp_destroy(pl_ocp* o) {
  if (!o) return;
  cas_forget(o);  // a bound CasADi handle must not outlive its OCP
  if (o->on_device) {
    hipSetDevice(o->h.device);
    hipStreamSynchronize(o->h.stream);
    for (void* p : o->allocs) hipFree(p);
    for (int k = 0; k < 5; ++k) hipEventDestroy(o->ev[k]);
    if (o->mpc_graph) hipGraphExecDestroy(o->mpc_graph);
    if (o->dl_host) hipHostFree(o->dl_host);
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

extern "C" int pl_ocp_get_admm_groups(const pl_ocp* o) {
  if (!o) { pl_set_error("null handle"); return -1; }
  return o->h.admm_rc ? rc_groups(&o->h) : 1;
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

// A generic point of node i for the structural probes: random parameters in (0.5, 1.5)
// with sane step sizes and gait counts, contact 0.5 and swing 0.3 (stance and swing rows both
// active), a unit x_init quaternion, w_i and dx_{i+1} in (-0.1, 0.1); lam (if given) of both
// signs.
void generic_point(const PlOcpHandle& h, const std::vector<PlNode>& nodes, int i, std::vector<double>& p,
                   std::vector<double>& xw, std::vector<double>* lam, uint64_t salt = 0) {
  const PlOcpConst& O = h.oc;
  uint64_t st = 0x9e3779b97f4a7c15ull ^ (uint64_t)(i + 1) ^ (salt << 32);
  auto rnd = [&]() {  // uniform in (0.5, 1.5)
    st = st * 6364136223846793005ull + 1442695040888963407ull;
    return 0.5 + (double)(st >> 11) / 9007199254740992.0;
  };
  p.assign(O.P.np, 0.0);
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
  xw.assign(nodes[i].nw + O.ndx, 0.0);
  for (double& v : xw) v = 0.2 * (rnd() - 1.0);
  if (lam) {
    lam->assign(nodes[i].nrow, 0.0);
    for (size_t r = 0; r < lam->size(); ++r) (*lam)[r] = (r & 1) ? rnd() : -rnd();
  }
}

void hess_pattern(const PlOcpHandle& h, const std::vector<PlNode>& nodes, int i, std::vector<uint8_t>& nz) {
  const PlOcpConst& O = h.oc;
  std::vector<double> p, xw, lam;
  generic_point(h, nodes, i, p, xw, &lam);
  const int nw = nodes[i].nw;
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
struct HostJacEmit {
  uint8_t* nz;  // [nrow] of one column
  int r;
  void operator()(const Dual& v, double, double) {
    nz[r] = v.d != 0.0;
    ++r;
  }
};

template <int DYN>
void probe_jac(const PlModel& M, const PlOcpConst& O, int i, const double* p, const double* xw, int nw, int nrow,
               std::vector<uint8_t>& nz) {
  std::vector<Dual> kst(PL_KIN_STORE);
  std::vector<double> aba_sh(PL_ABA_SH);
  if (DYN == PL_DYN_ABA) pl::aba_primal(M, O, p, xw, aba_sh.data());  // the implicit-function ABA's primal
  const int ndx = O.ndx, ncol = nw + ndx;
  nz.assign((size_t)ncol * nrow, 0);
  for (int c = 0; c < ncol; ++c) {
    pl::VecIn<Dual> dx{xw, nullptr, 0.0, c};
    pl::VecIn<Dual> u{xw + ndx, nullptr, 0.0, c - ndx};
    pl::VecIn<Dual> dxn{xw + nw, nullptr, 0.0, c - nw};
    HostJacEmit e{nz.data() + (size_t)c * nrow, 0};
    pl::node_rows<Dual, DYN>(M, O, i, p, dx, u, dxn, e, kst.data(), 1, nullptr, aba_sh.data());
  }
}
}  // namespace

// Numerically non-zero Jacobian entries of node i at a generic point (column-major
// [ncol][nrow] flags over the node's local columns w_i, dx_{i+1}): the structural-dependency
// pattern CasADi's symbolic jacobian(g, x) would report, a subset of the library's
// kinematic-dependency pattern (api_build.hip::node_row_deps).  One forward-mode dual pass
// per column on the host, with the device's row code.
static void jac_probe(const PlOcpHandle& h, const std::vector<PlNode>& nodes, int i, uint64_t salt,
                      std::vector<uint8_t>& nz) {
  const PlOcpConst& O = h.oc;
  std::vector<double> p, xw;
  generic_point(h, nodes, i, p, xw, nullptr, salt);
  const int nw = nodes[i].nw, nrow = nodes[i].nrow;
  const PlModel& M = h.model;
  switch (O.dyn) {
    case PL_DYN_RNEA: probe_jac<PL_DYN_RNEA>(M, O, i, p.data(), xw.data(), nw, nrow, nz); break;
    case PL_DYN_RNEAFD: probe_jac<PL_DYN_RNEAFD>(M, O, i, p.data(), xw.data(), nw, nrow, nz); break;
    case PL_DYN_ACC: probe_jac<PL_DYN_ACC>(M, O, i, p.data(), xw.data(), nw, nrow, nz); break;
    case PL_DYN_CV: probe_jac<PL_DYN_CV>(M, O, i, p.data(), xw.data(), nw, nrow, nz); break;
    case PL_DYN_CA: probe_jac<PL_DYN_CA>(M, O, i, p.data(), xw.data(), nw, nrow, nz); break;
    case PL_DYN_ACCNB: probe_jac<PL_DYN_ACCNB>(M, O, i, p.data(), xw.data(), nw, nrow, nz); break;
    case PL_DYN_CVNB: probe_jac<PL_DYN_CVNB>(M, O, i, p.data(), xw.data(), nw, nrow, nz); break;
    default: probe_jac<PL_DYN_ABA>(M, O, i, p.data(), xw.data(), nw, nrow, nz); break;
  }
}

// The union over two independent generic points (an entry that vanishes at one random point
// by accident does not vanish at both).
void jac_pattern(const PlOcpHandle& h, const std::vector<PlNode>& nodes, int i, std::vector<uint8_t>& nz) {
  std::vector<uint8_t> nz2;
  jac_probe(h, nodes, i, 0, nz);
  jac_probe(h, nodes, i, 1, nz2);
  for (size_t k = 0; k < nz.size(); ++k) nz[k] |= nz2[k];
}

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
        dalloc(o, &h->d.ip_iflag, (size_t)4 * h->B) || dalloc(o, &h->d.ip_act, (size_t)h->B + 2))
      return -2;
    // Lagrangian Hessian work list (k_hess.hip): the structurally non-zero column pairs
    // j <= k of every w_i block (hess_pattern, one probe per node type); node blocks packed
    // lower, the pairs not listed stay 0
    std::vector<int2> hl, hlin, hvv, htr, hcone, htrf;
    std::vector<int> hoff;
    long long off = 0;
    const PlOcpConst& O = h->oc;
    std::vector<uint8_t> pat[3];
    // whole_body_rnea / whole_body_acc: the rows are linear in a and in the contact forces, and only the RNEA rows
    // couple them to q, so the (dq, a) and (dq, f_feet) blocks are d/dq of M(q) lambda_tau and
    // of -J_e(q) lambda_tau (k_lag_hess_lin: two dual tree passes per dq column instead of one
    // hyper-dual pass per pair); PL_PATH_HESS_DUAL_ALL keeps them as pairs
    const bool lin = (O.dyn == PL_DYN_RNEA || O.dyn == PL_DYN_ACC) &&
                     !(h->debug_paths & PL_PATH_HESS_DUAL_ALL);
    const int lin_lo = O.ndx, lin_hi = O.ndx + O.na + 3 * O.nfeet;
    // rnea family and whole_body_acc: the chain of a w_i coordinate (-1: the base, or none).  The rows are sums of
    // per-chain terms that read the base and their own chain only, so a pair with a coordinate
    // of chain c has a mixed part from chain c's terms alone, and its pass skips the other
    // chains (tree_pass only_ch, packed as .x = node | (chain + 1) << 16).  PL_PATH_HESS_FULL_TREE: off
    const bool chains = (PL_IS_RNEA(O.dyn) || O.dyn == PL_DYN_ACC) &&
                        !(h->debug_paths & PL_PATH_HESS_FULL_TREE);
    const PlModel& Mo = h->model;
    const auto joint_chain = [&](int jt) {
      for (int c = 0; c < Mo.nchains; ++c)
        if (jt >= Mo.chain_first[c] && jt < Mo.chain_first[c] + Mo.chain_len[c]) return c;
      return -1;
    };
    const auto vidx_chain = [&](int vi) {
      if (vi < 6) return -1;
      for (int jt = 2; jt < Mo.njoints; ++jt)
        if (Mo.idx_v[jt] == vi) return joint_chain(jt);
      return -1;
    };
    const auto coord_chain = [&](int c) {
      if (c < O.ndx) return vidx_chain(c < O.nv ? c : c - O.nv);
      const int k = c - O.ndx;
      if (k < O.na) return vidx_chain(k);
      if (k < O.na + O.nf) {
        const int e = (k - O.na) / 3;
        return joint_chain(e < O.nfeet ? O.feet[e].joint : O.ext.joint);
      }
      return vidx_chain(6 + k - O.na - O.nf);
    };
    const auto pair_chain = [&](int j, int k) {
      if (!chains) return -1;
      const int cj = coord_chain(j), ck = coord_chain(k);
      if (cj < 0) return ck;
      if (ck < 0 || ck == cj) return cj;
      return -1;  // two chains: structurally zero, kept on the full pass
    };
    for (int i = 0; i <= h->N; ++i) {
      const int nw = o->nodes[i].nw;
      hoff.push_back((int)off);
      off += (long long)nw * (nw + 1) / 2;
      if (i == h->N) break;  // no rows on the last node
      const int type = pl::node_type(O, i);
      if (pat[type].empty()) hess_pattern(*h, o->nodes, i, pat[type]);
      for (int k = 0; k < nw; ++k)
        for (int j = 0; j <= k; ++j) {
          if (lin && j < O.nv && k >= lin_lo && k < lin_hi) continue;
          if (!pat[type][(size_t)k * (k + 1) / 2 + j]) continue;
          // two state columns: the curvature of the tree-pass rows alone (k_lag_hess_tree), and for
          // (dv, dv) the quadratic form of the RNEA bias term (k_lag_hess_vv)
          const int ff = O.ndx + O.na;  // the foot forces
          if (lin && j == k && j >= ff && j < ff + 3 * O.nfeet) {  // the friction cones (k_lag_hess_cone)
            hcone.push_back(make_int2(i, j));
            continue;
          }
          if (lin && j >= 3 && j < O.nv && k >= ff + 3 * O.nfeet && k < ff + 3 * O.nee) {  // (dq, f_ext)
            htrf.push_back(make_int2(i | ((pair_chain(j, k) + 1) << 16), j | (k << 16)));
            continue;
          }
          const bool st = lin && k < O.ndx;
          (st ? (j >= O.nv ? hvv : htr) : hl).push_back(make_int2(i | ((pair_chain(j, k) + 1) << 16), j | (k << 16)));
        }
      if (lin)  // RNEA ignores the base position
        for (int k = 3; k < O.nv; ++k) hlin.push_back(make_int2(i, k | ((chains ? vidx_chain(k) + 1 : 0) << 16)));
    }
    for (int t = 0; t < 3; ++t) {  // first row of the RNEA base / joint-torque row blocks per node type
      h->hl_rb_base[t] = h->hl_rb_tau[t] = -1;
      int r = 0;
      for (int bi = 0; bi < O.nblk[t]; ++bi) {
        if (O.blk[t][bi].kind == PL_RB_RNEA_BASE) h->hl_rb_base[t] = r;
        if (O.blk[t][bi].kind == PL_RB_TAU_EQ) h->hl_rb_tau[t] = r;
        r += O.blk[t][bi].count;
      }
    }
    // the written entries of a node block per node type (k_ip_refine's H_i dx): the pattern and,
    // with the linear-column identity, the whole (dq_k, a | f_feet) rows k_lag_hess_lin stores
    std::vector<int> hnz;
    for (int t = 0; t < 3; ++t) {
      h->hnz_off[t] = (int)hnz.size();
      int nw = -1;
      for (int i = 0; i < h->N; ++i)
        if (pl::node_type(O, i) == t) { nw = o->nodes[i].nw; break; }
      if (nw < 0 || pat[t].empty()) continue;
      for (int k = 0; k < nw; ++k)
        for (int j = 0; j <= k; ++j)
          if (pat[t][(size_t)k * (k + 1) / 2 + j] || (lin && j >= 3 && j < O.nv && k >= lin_lo && k < lin_hi))
            hnz.push_back(k | (j << 16));
    }
    h->hnz_off[3] = (int)hnz.size();
    if (!hnz.empty() && upload(o, &h->d.hnz, hnz)) return -2;
    // the (dq, dq) / (dq, dv) pairs as forward-over-reverse columns (k_lag_hess_col, r06): the pair
    // (j, k), j <= k, is written by the item (node, chain, j) with k's local coordinate in its mask
    // (hess_tree.h col_coord).  The column sweep assumes no frame on the root and at most one frame
    // (a foot or the external force) per chain; otherwise, without chain confinement, or with
    // PL_PATH_HESS_PAIRS the pair kernel runs.
    std::vector<int4> hcol;
    {
      bool ok = chains && !htr.empty() && !(h->debug_paths & PL_PATH_HESS_PAIRS);
      for (int e = 0; e < O.nee && ok; ++e)
        if ((e < O.nfeet ? O.feet[e].joint : O.ext.joint) == 1) ok = false;
      for (int c = 0; c < Mo.nchains && ok; ++c) {
        int nfr = 0;
        for (int e = 0; e < O.nee; ++e) {
          const int fj = e < O.nfeet ? O.feet[e].joint : O.ext.joint;
          if (fj >= Mo.chain_first[c] && fj < Mo.chain_first[c] + Mo.chain_len[c]) ++nfr;
        }
        if (nfr > 1 || 12 + 2 * Mo.chain_len[c] > 32) ok = false;
      }
      const auto loc_of = [&](int ch, int k) {  // k (a state dx index) in chain ch's local coordinates
        if (k < 6) return k;
        if (k >= O.nv && k < O.nv + 6) return 6 + k - O.nv;
        if (ch < 0) return -1;
        const int first = Mo.chain_first[ch], L = Mo.chain_len[ch];
        for (int kk = 0; kk < L; ++kk) {
          if (Mo.idx_v[first + kk] == k) return 12 + kk;
          if (O.nv + Mo.idx_v[first + kk] == k) return 12 + L + kk;
        }
        return -1;
      };
      std::map<long long, uint32_t> cols;  // (node, chain, j) -> mask, in work-list order
      for (const int2& pr : htr) {
        const int i = pr.x & 0xffff, ch = (pr.x >> 16) - 1, j = pr.y & 0xffff, k = pr.y >> 16;
        const int lk = loc_of(ch, k);
        if (lk < 0) { ok = false; break; }
        cols[((long long)i << 32) | ((long long)(ch + 1) << 16) | j] |= 1u << lk;
      }
      h->hcol_nbase = 0;
      if (ok)
        for (int pass = 0; pass < 2; ++pass)  // the whole-tree base columns first (k_lag_hess_col<true>)
          for (const auto& kv : cols) {
            const int chp = (int)((kv.first >> 16) & 0xffff);
            if ((chp == 0) != (pass == 0)) continue;
            hcol.push_back(make_int4((int)(kv.first >> 32) | (chp << 16), (int)(kv.first & 0xffff), (int)kv.second, 0));
            if (pass == 0) ++h->hcol_nbase;
          }
    }
    h->hcol_len = (int)hcol.size();
    // k_lag_hess_arm's pairs: those on the base or the arm's chain (the others have no arm-row curvature;
    // until r05 their waves ran and exited)
    std::vector<int2> harm;
    {
      int arm_ch = -1;
      for (int c = 0; c < Mo.nchains; ++c)
        if (O.arm.valid && O.arm.joint >= Mo.chain_first[c] && O.arm.joint < Mo.chain_first[c] + Mo.chain_len[c]) arm_ch = c;
      if (arm_ch >= 0)
        for (const int2& pr : htr) {
          const int ch = (pr.x >> 16) - 1;
          if (ch < 0 || ch == arm_ch) harm.push_back(pr);
        }
    }
    h->harm_len = (int)harm.size();
    h->hl_len = (int)hl.size();
    h->hlin_len = (int)hlin.size();
    h->hvv_len = (int)hvv.size();
    h->htr_len = (int)htr.size();
    h->hcone_len = (int)hcone.size();
    h->htrf_len = (int)htrf.size();
    h->hl_stride = (off + 1) & ~1LL;
    if ((!hl.empty() && upload(o, &h->d.hlist, hl)) || upload(o, &h->d.hoff, hoff) ||
        dalloc(o, &h->d.Hlag, (size_t)h->B * h->hl_stride))
      return -2;
    if (lin) {
      PlModel m0 = h->model;
      for (int k = 0; k < 3; ++k) m0.gravity[k] = 0.0;
      if (upload(o, &h->d.hlin, hlin) || (!hvv.empty() && upload(o, &h->d.hvv, hvv)) ||
          (!htr.empty() && upload(o, &h->d.htr, htr)) || (!hcone.empty() && upload(o, &h->d.hcone, hcone)) ||
          (!htrf.empty() && upload(o, &h->d.htrf, htrf)) || (!hcol.empty() && upload(o, &h->d.hcol, hcol)) ||
          (!harm.empty() && upload(o, &h->d.harm, harm)))
        return -2;
      if (!h->d.model0 && (dalloc(o, &h->d.model0, 1) ||
                           hipMemcpy(h->d.model0, &m0, sizeof(PlModel), hipMemcpyHostToDevice) != hipSuccess))
        return -2;
    }
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
    s.ref_solves = info[b].ref_solves;
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

// The key is the handle up to its profiling fields: every launcher takes its launch
// parameters (grid, LDS bytes, kernel choice, pointers, settings) from `h` and from
// nothing else (no getenv, statics or pl_ocp fields at launch time), so equal bytes mean
// an equal launch sequence.  Profiling runs never replay (pl_mpc_step), so the event
// handles and counters stay out of the key.
static constexpr size_t kMpcKeyBytes = offsetof(PlOcpHandle, profile);

static int mpc_sqp_graph(pl_ocp* o) {
  PlOcpHandle* h = &o->h;
  const unsigned char* hb = reinterpret_cast<const unsigned char*>(h);
  const bool same = o->mpc_key.size() == kMpcKeyBytes && !memcmp(o->mpc_key.data(), hb, kMpcKeyBytes);
  if (same && o->mpc_graph) {
    ++o->mpc_replays;
    return hipGraphLaunch(o->mpc_graph, h->stream) == hipSuccess ? 0 : -1;
  }
  if (o->mpc_graph) {
    hipGraphExecDestroy(o->mpc_graph);
    o->mpc_graph = nullptr;
  }
  if (!same) {  // first sighting of this state: eager, remember it
    o->mpc_key.assign(hb, hb + kMpcKeyBytes);
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
  ++o->mpc_replays;
  return hipGraphLaunch(o->mpc_graph, h->stream) == hipSuccess ? 0 : -1;
}

extern "C" int pl_mpc_set_ip_lam(pl_ocp* o, int carry) {
  if (!o || (carry != 0 && carry != 1)) { pl_set_error("pl_mpc_set_ip_lam: carry must be 0 or 1"); return -1; }
  o->h.ip_mpc_lam = carry;
  return 0;
}

// MPC-step graph state (tests): [captures, replays, eager fallback (1: capture or replay
// failed, or PL_MPC_GRAPH=0)].
extern "C" int pl_mpc_graph_info(const pl_ocp* o, long long* out) {
  if (!o || !out) { pl_set_error("null argument"); return -1; }
  out[0] = o->mpc_captures;
  out[1] = o->mpc_replays;
  out[2] = o->mpc_graph_off;
  return 0;
}

extern "C" int pl_mpc_step(pl_ocp* o, int k) {
  REQUIRE_DEVICE(o);
  // the event slots: 64 ADMM launches, 16 Hessian launches (an interior-point step makes <= 10)
  if (o->h.profile && (o->h.prof_n > 48 || o->h.prof_hn > 0)) prof_collect(&o->h);
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
    PlOcpHandle* h = &o->h;
    if (h->ip_mpc_lam) {
      // the Opti branch (compile_solver = False): warm_start() of the next step passes this
      // solve's lam_g back (ocp.py:373, ocp_*.py warm_start)
      PL_CHECK_HIP(hipMemcpyAsync(h->d.ip_lam0, h->d.ip_lam, (size_t)h->B * h->m * 8, hipMemcpyDeviceToDevice,
                                  h->stream));
      h->ip_lam_warm = 1;
    } else {
      // the reference's default driver (solver "fatrop", compile_solver = True, run_mpc.py:34-37,
      // 50-111): the compiled solver takes the primal warm start only (its inputs end with opti.x,
      // ocp_whole_body_rnea.py:239-257, the lam_g output commented out), so every solve starts
      // from cold multipliers
      h->ip_lam_warm = 0;
    }
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

extern "C" int pl_mpc_download(pl_ocp* o, double* host_dst) {
  REQUIRE_DEVICE(o);
  if (!host_dst) { pl_set_error("null argument"); return -1; }
  PlOcpHandle* h = &o->h;
  const int nu0 = o->nodes[0].nu;
  const size_t row = (size_t)nu0 + h->nx, bytes = row * h->B * 8;
  if (o->dl_bytes < bytes) {
    if (o->dl_host) hipHostFree(o->dl_host);
    o->dl_host = nullptr;
    o->dl_bytes = 0;
    PL_CHECK_HIP(hipHostMalloc(&o->dl_host, bytes, hipHostMallocDefault));
    o->dl_bytes = bytes;
  }
  char* dst = (char*)o->dl_host;
  PL_CHECK_HIP(hipMemcpy2DAsync(dst, row * 8, h->d.x + h->ndx, (size_t)h->n * 8, (size_t)nu0 * 8, h->B,
                                hipMemcpyDeviceToHost, h->stream));
  PL_CHECK_HIP(hipMemcpy2DAsync(dst + (size_t)nu0 * 8, row * 8, h->d.xstate, (size_t)h->nx * 8, (size_t)h->nx * 8,
                                h->B, hipMemcpyDeviceToHost, h->stream));
  PL_CHECK_HIP(hipStreamSynchronize(h->stream));
  memcpy(host_dst, o->dl_host, bytes);
  return 0;
}

static void prof_collect(PlOcpHandle* h) {
  if (!h->profile || (h->prof_n == 0 && h->prof_hn == 0)) return;
  hipStreamSynchronize(h->stream);
  for (int k = 0; k < h->prof_hn; ++k) {
    float ms = 0.f;
    hipEventElapsedTime(&ms, h->prof_hev[k][0], h->prof_hev[k][1]);
    h->prof_hess_ms += ms;
    h->prof_hess_launches++;
  }
  h->prof_hn = 0;
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
    for (int k = 0; k < 16; ++k) {
      hipEventCreate(&h->prof_hev[k][0]);
      hipEventCreate(&h->prof_hev[k][1]);
    }
  }
  h->profile = enable;
  h->prof_n = 0;
  h->prof_admm_ms = 0.0;
  h->prof_admm_launches = 0;
  h->prof_admm_iters = 0;
  h->prof_hn = 0;
  h->prof_hess_ms = 0.0;
  h->prof_hess_launches = 0;
  if (enable && h->d.ip_act) PL_CHECK_HIP(hipMemsetAsync(h->d.ip_act + h->B + 1, 0, sizeof(int), h->stream));
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

// Per-launch timing of the interior point's Lagrangian Hessian (k_lag_hess), recorded with the
// ADMM timing while pl_ocp_profile is on.  out: [total_ms, launches].
extern "C" int pl_ocp_profile_read_hess(pl_ocp* o, double* out) {
  REQUIRE_DEVICE(o);
  if (!out) { pl_set_error("null argument"); return -1; }
  prof_collect(&o->h);
  out[0] = o->h.prof_hess_ms;
  out[1] = (double)o->h.prof_hess_launches;
  int lanes = 0;  // Hessian lanes launched since profiling started (k_ip_compact)
  if (o->h.d.ip_act)
    PL_CHECK_HIP(hipMemcpy(&lanes, o->h.d.ip_act + o->h.B + 1, sizeof(int), hipMemcpyDeviceToHost));
  out[2] = o->h.prof_hess_launches > 0 ? (double)lanes / o->h.prof_hess_launches : 0.0;
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
  out[10] = admm_asb_cap(&o->h); out[11] = o->h.nent_max; out[12] = o->h.debug_paths;
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
      {"admm_t", h->d.dbg, h->d.dbg ? B * 40 : 0}, {"Ps", h->d.Ps, B * h->n},   {"P", h->d.P, B * h->n},         {"xa", h->d.xa, B * h->n},
      {"za", h->d.za, B * h->m},   {"ya", h->d.ya, B * h->m},       {"S", h->d.S, B * (size_t)h->S_stride},
      {"FS", h->d.FS, h->d.FS ? B * (size_t)h->fs_stride : 0},
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
      if (!it.p) { pl_set_error("array %s not allocated (set_solver first)", name); return -1; }
      if ((size_t)count < it.len) { pl_set_error("buffer too small for %s (%zu)", name, it.len); return -1; }
      if (out) PL_CHECK_HIP(hipMemcpyAsync(out, it.p, it.len * 8, hipMemcpyDeviceToHost, h->stream));
      else PL_CHECK_HIP(hipMemcpyAsync(it.p, in, it.len * 8, hipMemcpyHostToDevice, h->stream));
      if (in && it.p == h->d.Araw) {  // the constant entries are rewritten by the next (eager) step
        h->jac_cheap_ok = 0;
        o->mpc_key.clear();
      }
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
