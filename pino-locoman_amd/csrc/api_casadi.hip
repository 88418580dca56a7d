// CasADi external-function ABI over the batched OCP (see the section comment below).
#include "api_internal.h"

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
#include <string>

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
  // J_g: compressed columns of the structural-dependency pattern, the one CasADi's symbolic
  // J_g = jacobian(g, x) reports (ocp.py:283) and the reference sets OSQP's A up with
  // (ocp.py:305-306): the library's entries that are non-zero at a generic point
  // (jac_pattern, one dual probe per node type).  The library's own pattern (a superset:
  // kinematic dependencies, e.g. the base position columns RNEA never reads) stays internal.
  struct T { int col, row, e; };
  std::vector<T> t;
  t.reserve(h.nnz);
  std::vector<uint8_t> pat[3];
  for (int i = 0; i < h.N; ++i) {
    const PlNode& nd = o->nodes[i];
    const PlNode& nn = o->nodes[i + 1];
    const int* cp = o->colptr.data() + nd.colptr_off;
    const int type = pl::node_type(h.oc, i);
    if (pat[type].empty()) jac_pattern(h, o->nodes, i, pat[type]);
    for (int lc = 0; lc < nd.ncol; ++lc)
      for (int e = cp[lc]; e < cp[lc + 1]; ++e) {
        const int r = o->rowidx[nd.ent_off + e];
        if (!pat[type][(size_t)lc * nd.nrow + r]) continue;
        const int col = lc < nd.nw ? nd.x_off + lc : nn.x_off + (lc - nd.nw);
        t.push_back({col, nd.row_off + r, nd.ent_off + e});
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

void cas_forget_compiled(const pl_ocp* o);
void cas_forget(const pl_ocp* o) {
  {
    PL_CAS_LOCK;
    if (g_cas.o == o) g_cas.o = nullptr;
  }
  cas_forget_compiled(o);
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

// ---------------------------------------------------------------------------
// compiled_solver(params..., [x_warm_start], [tau_prev, W_diag]) -> x: the Fatrop branch's generated
// solver function (opti.to_function("compiled_solver", solver_params, [opti.x]),
// ocp.py:324-342, ocp_whole_body_rnea.py:237-258), loaded by the reference's hardware driver
// with ca.external("compiled_solver", "codegen/lib/...") (run_mpc.py:51-53) and called as
// sol_x = solver_function(*params) (run_mpc.py:100).  Its inputs, in order: x_init, dt_min,
// dt_max, contact_schedule (n_feet x N), swing_schedule (n_feet x N), n_contacts, swing_period,
// swing_height, swing_vel_limits, Q_diag, R_diag, base_vel_des, [ext_force_des if the OCP has
// the external-force frame], [arm_vel_des if it has the arm frame], [opti.x if compiled with
// warm_start], [tau_prev, W_diag for whole_body_rnea].  One call is one interior-point solve
// (pl_ocp_set_solver(PL_SOLVER_IP)) of the bound batch-1 handle from COLD multipliers (the
// generated function has no lam_g input; its output list has lam_g commented out); the
// parameters it does not list keep the values the handle held at bind time (Opti bakes them in
// at to_function), and without warm_start x starts from the bound initial guess.  A solve that
// stops at the iteration cap or in a failed line search returns its last iterate.
namespace {
struct CompiledSlot {
  int off, len;  // parameter-vector offset and length; off = -1: the primal warm start x
};
struct CompiledState {
  pl_ocp* o = nullptr;
  std::vector<CompiledSlot> slots;
  std::vector<std::vector<casadi_int>> sp_in;
  std::vector<casadi_int> sp_out;
  std::vector<double> p0, x0, p, x;
  std::vector<std::string> names;
};
CompiledState g_cs;
}  // namespace

extern "C" int pl_casadi_bind_compiled(pl_ocp* o, int warm_start, const double* x_initial) {
  if (!o) { pl_set_error("null handle"); return -1; }
  const PlOcpHandle& h = o->h;
  if (h.B != 1) { pl_set_error("compiled_solver: bind a batch-1 handle (the generated solver is single-problem)"); return -1; }
  if (h.solver != PL_SOLVER_IP) { pl_set_error("compiled_solver: the handle must use the interior-point solver (PL_SOLVER_IP)"); return -1; }
  if (!warm_start && !x_initial) { pl_set_error("compiled_solver without warm_start needs the initial guess"); return -1; }
  PL_CAS_LOCK;
  CompiledState& c = g_cs;
  c.o = o;
  c.slots.clear();
  c.sp_in.clear();
  c.names.clear();
  const PlOcpConst& O = h.oc;
  auto add = [&](const char* name, int off, int nrow, int ncol) {
    c.slots.push_back({off, nrow * ncol});
    c.sp_in.push_back(dense_sp(nrow, ncol));
    c.names.push_back(name);
  };
  add("x_init", O.P.x_init, O.nx, 1);
  add("dt_min", O.P.dt_min, 1, 1);
  add("dt_max", O.P.dt_max, 1, 1);
  add("contact_schedule", O.P.contact, 4, O.N);
  add("swing_schedule", O.P.swing, 4, O.N);
  add("n_contacts", O.P.n_contacts, 1, 1);
  add("swing_period", O.P.swing_period, 1, 1);
  add("swing_height", O.P.swing_height, 1, 1);
  add("swing_vel_limits", O.P.swing_vel_limits, 2, 1);
  add("Q_diag", O.P.Q_diag, O.ndx, 1);
  add("R_diag", O.P.R_diag, (O.P.base_vel_des - O.P.R_diag), 1);
  add("base_vel_des", O.P.base_vel_des, 6, 1);
  if (O.ext.valid) add("ext_force_des", O.P.ext_force_des, 3, 1);
  if (O.arm.valid) add("arm_vel_des", O.P.arm_vel_des, 3, 1);
  if (warm_start) add("x", -1, h.n, 1);
  if (PL_IS_RNEA(O.dyn)) {
    add("tau_prev", O.P.tau_prev, O.nj, 1);
    add("W_diag", O.P.W_diag, O.nj, 1);
  }
  c.sp_out = dense_sp(h.n, 1);
  c.p0.assign(o->h_params.begin(), o->h_params.begin() + h.np);
  c.x0.assign(h.n, 0.0);
  if (!warm_start) memcpy(c.x0.data(), x_initial, (size_t)h.n * 8);
  c.p.resize(h.np);
  c.x.resize(h.n);
  return 0;
}

void cas_forget_compiled(const pl_ocp* o) {
  PL_CAS_LOCK;
  if (g_cs.o == o) g_cs.o = nullptr;
}

static int cs_ready() {
  if (!g_cs.o) {
    pl_set_error("no OCP bound (pl_casadi_bind_compiled)");
    return 0;
  }
  return 1;
}

extern "C" int compiled_solver_alloc_mem(void) { return 0; }
extern "C" int compiled_solver_init_mem(int) { return 0; }
extern "C" void compiled_solver_free_mem(int) {}
extern "C" int compiled_solver_checkout(void) { return 0; }
extern "C" void compiled_solver_release(int) {}
extern "C" void compiled_solver_incref(void) {}
extern "C" void compiled_solver_decref(void) {}
extern "C" casadi_int compiled_solver_n_in(void) {
  PL_CAS_LOCK;
  return cs_ready() ? (casadi_int)g_cs.slots.size() : 0;
}
extern "C" casadi_int compiled_solver_n_out(void) { return 1; }
extern "C" double compiled_solver_default_in(casadi_int) { return 0.0; }
extern "C" int compiled_solver_work(casadi_int* sz_arg, casadi_int* sz_res, casadi_int* sz_iw, casadi_int* sz_w) {
  PL_CAS_LOCK;
  if (sz_arg) *sz_arg = cs_ready() ? (casadi_int)g_cs.slots.size() : 0;
  if (sz_res) *sz_res = 1;
  if (sz_iw) *sz_iw = 0;
  if (sz_w) *sz_w = 0;
  return 0;
}
extern "C" const char* compiled_solver_name_in(casadi_int i) {
  PL_CAS_LOCK;
  if (!cs_ready() || i < 0 || i >= (casadi_int)g_cs.names.size()) return nullptr;
  return g_cs.names[i].c_str();
}
extern "C" const char* compiled_solver_name_out(casadi_int i) { return i == 0 ? "x" : nullptr; }
extern "C" const casadi_int* compiled_solver_sparsity_in(casadi_int i) {
  PL_CAS_LOCK;
  if (!cs_ready() || i < 0 || i >= (casadi_int)g_cs.sp_in.size()) return nullptr;
  return g_cs.sp_in[i].data();
}
extern "C" const casadi_int* compiled_solver_sparsity_out(casadi_int i) {
  PL_CAS_LOCK;
  if (!cs_ready() || i != 0) return nullptr;
  return g_cs.sp_out.data();
}
extern "C" int compiled_solver(const double** arg, double** res, casadi_int*, double*, int) {
  PL_CAS_LOCK;
  if (!cs_ready()) return 1;
  CompiledState& c = g_cs;
  pl_ocp* o = c.o;
  c.p = c.p0;
  c.x = c.x0;
  for (size_t k = 0; k < c.slots.size(); ++k) {
    const CompiledSlot& s = c.slots[k];
    double* dst = s.off < 0 ? c.x.data() : c.p.data() + s.off;
    if (arg[k]) memcpy(dst, arg[k], (size_t)s.len * 8);
    else memset(dst, 0, (size_t)s.len * 8);  // CasADi passes null for an all-zero input
  }
  // as the reference's generated function: the objective's Hessian diagonal from these
  // parameters (ocp.py:293-296), x from the warm start, cold multipliers, one solve
  pl_stats st;
  if (pl_ocp_set_params(o, c.p.data()) || pl_ocp_init_solver(o) || pl_ocp_set_x(o, c.x.data()) ||
      pl_ocp_set_lam(o, nullptr) || pl_ocp_solve(o, &st, nullptr))
    return 1;
  if (res[0] && pl_ocp_get_x(o, res[0])) return 1;
  return 0;
}
