// TEST INFRASTRUCTURE: host build of the product's device math (rows.h / rbd.h /
// targets.h) so the CPU test suite can check the row function and its dual-number
// Jacobian against the numpy oracle without a GPU.  Not linked into the product.
#include <cstring>
#include "dyn.h"
#include "rows.h"
#include "targets.h"

namespace {
struct VEmit {
  double* g; double* l; double* u; int r;
  void operator()(double v, double lb, double ub) { g[r] = v; l[r] = lb; u[r] = ub; ++r; }
};
struct DEmit {
  double* t; int r;
  void operator()(const Dual& v, double, double) { t[r++] = v.d; }
};
template <int DYN>
int run(const PlModel& M, const PlOcpConst& O, int i, const double* p, const double* dx, const double* u,
        const double* dxn, int seed, double* g, double* lb, double* ub, double* tan) {
  if (seed < 0) {
    pl::VecIn<double> a{dx, nullptr, 0.0, -1}, b{u, nullptr, 0.0, -1}, c{dxn, nullptr, 0.0, -1};
    VEmit e{g, lb, ub, 0};
    double kst[PL_KIN_STORE];
    pl::node_rows<double, DYN>(M, O, i, p, a, b, c, e, kst, 1);
    return e.r;
  }
  const int ndx = O.ndx, nw = ndx + pl::node_nu(O, i);
  pl::VecIn<Dual> a{dx, nullptr, 0.0, seed}, b{u, nullptr, 0.0, seed - ndx}, c{dxn, nullptr, 0.0, seed - nw};
  DEmit e{tan, 0};
  Dual kst[PL_KIN_STORE];
  double aba_sh[PL_ABA_SH];
  if (DYN == PL_DYN_ABA) pl::aba_primal(M, O, p, dx, aba_sh);
  pl::node_rows<Dual, DYN>(M, O, i, p, a, b, c, e, kst, 1, nullptr, aba_sh);
  return e.r;
}
}  // namespace

extern "C" int th_node_rows(const void* model, const void* oc, int i, const double* p, const double* dx,
                            const double* u, const double* dxn, int seed, double* g, double* lb, double* ub,
                            double* tan) {
  PlModel M; PlOcpConst O;
  memcpy(&M, model, sizeof(M));
  memcpy(&O, oc, sizeof(O));
  switch (O.dyn) {
    case PL_DYN_RNEA: return run<PL_DYN_RNEA>(M, O, i, p, dx, u, dxn, seed, g, lb, ub, tan);
    case PL_DYN_ACC: return run<PL_DYN_ACC>(M, O, i, p, dx, u, dxn, seed, g, lb, ub, tan);
    case PL_DYN_CV: return run<PL_DYN_CV>(M, O, i, p, dx, u, dxn, seed, g, lb, ub, tan);
    case PL_DYN_CA: return run<PL_DYN_CA>(M, O, i, p, dx, u, dxn, seed, g, lb, ub, tan);
    case PL_DYN_ACCNB: return run<PL_DYN_ACCNB>(M, O, i, p, dx, u, dxn, seed, g, lb, ub, tan);
    case PL_DYN_CVNB: return run<PL_DYN_CVNB>(M, O, i, p, dx, u, dxn, seed, g, lb, ub, tan);
    case PL_DYN_RNEAFD: return run<PL_DYN_RNEAFD>(M, O, i, p, dx, u, dxn, seed, g, lb, ub, tan);
    default: return run<PL_DYN_ABA>(M, O, i, p, dx, u, dxn, seed, g, lb, ub, tan);
  }
}

extern "C" int th_dx_des(const void* model, const void* oc, const double* p, double* out) {
  PlModel M; PlOcpConst O;
  memcpy(&M, model, sizeof(M));
  memcpy(&O, oc, sizeof(O));
  pl::compute_dx_des(M, O, p, out);
  return 0;
}
