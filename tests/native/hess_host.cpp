// TEST INFRASTRUCTURE: host build of the Lagrangian-Hessian tree sweeps (csrc/hess_tree.h) so the
// CPU suite can check the forward-over-reverse columns (tree_col, r06) against the hyper-dual pair
// sweeps (tree_pair, r05) entry by entry without a GPU.  Not linked into the product.
#include <cstring>
#include "hess_tree.h"

extern "C" double th_hess_pair(const void* model, const void* oc, int i, int only_ch, int j, int k, const double* x,
                               const double* p, const double* lam) {
  PlModel M; PlOcpConst O;
  memcpy(&M, model, sizeof(M));
  memcpy(&O, oc, sizeof(O));
  return hess::tree_pair<false>(M, O, i, only_ch, j, k, x, p, lam);
}

// out[k] for every dx index k the column writes (others untouched)
extern "C" void th_hess_col(const void* model, const void* oc, int i, int only_ch, int j, unsigned mask,
                            const double* x, const double* p, const double* lam, double* out) {
  PlModel M; PlOcpConst O;
  memcpy(&M, model, sizeof(M));
  memcpy(&O, oc, sizeof(O));
  if (only_ch < 0) hess::tree_col<true>(M, O, i, only_ch, j, mask, x, p, lam, [&](int k, double v) { out[k] = v; });
  else hess::tree_col<false>(M, O, i, only_ch, j, mask, x, p, lam, [&](int k, double v) { out[k] = v; });
}

extern "C" int th_col_coord(const void* model, const void* oc, int only_ch, int loc) {
  PlModel M; PlOcpConst O;
  memcpy(&M, model, sizeof(M));
  memcpy(&O, oc, sizeof(O));
  return hess::col_coord(M, O, only_ch, loc);
}

extern "C" int th_chain_len(const void* model, int ch) {
  PlModel M;
  memcpy(&M, model, sizeof(M));
  return ch < 0 ? -1 : M.chain_len[ch];
}
extern "C" int th_nchains(const void* model) {
  PlModel M;
  memcpy(&M, model, sizeof(M));
  return M.nchains;
}
