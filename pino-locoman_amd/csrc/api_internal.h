// Host-side internals of the C-ABI shared by api.hip (handles, solve and MPC sequencing,
// profiling, debug access), api_build.hip (the layout / program builders) and
// api_casadi.hip (the CasADi external-function ABI).
#pragma once
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
  int mpc_graph_off = 0;               // 1: capture failed or PL_PATH_NO_MPC_GRAPH: launch eagerly
  long long mpc_captures = 0;
  long long mpc_replays = 0;           // graph launches (pl_mpc_graph_info)
  void* dl_host = nullptr;             // pinned staging of pl_mpc_download
  size_t dl_bytes = 0;
};

template <class T>
inline int dalloc(pl_ocp* o, T** p, size_t count) {
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

template <class T>
inline int upload(pl_ocp* o, T** p, const std::vector<T>& v) {
  if (dalloc(o, p, v.size())) return -2;
  if (!v.empty()) PL_CHECK_HIP(hipMemcpy(*p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  return 0;
}

// api_build.hip: variable / row / sparsity layout and the device programs of one OCP
void build_blocks(PlOcpConst& O, bool has_ext, bool has_arm);
int build_layout(pl_ocp* o);
int build_admm_prog(pl_ocp* o);
int build_factor_prog(pl_ocp* o);
// lin (use_lin, rnea): the a / f columns, for k_eval_jac_lin, instead of tree-pass lanes in list
// n_ex: entries of list before the cheap columns (whole waves)
int build_jac_list(pl_ocp* o, std::vector<int2>& list, std::vector<int2>& lin, bool use_lin, int* n_ex);
// api_casadi.hip: drop the CasADi binding of an OCP that is being destroyed
void cas_forget(const pl_ocp* o);
void jac_pattern(const PlOcpHandle& h, const std::vector<PlNode>& nodes, int i, std::vector<uint8_t>& nz);
