// Internal state of a batched OCP handle (not part of the C-ABI).
//
// Memory layout in HBM: every per-problem array is problem-major ([B][len]) so a
// workgroup that owns one problem streams contiguous memory; structure arrays
// (sparsity pattern, node tables) are shared by the whole batch and stay in L2.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "model.h"

#define PL_SIGMA_DEFAULT 1e-6

// Per-node structure, identical for every problem of the batch.
struct PlNode {
  int nw;          // variables owned by the node: dx_i + u_i (i < N) or dx_N
  int nu;
  int x_off;       // global column of dx_i
  int row_off;     // global row of the node's first row
  int nrow;        // rows of the node (node 0 includes the DX_0 == 0 rows)
  int ncol;        // local columns: nw + ndx (dx_{i+1}); 0 for node N
  int ent_off;     // first entry of the node in the entry arrays
  int nent;
  int colptr_off;  // into colptr (ncol + 1 values, relative to ent_off)
  int rowptr_off;  // into rowptr (nrow + 1 values, relative to the node's CSR list)
  int csr_off;     // into rowent
  int ntile;       // 4-row tile rows of the node's KKT block: T = ceil(nw / 4)
  int nunit;       // factor tile slots per lane: K = ceil(T (T + 1) / 2 / 64)
  int s_off;       // offset (doubles) of the node's factor block inside a problem's factor
  int cpl_off;     // coupling rows (rows with a dx_{i+1} entry): offset into cplrow
  int ncpl;
  int pad[2];
};

// Per-node tables of the factor and ADMM kernels.  Nodes with identical local
// structure share their programs (3-4 distinct programs per OCP).
//
// Factor program (k_factor.hip), u16 offsets relative to `fprog` in d.fprog:
//   f_rowptr[nrow+1], f_cplr[ncpl] (coupling rows = rows with a dx_{i+1} entry),
//   f_rowp[] = (entry, local col) pairs in CSR order;
//   coupling lists (same meaning as the ADMM program's cw / xc / cx):
//   f_cwptr[ncpl+1] f_cwp[] = (entry, col < nw), f_xcptr[ndx+1] f_xcp[] = (entry, coupling
//   index), f_cxptr[ncpl+1] f_cxp[] = (entry, dx_{i+1} col); flen = total u16 words.
// ADMM program (k_admm.hip), u16 offsets relative to `prog` in d.aprog; every
// distinct program is resident in LDS for the whole sweep kernel.  Pair lists hold
// (entry, index) as two consecutive u16 (one 32-bit read; their offsets are even):
//   rows (CSR over the node's rows):             rowe[] = entry (u16), rowc[] = local col (u8)
//   cols (CSC, entries in storage order):        colr[] = local row of each entry (u8)
//   w part of each coupling row s:               cwptr[ncpl+1], cwp[] = (entry, col)
//   dx_{i+1} part of each coupling row:          cxptr[ncpl+1], cxp[] = (entry, col - nw)
//   per column c < nw, entries in coupling rows: ccptr[nw+1],   ccp[] = (entry, coupling index)
//   per dx_{i+1} column c < ndx:                 xcptr[ndx+1],  xcp[] = (entry, coupling index)
//   row chunks (<= PL_CHUNK entries of one row): rchn chunks rch[] = (q0, q1) into rowe/rowc,
//                                                rchptr[nrow+1] = first chunk of each row
//   column chunks (<= PL_CHUNK entries):         cchn chunks cch[] = (e0, e1), cchptr[ncol+1]
//   owner of each chunk (u8):                    rchr[rchn] = local row, cchc[cchn] = local col
//
// Factor layout (k_factor writes, k_admm streams): the lower triangle of S_i in
// 4x4 tiles (I, J), J <= I < T, packed row-major t = I (I + 1) / 2 + J (diagonal
// tiles stored full).  Tile t belongs to lane l = t / K, slot k = t % K; its 16
// elements are 8 double2 (row r, cols 2h, 2h + 1 -> pair j = 2 r + h) stored at
// s_off + ((k * 8 + j) * 64 + l) * 2, so each 16-byte load of a wave is 1 KiB contiguous.
#define PL_CHUNK 6
// ADMM sweep kernel limits (one wave per problem, k_admm.hip)
#ifndef PL_ADMM_ATOMIC
#ifndef PL_IP_HESS_EXACT  // include/pinoloco.h (pl_ip_settings.hessian)
#define PL_IP_HESS_EXACT 0
#define PL_IP_HESS_GN 1
#endif
#define PL_ADMM_ATOMIC 1  // k_admm mat-vec: accumulate y with LDS f64 atomics (0: segment sums)
#endif
#define PL_ADMM_KM 4        // factor tile slots per lane held in registers (more: extra passes)
#define PL_ADMM_CWM 2       // w entries per coupling row held in registers (more: LDS path)
#define PL_ADMM_XCM 1       // coupling entries per dx_{i+1} column held in registers
#define PL_ADMM_MV 2        // columns per lane: nw <= 128
#define PL_ADMM_MR 3        // rows per lane: nrow <= 192
#define PL_ADMM_ASR_MAX 32  // A values per lane staged through registers (entries past 64 x ASR: global)
#define PL_ACPL (64 * (PL_ADMM_CWM + PL_ADMM_XCM))  // coupling A values per node (d.Acpl)
#define PL_RC_SYNC 32       // k_admm_rc hand-off words per problem (one 128-byte line)
struct PlAdmmNode {
  int nw, nrow, ncol, ncpl, nent, nunit, ntile, ntl;  // nunit = K slots, ntile = T, ntl = tiles
  unsigned kmagic;  // ceil(2^32 / K): t / K == umulhi(t, kmagic) for the tile counts used
  int x_off, row_off, ent_off, s_off;
  int prog, prog_len;
  int rowe, rowc, colr, cwptr, cwp, cxptr, cxp, ccptr, ccp, xcptr, xcp;
  int rchn, rch, rchptr, cchn, cch, cchptr, rchr, cchc;
  int fprog, flen, f_rowptr, f_cplr, f_rowp;
  int f_cwptr, f_cwp, f_xcptr, f_xcp, f_cxptr, f_cxp;  // coupling lists of the factor program
  int ttab;  // offset (u32) of the node's lane-tile table in d.ttab (-1: more than PL_ADMM_KM slots)
};

// Per-node table of the two-stage factor (k_factor.hip).  X = ndx, U = nu, w_i = [dx_i, u_i].
//   k_fnode  (parallel over problem x node): Kt_ii = diag(P) + sigma + sum_rows rho a a^T on w_i,
//            then C^-1 (u block), G = C^-1 B^T (U x X) and A' = A - B G (X x X), into d.FS;
//   k_fchain (one workgroup per problem, sequential over nodes): S_xx = (A' + E_i)^-1,
//            S_ux = -G S_xx, S_uu = C^-1 + G S_xx G^T, E_{i+1} = D - Kc S_i Kc^T.
// Assembly program: slot-owner streams over 256 threads, word [t][256] =
//   e1 | FLUSH << 15 | e2 << 16 (Kt slot += rho a_e1 * a_e2; e = nent is a zero entry),
//   flush slots (packed lower index) [f][256] in d.kfl.
// Coupling program (u32, at cp_off in d.kcpl), every dx_{i+1} column a owned by exactly
// one coupling row and every coupling row owning one dx_{i+1} column:
//   crow[X] local row, cent[X] its dx_{i+1} entry, cwptr[X+1], pcl[npc] (support columns
//   of the coupling rows' w parts), cw[] = e | p << 16 | pc << 24.
struct PlFacNode {
  int nw, nu, nrow, nent, ent_off, row_off, x_off, s_off, nunit, ntl;
  int asm_off, asm_len, fl_off, fl_len;
  int cp_off, npc;
  int nc;            // coupling rows (general coupling program, PlOcpHandle::fac_gc)
  long long fs_off;  // doubles: A' (X x X, full) | G (U x X) | C^-1 (U x U), row-major
};
#define PL_FAC_NT 256
#define PL_FAC_MAXGROUPS 16

struct PlSettings {
  double rho, sigma, alpha, eps_abs, eps_rel, eps_prim_inf, eps_dual_inf;
  int max_iter, scaling, check_termination, warm_start;
};

// Per-problem status/info written by the solver kernels.
struct PlProbInfo {
  int status;        // OSQP status code
  int iter;          // ADMM iterations run
  int done;          // ADMM terminated
  int ls_accepted;
  int ls_branch;
  int ls_trials;
  double ls_alpha;
  double pri_res, dua_res;
  double eps_pri, eps_dua;
  double f;          // objective at the returned point
  double viol_max;   // max bound violation at the returned point (ocp.py:412-414)
  double norm_dy, norm_dx;  // scratch for infeasibility checks
  long long iter_prof;      // ADMM iterations executed since pl_ocp_profile(o, 1) (roofline accounting)
};

// Interior-point solve (k_ip.hip, the Fatrop branch of the reference, ocp.py:248-263,
// 360-373): settings and per-problem state.  The filter holds at most one entry per
// iteration, so max_iter <= PL_IP_MAXFILT.
#define PL_IP_MAXFILT 32
struct PlIpSettings {
  double tol, mu_init, bound_push, bound_frac, delta_w, delta_c;
  int max_iter, ls_max, n_refine, pad;
  double warm_push;  // warm_start_mult_bound_push (1e-7, ocp.py:260)
};
struct PlIpInfo {
  double mu, theta_max, theta_min, err, f, alpha, alpha_z, viol_max;
  int iter, status, nfilt, trials, active, ref_solves;  // ref_solves: linear solves applied (k_ip_refine)
  double ref_last;                 // |correction|_inf of the last refinement solve (k_ip_refine)
  double filt[2 * PL_IP_MAXFILT];  // (theta, phi) pairs
  double alphas[PL_IP_MAXFILT];    // accepted step of each iteration
};

struct PlDev {
  // shared structure
  PlModel* model;
  PlOcpConst* oc;
  PlNode* nodes;     // N + 1
  int* colptr;
  int* rowidx;       // local row of each entry (CSC order)
  int* entcol;       // local column of each entry
  int* rowptr;
  int* rowent;       // CSR: entry index (local to the node) per row slot
  int* cplrow;       // coupling rows (local row ids)
  int* rownode;      // global row -> node
  int* colnode;      // global column -> node
  int* gr_ptr;       // global CSR of A: row r's (entry, column) pairs at gr_ec[gr_ptr[r] ..)
  int2* gr_ec;
  int* gc_ptr;       // global CSC of A: column j's (entry, row) pairs at gc_er[gc_ptr[j] ..)
  int2* gc_er;
  uint32_t* erc;         // (global row << 16 | global column) of each entry, for k_ruiz_fused (n, m < 65536)
  uint32_t* erl;         // (local row << 16 | local column) of each entry in its node (k_check_part)
  PlAdmmNode* anodes;    // N + 1 node tables (ADMM and factor programs)
  uint16_t* aprog;       // distinct ADMM programs, concatenated
  uint16_t* fprog;       // distinct factor programs, concatenated
  PlFacNode* fnodes;     // N + 1 (k_factor.hip)
  uint32_t* kasm;        // factor assembly streams
  uint16_t* kfl;         // factor flush slots
  uint32_t* kcpl;        // factor coupling programs
  double* FS;            // factor scratch [B][fs_stride]: A', G, C^-1 per node
  double* CH;            // reduced-chain blocks [B][ch_stride]: per node F_i^T | F_i | G_i (k_fred, k_admm_rc.hip)
  double* chv;           // reduced-chain vectors [B][chv_stride] (k_admm_rc)
  unsigned* rcsync;      // k_admm_rc hand-off words [B][PL_RC_SYNC]: fan-in count, fan-out epoch, give-up
                         // code (zeroed before every launch)
  uint32_t* ttab;        // lane-tile tables [64][PL_ADMM_KM] per distinct (T, K): (I << 24) | (J << 16) | cidx
  int2* jlist;           // k_eval_jac work list: (node, local column), tree-pass columns first (whole waves)
  int2* jlin;            // k_eval_jac_lin work list (rnea: the a / f columns, -1 padded to whole waves)
  // per problem [B][*]
  double* p;         // params
  double* x;         // SQP iterate (decision vector)
  double* x0;        // SQP iterate at the start of a solve (line search base)
  double* g;
  double* lbg;
  double* ubg;
  double* grad;
  double* Araw;      // constraint Jacobian values (nnz)
  double* P;         // Hessian diagonal (constant, ocp.py:293-296)
  double* As;        // scaled A
  double* qs;
  double* ls;
  double* us;
  double* rho;
  double* rhoc;      // rho of the coupling rows, [N+1][ncpl_max] per problem (ADMM prefetch)
  double* Acpl;      // scaled A of the coupling entries, [N+1][PL_ACPL] per problem, in the order the
                     // sweep's forward step gathers them (k_acpl: [s][PL_ADMM_CWM] | [c][PL_ADMM_XCM])
  double* D;
  double* E;
  double* cs;        // cost scaling c (1 per problem)
  double* Ps;        // scaled P diagonal
  double* xa;        // ADMM x (scaled, persistent warm start)
  double* za;
  double* ya;
  double* rhs;
  double* bt;
  double* dxs;       // delta x (check iterations)
  double* dys;       // delta y
  double* aty;       // A^T y scratch (check iterations)
  double* step;      // unscaled QP step dx
  double* S;         // factor blocks (tiled)
  double* work;      // generic reductions scratch
  double* chk;       // residual-norm partials [B][N+1][8] (k_check_part)
  PlProbInfo* info;
  // MPC (device loop)
  double* t0;        // per-problem gait time offset
  double* xstate;    // per-problem current state x_init (nx)
  double* dbg;       // optional kernel timing [B][16] (PL_ADMM_TIMING=1 at handle creation)
  // interior point [B][m] (allocated by pl_ocp_set_solver(o, PL_SOLVER_IP))
  double* ip_s;      // slacks of the inequality rows
  double* ip_lam;    // constraint multipliers (lam_g)
  double* ip_lam0;   // lam_g warm start (opti.set_initial(opti.lam_g, lam_g), ocp_whole_body_rnea.py:234-235)
  // exact Lagrangian Hessian (k_hess.hip) and its inertia correction (k_ip.hip)
  int* hnz;          // per node type: the written entries (row | col << 16) of a Lagrangian Hessian block
  const PlIpInfo* ipskip;  // set only inside an interior-point solve (enqueue_ip): the evaluation and
                           // factor kernels skip the problems that have terminated (active == 0)
  int2* hlist;       // (node, j | k << 16) column pairs of the w_i blocks
  int2* hcone;       // whole_body_rnea / whole_body_acc: (node, foot-force column) of the cone curvature (k_lag_hess_cone)
  int2* htrf;        // the (dq, external force) pairs (k_lag_hess_tree<true>)
  int2* htr;         // whole_body_rnea / whole_body_acc: the (dq, dq) and (dq, dv) pairs (k_lag_hess_tree)
  int2* harm;        // the pairs of d.htr on the base or the arm's chain (k_lag_hess_arm)
  int4* hcol;        // the same pairs as forward-over-reverse columns (k_lag_hess_col): (node | (chain + 1) << 16,
                     // column j, mask of the other coordinates (hess_tree.h col_coord), 0)
  int2* hvv;         // whole_body_rnea / whole_body_acc: the (dv, dv) pairs, packed as hlist (k_lag_hess_vv)
  int2* hlin;        // whole_body_rnea: (node, dq column k) of the linear-column Hessian blocks (k_lag_hess_lin)
  PlModel* model0;   // the model with zero gravity (M(q) lambda by an RNEA pass at v = 0)
  int* hoff;         // packed-lower offset of node i's block
  double* Hlag;      // [B][hl_stride] sum_r lam_r d^2 g_r / dw_i^2, packed lower per node
  double* ip_dwi;    // [B][2]: the inertia shift of this Newton system, the last nonzero one
  int* ip_act;       // [B + 2]: the active problems of the current IP iteration, compacted (k_ip_compact);
                     // ip_act[B] = their count, ip_act[B + 1] = the lanes of the Hessian waves launched
                     // since pl_ocp_profile(1) (the IP line's flop scaling)
  int* ip_iflag;     // [B][4]: not-SPD seen by the factor, refactor, resolved, tries
  double* ip_zl;     // lower / upper bound multipliers of the slacks
  double* ip_zu;
  double* ip_rh;     // r^ of the reduced Newton system
  double* ip_dl;     // Newton direction: multipliers, slacks
  double* ip_ds;
  double* ip_dx;     // Newton step dx [B][n] and J dx [B][m], accumulated over the refinement solves
  double* ip_jdx;
  PlIpInfo* ipinfo;  // [B]
};

// an interior-point solve's terminated problem (PlDev::ipskip): nothing downstream reads its
// evaluation or factor any more
__device__ inline bool ip_skip(const PlDev& d, int b) { return d.ipskip && !d.ipskip[b].active; }


struct PlOcpHandle {
  int device;
  hipStream_t stream;
  int B;
  int N, n, m, np, nnz, nx, ndx, nw_max, ncol_max, nrow_max, S_stride;
  int nunit_max;                    // max factor tile slots per lane (K)
  int ntile_max;                    // max 4-row tile rows (T)
  int ncpl_max, nent_max;
  int chunk_max;                    // max(rchn, cchn) over nodes (ADMM partial-sum buffer)
  int flen_max;                     // longest factor program (u16)
  int aprog_len;                    // all ADMM programs (u16), resident in LDS
  int prog_len_max;                 // longest single ADMM program (u16)
  int admm_asr;                     // A values per lane staged through registers (x 64 lanes)
  int admm_fwd_asb;                 // coupling rows too dense for registers: forward steps stage A in LDS
  int sqp_iters;                    // SQP iterations per solve (reference: 1, ocp.py:382-383)
  int admm_waves;                   // ADMM sweep kernel: 2 = k_admm2 (two waves per problem), 1 = k_admm
  int ruiz_fused;                   // 1: all equilibration passes in k_ruiz_fused (PL_PATH_RUIZ_PER_PASS: per-pass kernels)
  unsigned debug_paths;             // pl_ocp_desc.debug_paths (PL_PATH_*), 0 in production
  int admm_rc;                      // 1: reduced-chain ADMM (k_admm_rc.hip) instead of the sweeps
  int rc_waves;                     // waves per workgroup of k_admm_rc (4 or 8)
  int num_cu;                       // compute units of the device (k_admm_rc's co-residency bound)
  long long ch_stride;              // doubles of chain blocks per problem
  int chv_stride;                   // doubles of chain vectors per problem
  int jl_len;                       // k_eval_jac work-list entries (a multiple of 64 before the cheap part)
  int jl_ex;                        // jlist entries before the cheap columns
  int jac_cheap_every;              // PL_PATH_JAC_CONST_EVERY: evaluate them every time (the r03 path)
  int jlin_len;                     // k_eval_jac_lin work-list entries (0: those columns stay in jlist)
  int solver;                       // PL_SOLVER_OSQP (SQP + OSQP ADMM) or PL_SOLVER_IP (interior point)
  int ip_lam_warm;                  // 1: the next interior-point solve starts from lam = ip_lam0
  int ip_mpc_lam;                   // pl_mpc_step with the IP solver: 1 carries lam_g to the next step
                                    // (the Opti branch), 0 cold multipliers (the compiled-solver branch)
  int ip_hess;                      // interior point: PL_IP_HESS_EXACT (Lagrangian) or PL_IP_HESS_GN
  int hl_len;                       // Lagrangian Hessian work list (k_lag_hess)
  int hnz_off[4];                   // d.hnz per node type: [hnz_off[t], hnz_off[t + 1])
  int hcone_len;                    // k_lag_hess_cone work list
  int htrf_len;                     // k_lag_hess_tree<true> work list
  int htr_len;                      // k_lag_hess_tree work list
  int hcol_len;                     // k_lag_hess_col work list (0: the pair kernel runs)
  int harm_len;                     // k_lag_hess_arm work list
  int hcol_nbase;                   // its first hcol_nbase items are the whole-tree base columns
  int hvv_len;                      // k_lag_hess_vv work list
  int hlin_len;                     // k_lag_hess_lin work list (0: every pair by hyper-dual passes)
  int hl_rb_base[3], hl_rb_tau[3];  // per node type: first row of the RNEA base / joint-torque rows (-1: none)
  long long hl_stride;              // doubles per problem of d.Hlag
  int fac_hlag;                     // 1: k_fnode adds d.Hlag to Kt_ii and both factor kernels report pivots <= 0
  int fac_only;                     // 1: the factor kernels skip problems whose d.ip_iflag refactor flag is clear
  PlIpSettings ip;
  long long fs_stride;              // factor scratch per problem (doubles)
  int nfgroup;                      // k_fnode launches: consecutive nodes with one program
  int fg_i0[PL_FAC_MAXGROUPS], fg_n[PL_FAC_MAXGROUPS], fg_lds[PL_FAC_MAXGROUPS], fg_um[PL_FAC_MAXGROUPS];
  int fchain_lds;                   // k_fchain LDS bytes
  int fchain_ny, fchain_ncw;        // k_fchain Y buffer and staged coupling values (doubles)
  int fac_gc;                       // 1: general coupling (rows of node i touch several dx_{i+1} columns:
                                    //    whole_body_rnea include_acc = False), E_{i+1} = Wc^T Z Wc in k_fchain
  int fchain_nc, fchain_nxc;        // general coupling: max coupling rows, max dx_{i+1} entries per node
  int fchain_short;                 // k_fchain's E: 1 short coupling lists (straight from S), 2 MFMA, 0 lists via Y
  PlSettings set;
  PlModel model;
  PlOcpConst oc;
  int gait_type;     // 0 trot, 1 walk, 2 stand
  double gait_period, swing_period;
  double f_des[PL_MAXNU];
  PlDev d;
  // host copies of the structure
  int* h_nodes_raw;
  // optional per-kernel timing of the ADMM launches (HIP events on the handle's stream)
  int profile;
  // outside the MPC-graph key (api.hip kMpcKeyBytes): set by the first Jacobian evaluation,
  // which runs eagerly; a debug write of Araw clears it and the key
  int jac_cheap_ok;                 // the cheap columns' constant entries are in d.Araw
  hipEvent_t prof_ev[64][2];
  int prof_n;
  double prof_admm_ms;
  long long prof_admm_launches;
  long long prof_admm_iters;   // problem-iterations executed by the timed launches (sum of PlProbInfo::iter_prof)
  hipEvent_t prof_hev[16][2];  // the same for the interior point's Lagrangian-Hessian launches (k_lag_hess)
  int prof_hn;
  double prof_hess_ms;
  long long prof_hess_launches;
};

// ---- kernel launchers (defined in the k_*.hip translation units)
void launch_eval_values(PlOcpHandle* h, const double* xsrc);
void launch_eval_jac(PlOcpHandle* h);
void launch_objective(PlOcpHandle* h);
void launch_hess(PlOcpHandle* h);
void launch_qp_setup(PlOcpHandle* h);
void launch_factor(PlOcpHandle* h);
void launch_factor_pre(PlOcpHandle* h);   // launch_factor = pre + core + post
void launch_factor_core(PlOcpHandle* h);
void launch_factor_post(PlOcpHandle* h);
bool factor_supports_ndx(int ndx);
void launch_admm_init(PlOcpHandle* h);
void launch_admm(PlOcpHandle* h, int niter, int check, int it_base);
bool admm2_supported(const PlOcpHandle* h);
void launch_admm2(PlOcpHandle* h, int niter, int check);
bool admm_rc_supported(const PlOcpHandle* h);
void launch_admm_rc(PlOcpHandle* h, int niter, int check);
void launch_lag_hess(PlOcpHandle* h);
void launch_fred(PlOcpHandle* h);
void launch_acpl(PlOcpHandle* h);
long long rc_ch_stride(int N, int ndx, int W);
int rc_chv_stride(int N, int ndx);
int rc_groups(const PlOcpHandle* h);
void launch_check(PlOcpHandle* h, int it, int final_check);
void launch_unscale(PlOcpHandle* h);
void launch_line_search(PlOcpHandle* h);
void launch_mpc_prepare(PlOcpHandle* h, int k);
void launch_mpc_finish(PlOcpHandle* h);
void launch_reset_info(PlOcpHandle* h);
void launch_reset_iterates(PlOcpHandle* h);
void launch_reset_prof(PlOcpHandle* h);
void enqueue_ip(PlOcpHandle* h);
void enqueue_ip_direction(PlOcpHandle* h);

#define PL_CHECK_HIP(expr)                                                        \
  do {                                                                            \
    hipError_t _e = (expr);                                                       \
    if (_e != hipSuccess) {                                                       \
      pl_set_error("%s:%d %s -> %s", __FILE__, __LINE__, #expr, hipGetErrorString(_e)); \
      return -2;                                                                  \
    }                                                                             \
  } while (0)

void pl_set_error(const char* fmt, ...);
