// Plain-data model and OCP descriptors shared by the C-ABI and the HIP kernels.
//
// PlModel mirrors the fields of pinocchio::Model that the reference's dynamics
// plugins read (dynamics/dynamics.py:13-21): joint tree (parents, placements,
// axes), spatial inertias, gravity.  The tree is additionally split into
// "chains" (maximal runs of single-child joints hanging off the free-flyer
// root), which is the shape of every robot the reference ships (4 legs, plus the
// Z1 arm on B2G) and lets the RNEA kernel keep one chain of state in registers.
#pragma once
#include <stdint.h>

#define PL_MAXJ 32      // joints incl. universe (B2G: 20)
#define PL_MAXQ 28
#define PL_MAXV 28
#define PL_MAXCHAIN 8
#define PL_MAXCL 6      // longest chain (Z1 arm: 6)
#define PL_MAXNJ 32     // actuated joints
#define PL_MAXFEET 4
#define PL_MAXNU 128
#define PL_JAC_SLOTS 3  // nodes per Jacobian wave (k_eval_jac shared-value slots; 4 would exceed 40 KB of LDS per wave)
#define PL_JAC_SLOTS_CH 12  // the same for the chain-confined columns of whole_body_rnea / _acc (no ABA slots)

enum { PL_JT_UNIVERSE = 0, PL_JT_FREEFLYER = 1, PL_JT_REVOLUTE = 2 };
enum { PL_AX_X = 0, PL_AX_Y = 1, PL_AX_Z = 2, PL_AX_GEN = 3 };

struct PlModel {
  int njoints;                 // including universe (index 0); joint 1 = free-flyer root
  int nq, nv;
  int parent[PL_MAXJ];
  int jtype[PL_MAXJ];
  int axis_kind[PL_MAXJ];
  int idx_q[PL_MAXJ];
  int idx_v[PL_MAXJ];
  double axis[PL_MAXJ][3];
  double jR[PL_MAXJ][9];       // jointPlacement rotation, row-major
  double jp[PL_MAXJ][3];
  double mass[PL_MAXJ];
  double lever[PL_MAXJ][3];
  double Ic[PL_MAXJ][9];       // rotational inertia at the CoM, row-major
  double gravity[3];
  double total_mass;
  int nchains;
  int chain_first[PL_MAXCHAIN];
  int chain_len[PL_MAXCHAIN];
};

struct PlFrameRef {
  int joint;                   // parent joint id
  int valid;
  double R[9];                 // placement w.r.t. the parent joint
  double p[3];
};

// Row-code dynamics kinds.  0-4 are also the public pl_ocp_desc codes (include_base
// true); PL_DYN_ACCNB is internal: whole_body_acc and centroidal_acc with
// include_base = False (u = [a_j | f], the base acceleration solved from the 6 base
// equations), which share their rows; PL_DYN_CVNB is internal too: centroidal_vel with
// include_base = False (u = [v_j | f], the base velocity v_b = A_b^-1 (m h - A_j v_j));
// PL_DYN_RNEAFD is whole_body_rnea with include_acc = False (u = [f | tau_j], the RNEA
// acceleration a_i = (v_{i+1} - v_i) / dt_i by finite difference, ocp_whole_body_rnea.py:183-191,
// no dv_{i+1} rows).
enum { PL_DYN_RNEA = 0, PL_DYN_ACC = 1, PL_DYN_ABA = 2, PL_DYN_CV = 3, PL_DYN_CA = 4, PL_DYN_ACCNB = 5,
       PL_DYN_CVNB = 6, PL_DYN_RNEAFD = 7 };
// centroidal_vel in either form: x = [h, q], dx = [dh, dq]
#define PL_IS_CV(d) ((d) == PL_DYN_CV || (d) == PL_DYN_CVNB)
// whole_body_rnea in either form: u = [a | f | tau_j] (tau_j on the first tau_nodes nodes), na = 0 for FD
#define PL_IS_RNEA(d) ((d) == PL_DYN_RNEA || (d) == PL_DYN_RNEAFD)

// Row-block kinds, emitted per node in the reference's subject_to order
// (optimization/ocp.py:103-190 + setup_dynamics_constraints of each subclass).
enum {
  PL_RB_INIT = 0,     // DX_0 == 0                                 (ocp.py:109)
  PL_RB_DYNQ,         // dq_{i+1} == dq_i + v_i dt                 (ocp_whole_body_rnea.py:155)
  PL_RB_DYNV,         // dv_{i+1} == dv_i + a_i dt  (a = ABA for aba) (:158 / ocp_whole_body_aba.py:106)
  PL_RB_RNEA_BASE,    // tau_rnea[:6] == 0                         (:162, acc gaps)
  PL_RB_TAU_EQ,       // tau_rnea[6:] == tau_j                     (:166)
  PL_RB_TAU_BND,      // -tau_max <= tau_j <= tau_max              (:171)
  PL_RB_FZ,           // c * f_z >= 0                              (ocp.py:131)
  PL_RB_CONE,         // c mu^2 f_z^2 >= c (f_x^2 + f_y^2)         (ocp.py:132)
  PL_RB_SWINGF,       // (1 - c) f == 0                            (ocp.py:135)
  PL_RB_FVXY,         // c v_xy == 0                               (ocp.py:145)
  PL_RB_FVZ,          // c v_z + (1 - c)(v_z - v_z,des) == 0        (ocp.py:157)
  PL_RB_EXT,          // f_ee == ext_force_des                     (ocp.py:168)
  PL_RB_ARM,          // v_ee,rel == arm_vel_des                   (ocp.py:180)
  PL_RB_QJ,           // pos_min <= q_j <= pos_max                 (ocp.py:189)
  PL_RB_VJ,           // -vel_max <= v_j <= vel_max                (ocp.py:190)
  PL_RB_CV_DYNH,      // dh_{i+1} == dh_i + h_dot(q, f) dt         (ocp_centroidal_vel.py:100)
  PL_RB_CV_DYNQ,      // dq_{i+1} == dq_i + v dt, v = u[:nv]       (ocp_centroidal_vel.py:101)
  PL_RB_CV_GAP,       // A(q) v - m h == 0                         (ocp_centroidal_vel.py:103-106)
  PL_RB_CA_GAP,       // A a + dA v - dh(q, f) == 0               (ocp_centroidal_acc.py:107-109)
  PL_RB_COUNT
};

struct PlRowBlock {
  int kind;
  int count;                   // rows in the block
  int arg;                     // foot index for per-foot blocks
  int pad;
};

// Parameter-vector offsets (Opti declaration order, ocp.py:54-69 and
// ocp_whole_body_rnea.py:88-89; 4xN matrices column-major).
struct PlParamLayout {
  int x_init, dt_min, dt_max, contact, swing, n_contacts, swing_period, swing_height, swing_vel_limits;
  int Q_diag, R_diag, base_vel_des, ext_force_des, arm_vel_des, tau_prev, W_diag;
  int np;
};

#define PL_MAXBLK 48

// Everything a node kernel needs that is identical for every problem of a batch.
struct PlOcpConst {
  int dyn;
  int N, nq, nv, nj, nf, nx, ndx;
  int na;                      // acceleration inputs (rnea/acc), 0 for aba
  int tau_nodes;
  int n;                       // decision variables
  int m;                       // constraint rows
  int nfeet;
  int nee;                     // frames receiving a contact force (feet + ext)
  double mu;
  PlFrameRef feet[PL_MAXFEET];
  PlFrameRef ext;
  PlFrameRef arm;
  PlFrameRef base;
  double q0[PL_MAXQ];
  double pos_min[PL_MAXNJ], pos_max[PL_MAXNJ], vel_max[PL_MAXNJ], tau_max[PL_MAXNJ];
  PlParamLayout P;
  // node-type specific row block lists: 0 = node 0, 1 = 0 < i < tau_nodes, 2 = otherwise
  int nblk[3];
  PlRowBlock blk[3][PL_MAXBLK];
  int rows_of_type[3];
};
