/*
 * pinoloco -- C-ABI of the MI355X-native batched MPC inner loop.
 *
 * Drop-in boundary for the reference's OSQP-SQP solve path
 * (lukasmolnar/pino-locoman @ 2025-05-09).  Each entry point replaces a
 * reference interface, cited as file:line of the reference:
 *
 *   pl_model_create       <- RobotWrapper.BuildFromURDF + buildReducedRobot
 *                            (utils/robot.py:13-22); the host parser
 *                            pinoloco/model.py produces the tables.
 *   pl_ocp_create         <- make_ocp(dynamics, OCP_ARGS, robot, nodes, solver)
 *                            (optimization/ocp_factory.py:8-27) + setup_problem
 *                            (optimization/ocp.py:38-44): variable/row layout and
 *                            the Jacobian sparsity of J_g (ocp.py:283, 305).
 *   pl_ocp_set_params     <- opti.set_value(...) of every parameter
 *                            (ocp.py:216-242, ocp_whole_body_rnea.py:204); the
 *                            array is opti.p in declaration order (ocp.py:54-69).
 *   pl_ocp_set_x          <- opti.set_initial(...) / warm_start()
 *                            (ocp.py:161-163, ocp_whole_body_rnea.py:207-235).
 *   pl_ocp_init_solver    <- OCP.init_solver() OSQP branch (ocp.py:265-313):
 *                            constant Hessian diagonal, OSQP setup.
 *   pl_ocp_solve          <- OCP.solve() OSQP branch minus retract
 *                            (ocp.py:375-414): sqp_data, osqp.update/solve,
 *                            _armijo_line_search, max violation.
 *   pl_eval_sqp_data      <- the CasADi Function sqp_data(x, p) ->
 *                            (grad_f, J_g, g, lbg, ubg) (ocp.py:287, 386).
 *   pl_eval_f             <- f_data (ocp.py:289); g_data is the g/lbg/ubg part
 *                            of pl_eval_sqp_data (ocp.py:290).
 *   pl_mpc_*              <- run_mpc.mpc_loop OSQP branch (run_mpc.py:115-143)
 *                            executed on the device for a whole batch.
 *
 * Conventions: all host arrays are caller-owned, C-contiguous float64,
 * problem-major ([batch][len]).  The library copies them into device buffers
 * it owns.  Functions return 0 on success and a negative value on error; the
 * message is available from pl_last_error() (thread-local).  Per-problem
 * solver failures are reported in pl_stats.status, never as a call failure.
 * A handle is bound to one HIP device and stream and is not thread-safe.
 * Calls are synchronous with respect to host buffers on return.
 */
#ifndef PINOLOCO_H_
#define PINOLOCO_H_

#ifdef __cplusplus
extern "C" {
#endif

typedef struct pl_model pl_model;
typedef struct pl_ocp pl_ocp;

/* Joint types (JointModelFreeFlyer root + revolute joints, utils/robot.py:14). */
#define PL_JOINT_FREEFLYER 1
#define PL_JOINT_REVOLUTE 2

/* Dynamics kinds (ocp_factory.py:9-15). */
#define PL_DYN_WHOLE_BODY_RNEA 0
#define PL_DYN_WHOLE_BODY_ACC 1
#define PL_DYN_WHOLE_BODY_ABA 2
#define PL_DYN_CENTROIDAL_VEL 3      /* x = [h (6), q], dx = [dh, dq], u = [v | f] */
#define PL_DYN_CENTROIDAL_ACC 4      /* x = [q, v], u = [a | f] (include_base) or [a_j | f] */

typedef struct {
  int njoints;                 /* including the universe joint 0 */
  int nq, nv;
  const int* parent;           /* [njoints] */
  const int* jtype;            /* [njoints] PL_JOINT_* (0 for universe) */
  const double* axis;          /* [njoints*3] revolute axis in the joint frame */
  const double* placement_R;   /* [njoints*9] jointPlacement rotation (row-major) */
  const double* placement_p;   /* [njoints*3] */
  const double* mass;          /* [njoints] body inertias (fixed children merged) */
  const double* lever;         /* [njoints*3] CoM in the joint frame */
  const double* inertia;       /* [njoints*9] rotational inertia at the CoM */
  const double* gravity;       /* [3] */
  int nframes;
  const int* frame_parent;     /* [nframes] parent joint */
  const double* frame_R;       /* [nframes*9] placement w.r.t. the parent joint */
  const double* frame_p;       /* [nframes*3] */
} pl_model_desc;

typedef struct {
  int dynamics;                /* PL_DYN_* */
  int nodes;                   /* N */
  int tau_nodes;               /* OCP_ARGS["whole_body_rnea"]["tau_nodes"] (ocp_args.py:16) */
  int include_acc;             /* rnea: 1 = a in u (ocp_args.py:17), 0 = a = (v_{i+1} - v_i) / dt (ocp_whole_body_rnea.py:183-191; OSQP branch only) */
  int include_base;            /* acc / centroidal_acc / centroidal_vel: 1 = base in u (ocp_args.py:5-11);
                                  0 = base acceleration / velocity from the dynamics
                                  (ocp_whole_body_acc.py:124-135, ocp_centroidal_vel.py:119-129) */
  int n_feet;                  /* 4: FR, FL, RR, RL (utils/gait_sequence.py:7) */
  int foot_frames[4];
  int ext_force_frame;         /* -1: none */
  int arm_ee_frame;            /* -1: none */
  int base_frame;              /* "base_link" frame, -1 if absent (dynamics/dynamics.py:17) */
  double mu;                   /* friction coefficient 0.7 (ocp.py:103) */
  const double* q0;            /* [nq] reference pose (SRDF) */
  const double* joint_pos_min; /* [nj] */
  const double* joint_pos_max;
  const double* joint_vel_max;
  const double* joint_torque_max;
  /* OSQP settings (ocp.py:267-273 + OSQP 0.6 defaults) */
  double rho, sigma, alpha, eps_abs, eps_rel, eps_prim_inf, eps_dual_inf;
  int max_iter, scaling, check_termination, warm_start;
  /* gait used by the device-side MPC loop (utils/gait_sequence.py:5-24) */
  int gait_type;               /* 0 trot, 1 walk, 2 stand */
  double gait_period;
  /* 0 in production.  Bits of PL_PATH_*: the paths earlier builds used, kept as the references
     the regression tests compare the current kernels with (tests/test_r04_paths.py,
     tests/test_qp_kernels.py, tests/test_graph_gpu.py), and the phase-timing instrumentation.
     No environment variable changes a kernel path; pl_ocp_sizes reports this field.
     Callers must zero-initialise the struct: pl_ocp_create rejects bits outside PL_PATH_ALL. */
  unsigned debug_paths;
} pl_ocp_desc;

#define PL_PATH_JAC_DUAL_ALL    1u   /* rnea a / f Jacobian columns as dual lanes (not k_eval_jac_lin) */
#define PL_PATH_JAC_CONST_EVERY 2u   /* the constant Jacobian columns re-evaluated every time */
#define PL_PATH_HESS_FULL_TREE  4u   /* Lagrangian-Hessian passes over the whole tree (no chain confinement) */
#define PL_PATH_HESS_DUAL_ALL   8u   /* the (dq, a) / (dq, f) Hessian blocks as hyper-dual pairs */
#define PL_PATH_FCHAIN_LIST     16u  /* the factor chain's E_{i+1} by list sums (not the f64 MFMA) */
#define PL_PATH_RUIZ_PER_PASS   32u  /* Ruiz equilibration as per-pass kernels (not k_ruiz_fused) */
#define PL_PATH_NO_MPC_GRAPH    64u  /* pl_mpc_step launches eagerly (no HIP graph) */
#define PL_PATH_ADMM_TIMING     128u /* s_memtime phase timing in the sweep / factor kernels (pl_debug_get "admm_t") */
#define PL_PATH_IP_REFINE_GATHER 256u /* k_ip_refine's H_i dx by the per-column global gather (the nw > 192 path) */
#define PL_PATH_HESS_PAIRS      512u /* the (dq, dq) / (dq, dv) Hessian pairs by one hyper-dual sweep each (r05), not
                                        the forward-over-reverse columns */
#define PL_PATH_RC_ONE_GROUP    1024u /* the chain ADMM kernel on one workgroup per problem (r05), not the
                                         multi-workgroup node phases */
#define PL_PATH_ALL             2047u /* pl_ocp_create rejects any other bit: callers zero the struct */

typedef struct {
  int status;                  /* OSQP status code (1 solved, 2 inaccurate, -2 max iter, ...) */
  int admm_iters;
  int ls_accepted;             /* line search accepted a step (ocp.py:473-480) */
  int ls_branch;               /* 1: g high & improving, 2: armijo, 3: filter */
  int ls_trials;
  int pad;
  double ls_alpha;             /* accepted step length (a / a_decay, ocp.py:475) */
  double viol_max;             /* _constraint_violation_max after the step (ocp.py:412-414) */
  double pri_res, dua_res;
  double f;                    /* objective at the returned point */
} pl_stats;

const char* pl_last_error(void);
int pl_version(void);
/* "pl_src_sha256=<hex> arch=gfx950": the sha256 of the csrc/ and include/ sources this
   library was built from (pinoloco/build.py source_sha). */
const char* pl_build_info(void);

int pl_model_create(const pl_model_desc* desc, pl_model** out);
void pl_model_destroy(pl_model* m);

/* device = -1 builds a host-only handle (layout/pattern queries, no solves). */
int pl_ocp_create(const pl_model* model, const pl_ocp_desc* desc, int batch, int device, pl_ocp** out);
void pl_ocp_destroy(pl_ocp* o);

/* n decision variables, m rows, np parameters, nnz Jacobian entries. */
int pl_ocp_dims(const pl_ocp* o, int* n, int* m, int* np, int* nnz);
/* Jacobian pattern in the library's entry order: global (row, col) per entry. */
int pl_ocp_pattern(const pl_ocp* o, int* rows, int* cols);

int pl_ocp_set_params(pl_ocp* o, const double* P);   /* [batch][np] */
int pl_ocp_get_params(pl_ocp* o, double* P);
int pl_ocp_set_x(pl_ocp* o, const double* X);        /* [batch][n] */
int pl_ocp_get_x(pl_ocp* o, double* X);
int pl_ocp_init_solver(pl_ocp* o);                   /* Hessian diag + reset ADMM iterates */
/* One SQP iteration in place for the whole batch.  stats: [batch] or NULL;
 * phase_ms: [4] (data, update+factor, admm, line search) or NULL. */
int pl_ocp_solve(pl_ocp* o, pl_stats* stats, double* phase_ms);
/* SQP iterations per pl_ocp_solve / pl_mpc_step (default 1 = the reference's
 * `for _ in range(1)`, optimization/ocp.py:382-383). */
int pl_ocp_set_sqp_iters(pl_ocp* o, int sqp_iters);

/* Interior-point solve: the reference's Fatrop branch (ocp.py:248-263 settings,
 * :360-373 solve; run_mpc.py:34-37 selects it), restated as an IPOPT-style
 * primal-dual barrier method with a filter line search (oracle/ip_ref.py documents
 * the algorithm).  pl_ocp_set_solver(o, PL_SOLVER_IP) switches pl_ocp_solve and
 * pl_mpc_step to it; pl_stats then holds status (1 converged, -1 max_iter, -2 line
 * search failed, -3 non-finite), admm_iters = IP iterations, ls_trials (total),
 * ls_alpha (last step), viol_max, pri_res = scaled NLP error, dua_res = mu, f. */
#define PL_SOLVER_OSQP 0
#define PL_SOLVER_IP 1
typedef struct {
  double tol;          /* 1e-3  (ocp.py:257) */
  double mu_init;      /* 1e-4  (ocp.py:258) */
  double bound_push;   /* 1e-7  (ocp.py:261) */
  double bound_frac;   /* 1e-2 */
  double delta_w;      /* 1e-8  primal regularisation of the Newton system */
  double delta_c;      /* 1e-4  dual regularisation (equality rows weighted 1 / delta_c) */
  int max_iter;        /* 10    (ocp.py:256), at most 32 */
  int ls_max;          /* 12    line-search trials */
  int n_refine;        /* 8     most iterative-refinement solves of each Newton system (the Lagrangian
                          Hessian makes the reduced systems stiffer: B2G rnea needs ~6 to
                          reach the sparse LU's direction to 1e-9 with the block inverses); a
                          problem stops refining once a correction is below 1e-12 |dx|_inf or
                          more than 0.9 of the previous one (stagnation); a correction larger
                          than the previous one is not applied and ends the refinement */
  int hessian;         /* PL_IP_HESS_EXACT: the Lagrangian Hessian of f + lam^T g (CasADi's
                          exact Hessian of the Opti/Fatrop solve, ocp.py:248-263) with the
                          inertia correction; PL_IP_HESS_GN: the objective's diagonal only */
} pl_ip_settings;
#define PL_IP_HESS_EXACT 0
#define PL_IP_HESS_GN 1
typedef struct {
  int status, iter, ls_trials, nfilter;
  double err, mu, alpha, alpha_z, f, viol_max;
  double alphas[32];   /* accepted step of each iteration (0: failed line search) */
  int ref_solves;      /* linear solves of the Newton systems of this solve (first solve + the
                          refinement corrections applied), summed over its iterations */
  int pad;
} pl_ip_stats;
int pl_ocp_set_solver(pl_ocp* o, int solver);
int pl_ocp_set_ip_settings(pl_ocp* o, const pl_ip_settings* s);
int pl_ocp_ip_stats(pl_ocp* o, pl_ip_stats* stats);   /* [batch] */
int pl_ocp_get_lam(pl_ocp* o, double* lam);           /* [batch][m]: lam_g (ocp.py:373) */
/* [batch][m] lam_g warm start of the next interior-point solves (the OCPs' warm_start:
 * opti.set_initial(opti.lam_g, lam_g), ocp_whole_body_rnea.py:234-235); NULL = cold
 * (lam = 0, the reference's first solve).  pl_mpc_step carries lam_g itself. */
int pl_ocp_set_lam(pl_ocp* o, const double* lam);
/* Parity aid: the interior point's Newton direction from a given state (x set with
 * pl_ocp_set_x; slacks, multipliers [batch][m], mu [batch]); read it back with
 * pl_debug_get("ip_dx" / "ip_dl" / "ip_ds") and the step bounds with pl_ocp_ip_stats
 * (alpha = primal, alpha_z = bound-multiplier fraction-to-boundary step). */
int pl_debug_ip_direction(pl_ocp* o, const double* s, const double* lam, const double* zl, const double* zu,
                          const double* mu);

/* CasADi external-function ABI (include/pinoloco_casadi.h): bind the OCP whose
 * shapes / sparsity the exported sqp_data, f_data, g_data, hess_data and
 * retract_solution describe (replaces the generated code of ocp.py:299-302 and
 * ocp_whole_body_rnea.py:326-366; retract_steps = num_steps of compile_solution). */
int pl_casadi_bind(pl_ocp* o, int retract_steps);
void pl_casadi_unbind(void);
/* Bind the batch-1 interior-point handle (pl_ocp_set_solver(o, PL_SOLVER_IP)) whose Fatrop
 * solve the exported compiled_solver runs (include/pinoloco_casadi.h; replaces the generated
 * opti.to_function("compiled_solver", ...) of ocp_whole_body_rnea.py:237-258 / ocp.py:324-342,
 * loaded by run_mpc.py:51-53).  warm_start = the compile_solver argument (x_warm_start is then
 * an input); x_initial [n]: the initial guess baked in without it (may be NULL with it).  The
 * parameters the function does not take keep the handle's values at bind time. */
int pl_casadi_bind_compiled(pl_ocp* o, int warm_start, const double* x_initial);
/* Evaluate sqp_data at the current x: any output may be NULL. */
int pl_eval_sqp_data(pl_ocp* o, double* grad, double* Jvals, double* g, double* lbg, double* ubg);
/* f_data value at the current x. */
int pl_eval_f(pl_ocp* o, double* f);
/* Scaled-QP diagnostics after a solve: step dx [batch][n] (unscaled OSQP solution). */
int pl_ocp_get_step(pl_ocp* o, double* dx);

/* Device-side MPC loop (run_mpc.py:127-143) for the whole batch:
 * x_state [batch][nx] = x_init, t0 [batch] = gait time offset. */
int pl_mpc_setup(pl_ocp* o, const double* x_state, const double* t0);
/* One MPC step k: gait schedule at t0 + k*dt_min, x_init, warm start, solve,
 * x_state <- integrate(x_state, DX[1]).  No host transfers.  With the OSQP solver and
 * profiling off, the launches after the gait / warm-start kernel are replayed from a HIP
 * graph captured on the second step with unchanged handle settings (bit-identical to
 * launching them; PL_MPC_GRAPH=0 at creation launches them one by one). */
int pl_mpc_step(pl_ocp* o, int k);
int pl_mpc_get_state(pl_ocp* o, double* x_state);
/* Solver stats of the last MPC step's (last) SQP iteration, as pl_ocp_solve reports. */
int pl_mpc_get_stats(pl_ocp* o, pl_stats* stats);
/* Copy the first control input row u_0 [batch][nu_0] and x_state into a
 * caller-owned DEVICE buffer (for collectives): layout [batch][nu_0 + nx]. */
int pl_mpc_export(pl_ocp* o, void* device_dst);
/* The same rows [batch][nu_0 + nx] into caller-owned HOST memory, through a pinned staging
 * buffer of the handle; returns after the copy landed (the per-step controller output
 * run_mpc.py:138-141 reads: u_0 and the next state).  bench.py times it beside the step
 * for the PCIe-inclusive rate. */
int pl_mpc_download(pl_ocp* o, double* host_dst);
/* MPC-step HIP graph state: out[0] captures, out[1] graph launches, out[2] = 1 when the
 * step fell back to eager launches (a capture or replay failed, or PL_MPC_GRAPH=0). */
int pl_mpc_graph_info(const pl_ocp* o, long long* out);
/* Multipliers across pl_mpc_step with the interior-point solver.  carry = 0 (default): the
 * reference's default driver, solver "fatrop" with compile_solver = True (run_mpc.py:34-37,
 * 50-111): the compiled solver function takes the primal warm start only
 * (ocp_whole_body_rnea.py:239-257), so each solve starts from cold multipliers.  carry = 1: the
 * Opti branch (compile_solver = False, run_mpc.py:115-143 through OCP.solve): warm_start() passes
 * the previous solve's lam_g (ocp_whole_body_rnea.py:234-235, ocp.py:373). */
int pl_mpc_set_ip_lam(pl_ocp* o, int carry);
int pl_ocp_sync(pl_ocp* o);

/* Host-side state maps, x = [q, v], dx = [dq, dv]
 * (DynamicsWholeBodyTorque.state_integrate / state_difference,
 *  dynamics/dynamics_whole_body_torque.py:11-40). */
int pl_state_integrate(const pl_model* m, const double* x, const double* dx, double* out);
int pl_state_difference(const pl_model* m, const double* x0, const double* x1, double* dx);

/* ---- Dynamics plugin surface (dynamics/*.py factories -> batched point functions).
 * A pl_dyn handle holds the contact frames (FR, FL, RR, RL feet, optional
 * external-force frame) and the "base_link" frame of Dynamics.__init__
 * (dynamics/dynamics.py:13-17).  pl_dyn_eval evaluates `batch` points of one
 * function: inputs in0..in3 and the output are caller-owned [batch][len] float64
 * arrays (lengths from pl_dyn_sizes; unused inputs may be NULL).  flags: bit 0 =
 * the forces include the external-force frame (the factories' ext_force_frame
 * argument), bit 1 = relative_to_base (get_frame_velocity).  device >= 0 runs one
 * GPU thread per point; device = -1 evaluates the same code on the host. */
typedef struct pl_dyn pl_dyn;
#define PL_FN_RNEA 0           /* rnea_dynamics(q, v, a, forces) -> tau[nv]      dynamics/dynamics.py:33-65 */
#define PL_FN_ABA 1            /* aba_dynamics(q, v, tau_j, forces) -> a[nv]     dynamics_whole_body_torque.py:73-103 */
#define PL_FN_FRAME_POS 2      /* get_frame_position(frame)(q) -> [3]            dynamics/dynamics.py:67-75 */
#define PL_FN_FRAME_VEL 3      /* get_frame_velocity(frame, rel)(q, v) -> [6]    dynamics/dynamics.py:77-118 */
#define PL_FN_GAPS_WB 4        /* dynamics_gaps(q, v, a, forces) -> [6]          dynamics_whole_body_acc.py:85-126 */
#define PL_FN_BASE_ACC_WB 5    /* base_acc_dynamics(q, v, a_j, forces) -> [6]    dynamics_whole_body_acc.py:43-83 */
#define PL_FN_COM_DYN 6        /* com_dynamics(q, forces) -> h_dot[6]            dynamics_centroidal_vel.py:43-71 */
#define PL_FN_BASE_VEL_CV 7    /* base_vel_dynamics(h, q, v_j) -> v_b[6]         dynamics_centroidal_vel.py:73-89 */
#define PL_FN_BASE_ACC_CV 8    /* base_acc_dynamics(q, v, a_j, forces) -> a_b[6] dynamics_centroidal_vel.py:91-134 */
#define PL_FN_GAPS_CV 9        /* dynamics_gaps(h, q, v) -> A v - m h [6]        dynamics_centroidal_vel.py:136-148 */
#define PL_FN_CRBA 10          /* pinocchio crba(q) -> M[nv][nv]                 run_mpc.py:202 */
#define PL_FN_NLE 11           /* nonLinearEffects(q, v) -> [nv]                 run_mpc.py:203 */
#define PL_FN_FRAME_JAC 12     /* computeFrameJacobian(q, frame, LWA) -> [6][nv] run_mpc.py:206-209 */
#define PL_FN_CMAP 13          /* computeCentroidalMap(q) -> A_G[6][nv]          dynamics_centroidal_vel.py:80 */
#define PL_FN_COM 14           /* centerOfMass(q) -> [3]                         dynamics_centroidal_vel.py:55 */
#define PL_FN_INTEGRATE_WB 15  /* state_integrate (x=[q,v], dx) -> x'            dynamics_whole_body_torque.py:11-25 */
#define PL_FN_DIFFERENCE_WB 16 /* state_difference (x0, x1) -> dx                dynamics_whole_body_torque.py:27-40 */
#define PL_FN_INTEGRATE_CV 17  /* state_integrate (x=[h,q], dx=[dh,dq]) -> x'    dynamics_centroidal_vel.py:12-26 */
#define PL_FN_DIFFERENCE_CV 18 /* state_difference (x0, x1) -> dx                dynamics_centroidal_vel.py:28-41 */
#define PL_FN_GAPS_CA 19       /* dynamics_gaps(q, v, a, forces) -> [6]          dynamics_centroidal_acc.py:92-119 */
int pl_dyn_create(const pl_model* model, const int* foot_frames, int ext_force_frame, int base_frame, int device,
                  pl_dyn** out);
void pl_dyn_destroy(pl_dyn* d);
/* in_len: [4] input lengths, out_len: output length per point. */
int pl_dyn_sizes(const pl_dyn* d, int fn, int flags, int* in_len, int* out_len);
int pl_dyn_eval(pl_dyn* d, int fn, int batch, int frame, int flags, const double* in0, const double* in1,
                const double* in2, const double* in3, double* out);

/* ADMM linear-solve kernel.  All of them run the same OSQP 0.6 iteration on the same
 * block factor and agree to round-off; they differ in how the block-tridiagonal solve is
 * mapped to the GPU.  PL_ADMM_AUTO picks by batch size;
 * PL_ADMM_SWEEP: one wave per problem, node-by-node sweeps (large batches);
 * PL_ADMM_SWEEP2: two waves per problem; PL_ADMM_CHAIN: reduced chain, one workgroup
 * per problem (small batches).  Internal to osqp.solve() (optimization/ocp.py:401). */
#define PL_ADMM_AUTO 0
#define PL_ADMM_SWEEP 1
#define PL_ADMM_SWEEP2 2
#define PL_ADMM_CHAIN 3
int pl_ocp_set_admm_kernel(pl_ocp* o, int kind);
int pl_ocp_get_admm_kernel(const pl_ocp* o);
/* Workgroups per problem of the next ADMM launch: 1 for the sweep kernels; for the chain kernel
 * ceil((N + 1) / 8) while the batch's workgroups fit one per CU, else fewer (1 under
 * PL_PATH_RC_ONE_GROUP). */
int pl_ocp_get_admm_groups(const pl_ocp* o);

/* Timing of the dominant kernel (ADMM sweeps) with HIP events on the handle's
 * stream: pl_ocp_profile(o, 1) clears and starts, pl_ocp_profile_read returns
 * [total_ms, launches, problem_iterations]. pl_ocp_sizes (out[13]): [n, m, nnz,
 * factor doubles per problem, largest node block, N, ADMM gather program length
 * (u16 words, LDS-resident), problems per ADMM workgroup, ADMM LDS bytes per
 * workgroup, A values per thread, A values per problem staged in LDS by the sweep,
 * largest node's A count, the descriptor's debug_paths bits]. */
int pl_ocp_profile(pl_ocp* o, int enable);
int pl_ocp_profile_read(pl_ocp* o, double* out);
/* The same for the interior point's Lagrangian-Hessian launches (k_lag_hess_*): out[0] total ms,
 * out[1] launches, out[2] problem lanes per launch (the active problems rounded up to whole
 * waves; bench.py --solver fatrop scales the per-launch flops by it). */
int pl_ocp_profile_read_hess(pl_ocp* o, double* out);
int pl_ocp_sizes(const pl_ocp* o, long long* out);

/* Test / parity access to internal per-problem arrays and the node table. */
int pl_debug_get(pl_ocp* o, const char* name, double* out, long long count);
int pl_debug_set(pl_ocp* o, const char* name, const double* in, long long count);
int pl_debug_nodes(const pl_ocp* o, int* out);
int pl_debug_consts(const pl_ocp* o, void* model_out, void* oc_out, int* sizes);
int pl_debug_admm(pl_ocp* o, int niter, int reset);

#ifdef __cplusplus
}
#endif
#endif /* PINOLOCO_H_ */
