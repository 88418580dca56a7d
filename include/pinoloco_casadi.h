/* CasADi external-function ABI exported by libpinoloco.so.
 *
 * The reference evaluates its SQP data with CasADi Functions and can load generated
 * code instead:
 *   sqp_data(x, p) -> (grad_f, J_g, g, lbg, ubg)     optimization/ocp.py:287
 *   hess_data(x, p) -> hess_f                         optimization/ocp.py:288
 *   f_data(x, p) -> (f, grad_f)                       optimization/ocp.py:289
 *   g_data(x, p) -> (g, lbg, ubg)                     optimization/ocp.py:290
 *   retract_solution(sol_x, x_init) -> (q, v, a, forces, tau)
 *                                                     optimization/ocp_whole_body_rnea.py:326-366
 *   compiled_solver(params..., [x_warm_start], [tau_prev, W_diag]) -> x
 *                                                     ocp_whole_body_rnea.py:237-258, run_mpc.py:51-53
 *   self.sqp_data = ca.external("sqp_data", "codegen/sqp/libsqp_data_....so")
 *                                                     optimization/ocp.py:299-302, run_mpc.py:53
 * libpinoloco.so exports each NAME with CasADi's generated-code calling convention
 * (casadi_int = long long, casadi_real = double, compressed-column sparsity
 * [nrow, ncol, colind[ncol+1], row[nnz]]), so ca.external("sqp_data", <libpinoloco.so>)
 * works unchanged once pl_casadi_bind() (include/pinoloco.h) has bound the OCP.
 * Evaluations run on the bound handle's GPU (problem slot 0); J_g is in CasADi CCS order
 * over the structural-dependency pattern of jacobian(g, x) -- the library's entries that
 * are non-zero at a generic point (one dual-number probe per node type at bind time) --
 * so the reference's A pattern from J_g.sparsity() (optimization/ocp.py:305-306) and the
 * J_g.nonzeros() it feeds OSQP (ocp.py:391) have the same length and order: swapping in
 * ca.external is the one-line change of ocp.py:299-302.  Return value 0 = success.
 */
#ifndef PINOLOCO_CASADI_H
#define PINOLOCO_CASADI_H
#ifdef __cplusplus
extern "C" {
#endif

#define PL_CASADI_DECLARE(NAME)                                                          \
  int NAME(const double** arg, double** res, long long* iw, double* w, int mem);      \
  int NAME##_alloc_mem(void);                                                          \
  int NAME##_init_mem(int mem);                                                        \
  void NAME##_free_mem(int mem);                                                       \
  int NAME##_checkout(void);                                                           \
  void NAME##_release(int mem);                                                        \
  void NAME##_incref(void);                                                            \
  void NAME##_decref(void);                                                            \
  long long NAME##_n_in(void);                                                         \
  long long NAME##_n_out(void);                                                        \
  double NAME##_default_in(long long i);                                               \
  const char* NAME##_name_in(long long i);                                             \
  const char* NAME##_name_out(long long i);                                            \
  const long long* NAME##_sparsity_in(long long i);                                    \
  const long long* NAME##_sparsity_out(long long i);                                   \
  int NAME##_work(long long* sz_arg, long long* sz_res, long long* sz_iw, long long* sz_w);

PL_CASADI_DECLARE(sqp_data)
PL_CASADI_DECLARE(f_data)
PL_CASADI_DECLARE(g_data)
PL_CASADI_DECLARE(hess_data)
PL_CASADI_DECLARE(retract_solution)
/* compiled_solver(x_init, dt_min, dt_max, contact_schedule, swing_schedule, n_contacts,
 *                 swing_period, swing_height, swing_vel_limits, Q_diag, R_diag, base_vel_des,
 *                 [ext_force_des], [arm_vel_des], [x_warm_start], [tau_prev, W_diag]) -> x
 *   the Fatrop branch's generated solver (ocp_whole_body_rnea.py:237-258, ocp.py:324-342),
 *   loaded with ca.external("compiled_solver", lib) at run_mpc.py:51-53; bound with
 *   pl_casadi_bind_compiled (include/pinoloco.h).  One interior-point solve on the GPU. */
PL_CASADI_DECLARE(compiled_solver)

#ifdef __cplusplus
}
#endif
#endif
