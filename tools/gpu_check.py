"""GPU smoke/parity script (development): HIP path vs numpy oracle on one SQP step."""
import sys, time, os, json
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', 'pino-locoman_amd')); sys.path.insert(0, os.path.join(HERE, '..'))
from pinoloco import robots, gait
from pinoloco.ocp import BatchedOCP
from oracle.ocp import OracleOCP

def setup(rname, dyn, N, B, seed=0):
    R = robots.ROBOTS[rname](); R.set_gait_sequence('trot', 0.8)
    o = OracleOCP(R, dyn, N)
    Q, Rw, W = o.default_weights()
    dts = gait.horizon_dts(0.01, 0.08, N)
    rng = np.random.default_rng(seed)
    Ps, Xs = [], []
    for b in range(B):
        c, s = R.gait_sequence.get_gait_schedule(rng.uniform(0, 0.8), dts, N)
        xinit = np.concatenate([R.q0, rng.normal(size=R.nv) * 0.05])
        p = o.pack_params(x_init=xinit, dt_min=0.01, dt_max=0.08, contact=c, swing=s, n_contacts=2, swing_period=0.4,
                          swing_height=0.07, swing_vel_limits=[0.1, -0.2], Q_diag=Q, R_diag=Rw,
                          base_vel_des=[0.2, 0, 0, 0, 0, 0], ext_force_des=[0, 0, 0], arm_vel_des=[0, 0, 0],
                          tau_prev=np.zeros(R.nj), W_diag=W)
        Ps.append(p); Xs.append(o.initial_guess(o.unpack(p)))
    return R, o, np.array(Ps), np.array(Xs)

def main():
    rname, dyn, N, B = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
    R, o, P, X = setup(rname, dyn, N, B)
    t = time.time()
    bo = BatchedOCP(R, dyn, N, batch=B, device=0)
    bo.set_params(P); bo.set_x(X); bo.init_solver()
    print('create', time.time() - t, flush=True)
    grad, J, g, lbg, ubg = bo.eval_sqp_data()
    rows, cols = bo.pattern()
    res = {}
    for b in range(min(B, 2)):
        g_r, l_r, u_r = o.eval_g(X[b], P[b])
        f_r, gr_r = o.f_and_grad(X[b], P[b])
        Jr = o.eval_J(X[b], P[b]).tocsr()
        Jd = np.asarray(Jr[rows, cols]).ravel()
        print('b', b, 'g err', np.abs(g[b] - g_r).max(), 'grad err', np.abs(grad[b] - gr_r).max(),
              'J err', np.abs(J[b] - Jd).max(), 'bounds eq', np.array_equal(lbg[b], l_r), flush=True)
    t = time.time()
    st = bo.solve(timed=True)
    print('solve', time.time() - t, st, flush=True)
    step = bo.get_step(); xnew = bo.get_x()
    for b in range(min(B, 2)):
        o.init_solver(X[b], P[b])
        xo, dxo, sto = o.sqp_step(X[b], P[b])
        print('oracle', b, sto, flush=True)
        err = np.abs(step[b] - dxo).max() / max(1e-12, np.abs(dxo).max())
        print('b', b, 'step rel err', err, 'x rel err', np.abs(xnew[b] - xo).max() / np.abs(xo).max(), flush=True)

if __name__ == '__main__':
    main()
