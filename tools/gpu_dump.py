"""Dump internal solver arrays of one small batch (diagnostics)."""
import sys, os, numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', 'pino-locoman_amd')); sys.path.insert(0, os.path.join(HERE, '..'))
exec(open(os.path.join(HERE, 'gpu_check.py')).read().split("def main")[0])
rname, dyn, N, B = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4])
R, o, P, X = setup(rname, dyn, N, B)
bo = BatchedOCP(R, dyn, N, batch=B, device=0)
bo.set_params(P); bo.set_x(X); bo.init_solver()
sz = bo.sizes()
st = bo.solve()
out = dict(P=P, X=X, nodes=bo.node_table(), rows=bo.pattern()[0], cols=bo.pattern()[1])
for name, ln in [('As', sz['nnz']), ('Araw', sz['nnz']), ('qs', sz['n']), ('ls', sz['m']), ('us', sz['m']), ('rho', sz['m']),
                 ('D', sz['n']), ('E', sz['m']), ('cs', 1), ('Ps', sz['n']), ('P', sz['n']), ('S', sz['S_stride']),
                 ('step', sz['n']), ('xa', sz['n']), ('za', sz['m']), ('ya', sz['m']), ('grad', sz['n']), ('g', sz['m'])]:
    out[name] = bo.debug(name, ln * B).reshape(B, -1)
for k, v in st.items(): out['st_' + k] = v
np.savez_compressed(os.path.join(HERE, '..', 'gpurun_out', f'dump_{rname}.npz'), **out)
print('ok', st)
