"""Dump ADMM iterates after k iterations (diagnostics)."""
import sys, os, numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, '..', 'pino-locoman_amd')); sys.path.insert(0, os.path.join(HERE, '..'))
exec(open(os.path.join(HERE, 'gpu_check.py')).read().split("def main")[0])
from pinoloco import _lib
R, o, P, X = setup('go2', 'whole_body_rnea', 20, 2)
bo = BatchedOCP(R, 'whole_body_rnea', 20, batch=2, device=0)
bo.set_params(P); bo.set_x(X); bo.init_solver()
sz = bo.sizes(); out = {}
for k in (0, 1, 2, 5):
    _lib.check(_lib.lib().pl_debug_admm(bo.h, k, 1))
    for name, ln in [('xa', sz['n']), ('za', sz['m']), ('ya', sz['m']), ('rhs', sz['n'])]:
        out[f'{name}_{k}'] = bo.debug(name, ln * 2).reshape(2, -1)
for name, ln in [('As', sz['nnz']), ('qs', sz['n']), ('ls', sz['m']), ('us', sz['m']), ('rho', sz['m']), ('D', sz['n']), ('Ps', sz['n']), ('S', sz['S_stride'])]:
    out[name] = bo.debug(name, ln * 2).reshape(2, -1)
out['nodes'] = bo.node_table(); out['rows'], out['cols'] = bo.pattern()
np.savez_compressed(os.path.join(HERE, '..', 'gpurun_out', 'dump2.npz'), **out)
print('ok')
