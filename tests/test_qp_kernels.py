"""QP-setup kernels on the MI355X: the fused equilibration (k_ruiz_fused, all Ruiz passes of
OSQP 0.6 scale_data in one launch) against the per-pass kernels (k_ruiz_norms +
k_ruiz_update, debug path ruiz_per_pass): D, E, c and the scaled data bit for bit, and the SQP
outcome and step bit for bit (optimization/ocp.py:391-401, osqp.update + osqp.solve)."""
import numpy as np
import pytest

from conftest import golden
from test_gpu import ACCF, CONFIGS, EDGE, _batched

pytestmark = pytest.mark.gpu


def _run(name, rname, dyn, N, fused):
    G = golden(f"sqp_{name}.npz")
    R, bo = _batched(rname, dyn, N, G, debug_paths=() if fused else ("ruiz_per_pass",))
    st = bo.solve()
    B = bo.batch
    out = {k: bo.debug(k, B * sz) for k, sz in (("D", bo.n), ("E", bo.m), ("cs", 1), ("As", bo.nnz), ("Ps", bo.n),
                                                ("qs", bo.n), ("ls", bo.m), ("us", bo.m))}
    out["x"] = bo.get_x()
    out["step"] = bo.get_step()
    for k in ("status", "admm_iters", "ls_branch", "ls_trials", "ls_alpha"):
        out[k] = np.asarray(st[k])
    bo.close()
    return out


@pytest.mark.parametrize("name,rname,dyn,N", CONFIGS + EDGE[:2] + ACCF[-2:])
def test_fused_ruiz_bit_identical(name, rname, dyn, N):
    a = _run(name, rname, dyn, N, True)
    b = _run(name, rname, dyn, N, False)
    for k in a:
        assert np.array_equal(a[k], b[k], equal_nan=True), k
