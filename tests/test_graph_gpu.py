"""MPC-step graph replay (pl_mpc_step, api.hip): the OSQP-SQP launches of a step are
captured once into a HIP graph and replayed.  A replay must be the eager launch sequence:
states, iterates and solver statistics bit-identical to a handle created with
the no_mpc_graph debug path, including across a setter that changes the handle mid-loop (re-capture), and the capture /
replay counters (pl_mpc_graph_info) show that the graph path ran."""
import numpy as np
import pytest

from conftest import make_robot

pytestmark = pytest.mark.gpu


def _loop(R, dyn, N, B, steps, graph, switch_at=None):
    from pinoloco.ocp import BatchedOCP
    from pinoloco.synthetic import build_batch
    lay, P, X, XS, T0 = build_batch(R, dyn, N, B, 0)
    bo = BatchedOCP(R, dyn, N, batch=B, device=0, debug_paths=() if graph else ("no_mpc_graph",))
    bo.set_params(P)
    bo.set_x(X)
    bo.init_solver()
    bo.mpc_setup(XS, T0)
    states, stats = [], []
    for k in range(steps):
        if switch_at is not None and k == switch_at:
            bo.set_sqp_iters(2)  # changes the captured sequence: the next steps re-capture
        bo.mpc_step(k)
        states.append(bo.mpc_state().copy())
        st = bo.mpc_stats()
        stats.append({key: np.array(v).copy() for key, v in st.items()})
    x = bo.get_x().copy()
    info = bo.mpc_graph_info()
    bo.close()
    return states, stats, x, info


@pytest.mark.parametrize("rname,dyn,N,B,switch_at", [
    ("go2", "whole_body_rnea", 20, 1, None),     # config 2 shape: chain ADMM kernel
    ("go2", "centroidal_vel", 20, 64, 3),        # re-capture after set_sqp_iters
    ("b2", "whole_body_aba", 40, 300, None),     # two-wave sweep kernel
])
def test_graph_replay_is_bit_identical_to_eager(rname, dyn, N, B, switch_at):
    R = make_robot(rname)
    eager = _loop(R, dyn, N, B, 6, False, switch_at)
    graph = _loop(R, dyn, N, B, 6, True, switch_at)
    for k in range(6):
        assert np.array_equal(eager[0][k], graph[0][k]), k
        for key in eager[1][k]:
            assert np.array_equal(eager[1][k][key], graph[1][k][key], equal_nan=True), (k, key)
    assert np.array_equal(eager[2], graph[2])
    # the replay path really ran: step 0 eager (first sighting of the handle state), step 1
    # captures and launches the graph, later steps replay it; set_sqp_iters changes the state,
    # so that step runs eagerly and the next one captures again
    assert eager[3] == {"captures": 0, "replays": 0, "eager_fallback": 1}
    if switch_at is None:
        assert graph[3] == {"captures": 1, "replays": 5, "eager_fallback": 0}, graph[3]
    else:
        assert graph[3] == {"captures": 2, "replays": 6 - 2, "eager_fallback": 0}, graph[3]
