"""C-ABI boundary (include/pinoloco.h) without a GPU.

* the library loads and exports every function the header declares;
* a host-only handle (device = -1) reports the SURVEY 8 sizes, and its Jacobian
  pattern covers every structurally non-zero entry of the oracle's J_g;
* the host Lie-group maps (pl_state_integrate / pl_state_difference) match the oracle;
* the Python Layout packs parameters exactly like the oracle (Opti declaration order);
* errors come back as negative codes with pl_last_error(), never as crashes.
"""
import ctypes as C
import os
import re

import numpy as np
import pytest

from conftest import ROOT, make_robot
from oracle import rbd
from oracle.ocp import OracleOCP

HEADER = os.path.join(ROOT, "include", "pinoloco.h")
CONFIGS = [("go2", "whole_body_rnea", 20, 1392, 2032, 318), ("b2", "whole_body_aba", 40, 2436, 3680, None),
           ("b2g", "whole_body_acc", 50, 4398, 6397, None), ("b2g", "whole_body_rnea", 50, 4452, 6505, 609),
           ("go2", "centroidal_vel", 20, 1104, 1744, None)]


def header_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pl_[a-z_0-9]+)\s*\(", text)))


def test_header_symbols_exported():
    from pinoloco import _lib
    L = _lib.lib()
    names = header_functions()
    assert len(names) >= 30
    for n in names:
        assert hasattr(L, n), n
        assert n in _lib.EXPORTS, f"{n} declared in pinoloco.h but not bound in _lib.EXPORTS"
    assert set(_lib.EXPORTS) == set(names)
    assert L.pl_version() >= 1


def test_struct_layouts_match_header(tmp_path):
    """ctypes mirrors of pl_model_desc / pl_ocp_desc / pl_stats have the C compiler's layout."""
    import shutil
    import subprocess
    from pinoloco import _lib
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    src = tmp_path / "sz.c"
    fields = {"pl_stats": (_lib.Stats, ["f", "ls_alpha", "viol_max"]),
              "pl_ocp_desc": (_lib.OcpDesc, ["gait_period", "rho", "mu", "foot_frames", "max_iter"]),
              "pl_model_desc": (_lib.ModelDesc, ["nframes", "frame_p", "gravity"]),
              "pl_ip_stats": (_lib.IpStats, ["err", "alphas", "ref_solves"])}
    body = "".join(f'printf("{t} %zu\\n", sizeof({t}));' + "".join(
        f'printf("{t}.{f} %zu\\n", offsetof({t}, {f}));' for f in fl) for t, (_, fl) in fields.items())
    src.write_text(f'#include <stdio.h>\n#include <stddef.h>\n#include "pinoloco.h"\nint main(void){{{body}return 0;}}\n')
    exe = tmp_path / "sz"
    subprocess.run([cc, "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    out = dict(line.split() for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                       check=True).stdout.split("\n") if line)
    for t, (cls, fl) in fields.items():
        assert int(out[t]) == C.sizeof(cls), t
        for f in fl:
            assert int(out[f"{t}.{f}"]) == getattr(cls, f).offset, (t, f)


@pytest.mark.parametrize("rname,dyn,N,n,m,np_", CONFIGS)
def test_host_handle_dims_and_pattern(rname, dyn, N, n, m, np_):
    from pinoloco.ocp import BatchedOCP
    from pinoloco.synthetic import build_batch
    R = make_robot(rname)
    bo = BatchedOCP(R, dyn, N, batch=1, device=-1)
    assert (bo.n, bo.m) == (n, m)
    if np_ is not None:
        assert bo.np == np_
    rows, cols = bo.pattern()
    assert len(rows) == bo.nnz and rows.min() >= 0 and rows.max() < m and cols.max() < n
    assert len(set(zip(rows.tolist(), cols.tolist()))) == bo.nnz  # no duplicate entries
    if rname == "b2g" and dyn == "whole_body_rnea":
        assert bo.nnz == 52313
    # every entry the oracle finds non-zero at a random point is in the pattern
    o = OracleOCP(R, dyn, N)
    lay, P, X, _, _ = build_batch(R, dyn, N, 1, 3)
    x = X[0] + np.random.default_rng(0).normal(0, 0.05, n)
    J = o.eval_J(x, P[0]).tocoo()
    mine = set(zip(rows.tolist(), cols.tolist()))
    big = {(r, c) for r, c, v in zip(J.row, J.col, J.data) if abs(v) > 1e-12}
    assert not (big - mine)
    # the node table tiles the decision vector and the rows
    nt = bo.node_table()
    assert nt[:, 0].sum() == n and nt[:, 4].sum() == m
    assert np.all(nt[1:, 3] == np.cumsum(nt[:-1, 4]))
    bo.close()


@pytest.mark.parametrize("rname,N", [("go2", 20), ("b2g", 50)])
def test_host_handle_rnea_include_acc_false(rname, N):
    """whole_body_rnea include_acc=False (ocp_whole_body_rnea.py:21-26, 69-76, 157-159):
    na_opt = 0 (u = [f | tau_j]), no dv_{i+1} rows, n and m as the oracle counts them, the
    pattern covers the oracle's non-zeros (the RNEA rows of node i read dv_{i+1})."""
    from pinoloco.ocp import BatchedOCP
    from pinoloco.synthetic import build_batch
    R = make_robot(rname)
    bo = BatchedOCP(R, "whole_body_rnea", N, batch=1, device=-1, include_acc=False)
    o = OracleOCP(R, "whole_body_rnea", N, include_acc=False)
    full = OracleOCP(R, "whole_body_rnea", N)
    assert bo.n == o.n == full.n - N * R.nv
    lay, P, X, _, _ = build_batch(R, "whole_body_rnea", N, 1, 3, include_acc=False)
    g, _, _ = o.eval_g(X[0], P[0])
    gf, _, _ = full.eval_g(np.zeros(full.n), build_batch(R, "whole_body_rnea", N, 1, 3)[1][0])
    assert bo.m == g.size == gf.size - N * R.nv
    rows, cols = bo.pattern()
    x = X[0] + np.random.default_rng(0).normal(0, 0.05, bo.n)
    J = o.eval_J(x, P[0]).tocoo()
    mine = set(zip(rows.tolist(), cols.tolist()))
    big = {(r, c) for r, c, v in zip(J.row, J.col, J.data) if abs(v) > 1e-12}
    assert not (big - mine)
    # node 1's RNEA base rows reach into dv_2 (finite-difference a)
    nt = bo.node_table()
    dv2 = set(range(nt[2, 2] + R.nv, nt[2, 2] + 2 * R.nv))
    assert any(c in dv2 for r, c in big if nt[1, 3] <= r < nt[1, 3] + nt[1, 4])
    bo.close()


def test_build_info_matches_tree():
    """pl_build_info carries the sha256 of the sources the library was built from, and build()
    rebuilds by that hash (not by file times): the library under test is this tree's."""
    from pinoloco import _lib
    from pinoloco import build as _build
    info = _lib.lib().pl_build_info().decode()
    assert info.startswith("pl_src_sha256=") and "arch=gfx950" in info
    assert _lib.build_sha() == _build.source_sha() == _build.embedded_sha()


def test_debug_paths_outside_mask_rejected(monkeypatch):
    """pl_ocp_create rejects debug_paths bits outside PL_PATH_ALL (a caller that does not zero
    the pl_ocp_desc gets an error, not a silently different kernel path)."""
    from pinoloco import _lib
    from pinoloco.ocp import BatchedOCP
    R = make_robot("go2")
    monkeypatch.setitem(_lib.PATHS, "undefined_bit", 1 << 20)
    with pytest.raises(_lib.PinolocoError, match="debug_paths"):
        BatchedOCP(R, "whole_body_rnea", 10, batch=1, device=-1, debug_paths=("undefined_bit",))
    bo = BatchedOCP(R, "whole_body_rnea", 10, batch=1, device=-1, debug_paths=tuple(k for k in _lib.PATHS
                                                                                   if k != "undefined_bit"))
    assert bo.sizes()["debug_paths"] == 2047
    bo.close()


def test_host_handle_refuses_solves():
    from pinoloco import _lib
    from pinoloco.ocp import BatchedOCP
    R = make_robot("go2")
    bo = BatchedOCP(R, "whole_body_rnea", 10, batch=2, device=-1)
    with pytest.raises(_lib.PinolocoError):
        bo.solve()
    with pytest.raises(_lib.PinolocoError):
        bo.set_params(np.zeros((2, bo.np)))
    bo.close()


def test_bad_arguments_are_errors():
    from pinoloco import _lib
    from pinoloco.ocp import BatchedOCP, make_ocp, OCP_ARGS
    L = _lib.lib()
    assert L.pl_ocp_dims(None, None, None, None, None) < 0
    assert L.pl_last_error()
    R = make_robot("go2")
    with pytest.raises(ValueError):
        BatchedOCP(R, "centroidal_jerk", 10, device=-1)
    with pytest.raises(ValueError):
        make_ocp("nonsense", OCP_ARGS, robot=R, nodes=10, solver="osqp")
    with pytest.raises(_lib.PinolocoError):
        BatchedOCP(R, "whole_body_rnea", 10, batch=0, device=-1)
    bo = BatchedOCP(R, "whole_body_rnea", 10, batch=1, device=-1)
    bo.set_sqp_iters(3)  # a setting: allowed on a host-only handle
    for bad in (0, -1, 1001):
        with pytest.raises(_lib.PinolocoError):
            bo.set_sqp_iters(bad)
    bo.close()


@pytest.mark.parametrize("rname", ["go2", "b2g"])
def test_host_state_maps_match_oracle(rname):
    from pinoloco.ocp import Dynamics
    R = make_robot(rname)
    M = rbd.ModelArrays(R.model)
    dyn = Dynamics(R)
    integ, diff = dyn.state_integrate(), dyn.state_difference()
    rng = np.random.default_rng(11)
    for _ in range(4):
        qu = rng.normal(size=4)
        q = R.q0.copy()
        q[3:7] = qu / np.linalg.norm(qu)
        xs = np.concatenate([q, rng.normal(size=R.nv)])
        dx = rng.normal(size=2 * R.nv) * 0.3
        out = integ(xs, dx)
        ref = np.concatenate([rbd.integrate(M, xs[:R.nq], dx[:R.nv]), xs[R.nq:] + dx[R.nv:]])
        assert np.abs(out - ref).max() < 1e-14
        assert np.abs(diff(xs, out) - dx).max() < 1e-11


@pytest.mark.parametrize("rname,dyn,N", [("go2", "whole_body_rnea", 20), ("b2", "whole_body_aba", 40),
                                         ("b2g", "whole_body_acc", 50), ("go2", "centroidal_vel", 20)])
def test_layout_pack_matches_oracle(rname, dyn, N):
    from pinoloco.ocp import Layout
    from pinoloco.synthetic import problem_values, initial_guess
    R = make_robot(rname)
    lay = Layout(R, dyn, N)
    vals, _, _ = problem_values(R, dyn, N, 5, lay)
    o = OracleOCP(R, dyn, N)
    kw = {k: v for k, v in vals.items() if k not in ("contact_schedule", "swing_schedule")}
    kw.update(contact=vals["contact_schedule"], swing=vals["swing_schedule"])
    if dyn != "whole_body_rnea":
        kw.pop("tau_prev")
        kw.pop("W_diag")
    p = lay.pack(vals)
    assert np.array_equal(p, o.pack_params(**kw))
    assert np.array_equal(initial_guess(R, lay, vals["n_contacts"]), o.initial_guess(o.unpack(p)))
    assert lay.x_off == o.x_off and lay.n == o.n


def test_shard_partition():
    from pinoloco.synthetic import shard
    for G in (1, 2, 3, 8):
        spans = [shard(1000, G, r) for r in range(G)]
        assert spans[0][0] == 0 and sum(c for _, c in spans) == 1000
        for (f0, c0), (f1, _) in zip(spans, spans[1:]):
            assert f0 + c0 == f1
