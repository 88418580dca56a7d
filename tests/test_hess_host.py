"""The Lagrangian Hessian's forward-over-reverse columns against the hyper-dual pair sweeps, on the CPU.

csrc/hess_tree.h holds both sweeps of the whole_body_rnea / whole_body_acc state pairs as host/device
code: tree_pair (one hyper-dual sweep per (j, k) pair, the r05 kernel k_lag_hess_tree) and tree_col
(r06: a dual sweep seeded on column j, then the reverse sweep in dual numbers, giving the whole column
at once; the kernel k_lag_hess_col).  tests/native/hess_host.cpp builds them for the host; here every
column of every chain (and the whole-tree base columns) of several node types is compared with the
pairs at random states and multipliers: <= 1e-12 of the block's largest entry.  On the GPU the two
kernels are compared the same way (tests/test_r04_paths.py) and the IP fixtures hold with the columns.
"""
import ctypes as C
import os
import shutil
import subprocess

import numpy as np
import pytest

from conftest import ROOT, make_robot

_dp = C.POINTER(C.c_double)


@pytest.fixture(scope="module")
def harness(tmp_path_factory):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc) and shutil.which(hipcc) is None:
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("hess") / "libhess_host.so"
    cmd = [hipcc, "-std=c++17", "-O2", "-fPIC", "-shared", "-x", "hip", "--offload-arch=gfx950",
           "-Wno-unused-result", "-I", os.path.join(ROOT, "pino-locoman_amd", "csrc"),
           os.path.join(ROOT, "tests", "native", "hess_host.cpp"), "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True)
    L = C.CDLL(str(out))
    L.th_hess_pair.restype = C.c_double
    L.th_hess_pair.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, _dp, _dp, _dp]
    L.th_hess_col.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_uint, _dp, _dp, _dp, _dp]
    L.th_col_coord.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int]
    L.th_chain_len.argtypes = [C.c_void_p, C.c_int]
    L.th_nchains.argtypes = [C.c_void_p]
    return L


def _consts(bo):
    from pinoloco import _lib
    L = _lib.lib()
    sizes = (C.c_int * 2)()
    _lib.check(L.pl_debug_consts(bo.h, None, None, sizes))
    mb, ob = C.create_string_buffer(sizes[0]), C.create_string_buffer(sizes[1])
    _lib.check(L.pl_debug_consts(bo.h, mb, ob, None))
    return mb, ob


def _d(a):
    return a.ctypes.data_as(_dp)


@pytest.mark.parametrize("rname,dyn,N,nodes", [("go2", "whole_body_rnea", 20, [0, 1, 7]),
                                               ("b2g", "whole_body_rnea", 50, [0, 2, 30]),
                                               ("b2g", "whole_body_acc", 50, [0, 11])])
def test_columns_match_pairs(harness, rname, dyn, N, nodes):
    from pinoloco.ocp import BatchedOCP
    from pinoloco.synthetic import build_batch
    R = make_robot(rname)
    lay, P, X, _, _ = build_batch(R, dyn, N, 2, 5)
    bo = BatchedOCP(R, dyn, N, batch=1, device=-1)
    mb, ob = _consts(bo)
    nt = bo.node_table()  # nw, ..., x_off (col 2), row_off (col 3), nrow (col 4)
    rng = np.random.default_rng(3)
    H = harness
    nch = H.th_nchains(mb)
    worst = 0.0
    checked = 0
    for b in range(2):
        x = X[b] + rng.normal(0, 0.05, X.shape[1])
        p = np.ascontiguousarray(P[b])
        lam_all = rng.normal(0, 5.0, bo.m)
        for i in nodes:
            xo, ro = int(nt[i, 2]), int(nt[i, 3])
            xi = np.ascontiguousarray(x[xo:])
            lam = np.ascontiguousarray(lam_all[ro:])
            for ch in range(-1, nch):
                nloc = 12 if ch < 0 else 12 + 2 * H.th_chain_len(mb, ch)
                coords = [H.th_col_coord(mb, ob, ch, loc) for loc in range(nloc)]
                for j in [c for c in coords if c < bo.layout.ndx // 2]:  # the dq columns (htr pairs: j < nv)
                    # the pairs a work item of this kind writes (api.hip set_solver): the whole-tree items
                    # the base pairs; a chain item with a base-rotation column j its chain's coordinates,
                    # with a chain column also the base velocities (the base-base pairs are whole-tree)
                    jchain = ch >= 0 and coords.index(j) >= 12
                    locs = [loc for loc, k in enumerate(coords) if k >= j and
                            (ch < 0 or loc >= 12 or (jchain and 6 <= loc < 12))]
                    mask = sum(1 << loc for loc in locs)
                    out = np.full(bo.layout.ndx, np.nan)
                    H.th_hess_col(mb, ob, i, ch, j, mask, _d(xi), _d(p), _d(lam), _d(out))
                    pairs = np.array([H.th_hess_pair(mb, ob, i, ch, j, coords[loc], _d(xi), _d(p), _d(lam))
                                      for loc in locs])
                    got = np.array([out[coords[loc]] for loc in locs])
                    scale = max(1.0, np.abs(pairs).max())
                    err = np.abs(got - pairs).max() / scale
                    worst = max(worst, err)
                    checked += len(locs)
                    assert err < 1e-12, (i, ch, j, err, np.c_[[coords[l] for l in locs], got, pairs])
    bo.close()
    print(f"{rname} {dyn}: {checked} entries, worst {worst:.2e}")
