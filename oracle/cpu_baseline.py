"""CPU BASELINE (test infrastructure): ctypes driver of oracle/cpu/sqp_cpu.cpp.

A compiled C++ restatement of the reference's CPU solve path (OSQP 0.6 with the
QDLDL LDL^T on the quasi-definite KKT, the Armijo / filter line search, the MPC
loop of run_mpc.py:127-143), and of the interior-point stand-in for its Fatrop
branch (oracle/ip_ref.py: exact Lagrangian Hessian, QDLDL on the IP's KKT), run with
OpenMP over independent problems.  bench.py
times it on the GPU box's host cores beside the GPU run (``cpu_baseline``);
tests/test_cpu_baseline.py checks it against the numpy oracle's golden vectors.
Only tests/, bench.py's cpu_baseline leg and __graft_entry__ use this module.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.normpath(os.path.join(HERE, ".."))
SRC = os.path.join(HERE, "cpu", "sqp_cpu.cpp")
LIB = os.path.join(HERE, "_build", "libsqp_cpu.so")
CSRC = os.path.join(ROOT, "pino-locoman_amd", "csrc")
# x86-64-v3 (AVX2 + FMA): built in the development container, run on the GPU box's host
CXXFLAGS = ["-std=c++17", "-O3", "-march=x86-64-v3", "-fopenmp", "-fPIC", "-shared", "-Wno-unknown-pragmas",
            "-Wno-maybe-uninitialized", "-Wno-uninitialized"]

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)
_lib = None


def _inputs():
    hdrs = ("ad.h", "model.h", "rbd.h", "rows.h", "targets.h")
    return [SRC, os.path.abspath(__file__)] + [os.path.join(CSRC, h) for h in hdrs]


def source_sha():
    """sha256 of the baseline's inputs (the C++ source, this driver, the shared row headers) and
    flags; the library is rebuilt whenever its stamp file holds another hash (not by mtime)."""
    h = hashlib.sha256(" ".join(CXXFLAGS).encode())
    for p in _inputs():
        h.update(os.path.basename(p).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()


def build(force=False):
    sha = source_sha()
    stamp = LIB + ".sha256"
    if not force and os.path.exists(LIB) and os.path.exists(stamp) and open(stamp).read().strip() == sha:
        return LIB
    os.makedirs(os.path.dirname(LIB), exist_ok=True)
    cmd = ["g++"] + CXXFLAGS + ["-I", CSRC, SRC, "-o", LIB + ".tmp"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"CPU baseline build failed:\n{r.stderr[-4000:]}")
    os.replace(LIB + ".tmp", LIB)
    with open(stamp, "w") as f:
        f.write(sha + "\n")
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        L.cpu_create.restype = C.c_void_p
        L.cpu_create.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, _ip, _ip, _ip, _ip,
                                 _ip, _ip, _dp, C.c_int, C.c_double]
        L.cpu_destroy.argtypes = [C.c_void_p]
        L.cpu_factor_nnz.restype = C.c_longlong
        L.cpu_factor_nnz.argtypes = [C.c_void_p]
        L.cpu_mpc_batch.restype = C.c_double
        L.cpu_mpc_batch.argtypes = [C.c_void_p, C.c_int, _dp, _dp, _dp, _dp, C.c_int, C.c_int, _dp, _ip]
        L.cpu_sqp_step.argtypes = [C.c_void_p, _dp, _dp, _dp, _ip, _dp]
        L.cpu_ip_prepare.restype = C.c_longlong
        L.cpu_ip_prepare.argtypes = [C.c_void_p]
        L.cpu_ip_solve.argtypes = [C.c_void_p, _dp, _dp, _dp, C.c_int, _dp, _ip, _dp]
        L.cpu_ip_lag_hess.argtypes = [C.c_void_p, _dp, _dp, _dp, _dp]
        L.cpu_ip_mpc_batch.restype = C.c_double
        L.cpu_ip_mpc_batch.argtypes = [C.c_void_p, C.c_int, _dp, _dp, _dp, _dp, C.c_int, C.c_int, _dp, _dp, _ip]
        _lib = L
    return _lib


def _d(a):
    return a.ctypes.data_as(_dp)


def _i(a):
    return a.ctypes.data_as(_ip)


class CpuOCP:
    """One (robot, dynamics, N) OCP on the CPU baseline; structure from the product's
    host-only handle (layout and Jacobian pattern, pl_ocp_pattern / pl_debug_consts)."""

    def __init__(self, robot, dynamics, nodes, osqp_settings=None, gait_type="trot", gait_period=0.8, **kw):
        from pinoloco import _lib as plib
        from pinoloco.ocp import GAIT_CODES, OSQP_SETTINGS, BatchedOCP
        s = dict(OSQP_SETTINGS)
        s.update(osqp_settings or {})
        bo = BatchedOCP(robot, dynamics, nodes, batch=1, device=-1, osqp_settings=s, gait_type=gait_type,
                        gait_period=gait_period, **kw)  # kw: include_base / include_acc
        sizes = (C.c_int * 2)()
        plib.check(plib.lib().pl_debug_consts(bo.h, None, None, sizes))
        mb, ob = C.create_string_buffer(sizes[0]), C.create_string_buffer(sizes[1])
        plib.check(plib.lib().pl_debug_consts(bo.h, mb, ob, None))
        rows, cols = bo.pattern()
        nt = bo.node_table()
        self.n, self.m, self.np, self.N = bo.n, bo.m, bo.np, nodes
        self.nx = bo.layout.nx
        arrs = [np.ascontiguousarray(nt[:, k], dtype=np.int32) for k in (2, 3, 4, 0)]  # x_off, row_off, nrow, nw
        st = np.array([s["rho"], s["sigma"], s["alpha"], s["eps_abs"], s["eps_rel"], s["eps_prim_inf"],
                       s["eps_dual_inf"], s["max_iter"], s["check_termination"], s["scaling"]], dtype=np.float64)
        self._keep = (mb, ob, arrs, rows, cols, st)
        self.h = lib().cpu_create(mb, ob, nodes, bo.n, bo.m, bo.nnz, *[_i(a) for a in arrs], _i(rows), _i(cols),
                                  _d(st), GAIT_CODES[gait_type], float(gait_period))
        bo.close()

    def factor_nnz(self):
        return int(lib().cpu_factor_nnz(self.h))

    def sqp_step(self, x, p):
        """One SQP iteration from a cold OSQP (like OracleOCP.init_solver + sqp_step)."""
        x = np.ascontiguousarray(np.array(x, dtype=np.float64))
        p = np.ascontiguousarray(np.asarray(p, dtype=np.float64))
        dx = np.zeros(self.n)
        stats = np.zeros(4, dtype=np.int32)
        alpha = C.c_double()
        lib().cpu_sqp_step(self.h, _d(p), _d(x), _d(dx), _i(stats), C.byref(alpha))
        return x, dx, dict(status=int(stats[0]), iter=int(stats[1]), branch=int(stats[2]), trials=int(stats[3]),
                           alpha=alpha.value)

    def mpc(self, P, X, XS, T0, steps, threads=0):
        """`steps` MPC steps of every problem; returns (wall seconds, final states, stats)."""
        B = P.shape[0]
        P, X, XS = (np.ascontiguousarray(a, dtype=np.float64) for a in (P, X, XS))
        T0 = np.ascontiguousarray(T0, dtype=np.float64)
        xs = np.zeros((B, self.nx))
        stats = np.zeros((B, steps, 4), dtype=np.int32)
        wall = lib().cpu_mpc_batch(self.h, B, _d(P), _d(X), _d(XS), _d(T0), steps, threads, _d(xs), _i(stats))
        return wall, xs, stats

    @staticmethod
    def _ip_settings(settings=None):
        from oracle.ip_ref import IP_SETTINGS
        s = dict(IP_SETTINGS)
        s.update(settings or {})
        if s["hessian"] != "exact":
            raise ValueError("the CPU interior point restates the exact-Hessian form only")
        return np.array([s["tol"], s["mu_init"], s["bound_push"], s["bound_frac"], s["warm_start_mult_bound_push"],
                         s["delta_w"], s["delta_c"], s["max_iter"], s["ls_max"], s["n_refine"], s["inertia_cap"],
                         1.0 if s["kkt_refine"] == "exact" else 0.0, 1.0 if s.get("mpc_lam", False) else 0.0],
                        dtype=np.float64)

    def hess_pairs(self):
        """Number of Lagrangian-Hessian column pairs over the horizon (structural probe)."""
        n = int(lib().cpu_ip_prepare(self.h))
        if n < 0:
            raise ValueError("the interior-point restatement needs include_acc=True")
        return n

    def lag_hess(self, x, p, lam):
        """The restatement's Lagrangian Hessian blocks at (x, p, lam): dense n x n."""
        H = np.zeros((self.n, self.n))
        args = [np.ascontiguousarray(np.asarray(a, dtype=np.float64)) for a in (p, x, lam)]
        if lib().cpu_ip_lag_hess(self.h, *[_d(a) for a in args], _d(H)) != 0:
            raise ValueError("the interior-point restatement needs include_acc=True")
        return H

    def ip_solve(self, x, p, lam0=None, settings=None):
        """One interior-point solve (oracle/ip_ref.py IPRef.solve restated in C++):
        returns x, lam, dict(status, iter, trials, err, f)."""
        x = np.ascontiguousarray(np.array(x, dtype=np.float64))
        p = np.ascontiguousarray(np.asarray(p, dtype=np.float64))
        lam = np.zeros(self.m) if lam0 is None else np.ascontiguousarray(np.array(lam0, dtype=np.float64))
        st = self._ip_settings(settings)
        stats = np.zeros(3, dtype=np.int32)
        ef = np.zeros(2)
        if lib().cpu_ip_solve(self.h, _d(p), _d(x), _d(lam), int(lam0 is not None), _d(st), _i(stats), _d(ef)) != 0:
            raise ValueError("the interior-point restatement needs include_acc=True")
        return x, lam, dict(status=int(stats[0]), iter=int(stats[1]), trials=int(stats[2]), err=float(ef[0]),
                            f=float(ef[1]))

    def ip_mpc(self, P, X, XS, T0, steps, threads=0, settings=None):
        """`steps` MPC steps of every problem with the interior point (settings mpc_lam=True:
        lam_g carried, the Opti branch; default False: cold multipliers per solve, the
        reference's default compiled-solver driver);
        returns (wall seconds, final states, stats [B][steps][2] = (status, iterations))."""
        B = P.shape[0]
        P, X, XS = (np.ascontiguousarray(a, dtype=np.float64) for a in (P, X, XS))
        T0 = np.ascontiguousarray(T0, dtype=np.float64)
        xs = np.zeros((B, self.nx))
        stats = np.zeros((B, steps, 2), dtype=np.int32)
        st = self._ip_settings(settings)
        wall = lib().cpu_ip_mpc_batch(self.h, B, _d(P), _d(X), _d(XS), _d(T0), steps, threads, _d(st), _d(xs),
                                      _i(stats))
        return wall, xs, stats

    def __del__(self):
        try:
            if getattr(self, "h", None) and _lib is not None:
                _lib.cpu_destroy(self.h)
        except Exception:  # noqa: BLE001
            pass
