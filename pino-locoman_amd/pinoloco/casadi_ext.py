"""CasADi external-function bridge.

The reference can swap its CasADi data functions for generated code loaded with
``ca.external`` (optimization/ocp.py:299-302)::

    self.sqp_data = ca.external("sqp_data", "codegen/sqp/libsqp_data_b2_waj_N30.so")

libpinoloco.so exports ``sqp_data``, ``f_data``, ``g_data``, ``hess_data`` and
``retract_solution`` with CasADi's generated-code calling convention
(include/pinoloco_casadi.h).  After :func:`bind` the same line works with
``library_path()``, and the evaluations run on the GPU::

    from pinoloco import casadi_ext
    casadi_ext.bind(ocp)                      # the OCP built by make_ocp(...)
    self.sqp_data = ca.external("sqp_data", casadi_ext.library_path())

:class:`ExternalFunction` drives the same symbols through ctypes exactly as CasADi
does (n_in / n_out / work / sparsity / call); the tests use it, and so can callers
without casadi.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import scipy.sparse as sp

from . import _lib

FUNCTIONS = ("sqp_data", "f_data", "g_data", "hess_data", "retract_solution", "compiled_solver")


def library_path() -> str:
    return _lib.LIB_PATH


def bind(ocp, retract_steps: int = 3) -> None:
    """Bind the OCP whose shapes the exported functions describe.  `ocp` is an
    ``OCP`` (make_ocp) or a ``BatchedOCP``; evaluations use problem slot 0 of its
    device handle.  retract_steps = num_steps of compile_solution (default 3)."""
    h = getattr(getattr(ocp, "_backend", ocp), "h")
    _lib.check(_lib.lib().pl_casadi_bind(h, int(retract_steps)))


def bind_compiled(ocp, warm_start: bool = True) -> None:
    """Bind the interior-point OCP whose solve the exported ``compiled_solver`` runs: the
    reference's ``ocp.compile_solver(warm_start)`` (ocp_whole_body_rnea.py:237-258) as a library
    symbol, loadable the way run_mpc.py:51-53 loads the generated one::

        casadi_ext.bind_compiled(ocp, warm_start=True)   # ocp = make_ocp(..., solver="fatrop")
        solver_function = ca.external("compiled_solver", casadi_ext.library_path())

    `ocp` is an ``OCP`` with the fatrop solver (batch 1); the parameters the function does not
    take keep their current values, and without warm_start x starts from the OCP's initial guess."""
    be = getattr(ocp, "_backend", ocp)
    if hasattr(ocp, "param_vector"):  # the values the function bakes in (Opti's at to_function)
        be.set_params(np.asarray(ocp.param_vector(), dtype=np.float64)[None, :])
    x0 = getattr(ocp, "_x_initial", None)
    x0 = None if x0 is None else np.ascontiguousarray(np.asarray(x0, dtype=np.float64).ravel())
    if not warm_start and x0 is None:
        raise ValueError("bind_compiled(warm_start=False) needs an OCP with an initial guess")
    _lib.check(_lib.lib().pl_casadi_bind_compiled(be.h, int(bool(warm_start)),
                                                  None if x0 is None else x0.ctypes.data_as(C.c_void_p)))


def unbind() -> None:
    _lib.lib().pl_casadi_unbind()


class ExternalFunction:
    """Call NAME from libpinoloco.so the way CasADi's ``external`` does."""

    def __init__(self, name: str):
        if name not in FUNCTIONS:
            raise ValueError(f"unknown external function {name!r}")
        L = _lib.lib()
        self.name = name
        self._f = getattr(L, name)
        self._f.restype = C.c_int
        self._f.argtypes = [C.POINTER(C.POINTER(C.c_double)), C.POINTER(C.POINTER(C.c_double)),
                            C.POINTER(C.c_longlong), C.POINTER(C.c_double), C.c_int]
        for suffix in ("n_in", "n_out"):
            fn = getattr(L, f"{name}_{suffix}")
            fn.restype, fn.argtypes = C.c_longlong, []
        for suffix in ("sparsity_in", "sparsity_out"):
            fn = getattr(L, f"{name}_{suffix}")
            fn.restype, fn.argtypes = C.POINTER(C.c_longlong), [C.c_longlong]
        work = getattr(L, f"{name}_work")
        work.restype = C.c_int
        work.argtypes = [C.POINTER(C.c_longlong)] * 4
        self.n_in = int(getattr(L, f"{name}_n_in")())
        self.n_out = int(getattr(L, f"{name}_n_out")())
        sz = [C.c_longlong() for _ in range(4)]
        if work(*[C.byref(s) for s in sz]) != 0:
            raise _lib.PinolocoError(f"{name}_work failed")
        self.sz_arg, self.sz_res, self.sz_iw, self.sz_w = (int(s.value) for s in sz)
        self.sp_in = [self._sparsity(getattr(L, f"{name}_sparsity_in"), i) for i in range(self.n_in)]
        self.sp_out = [self._sparsity(getattr(L, f"{name}_sparsity_out"), i) for i in range(self.n_out)]

    @staticmethod
    def _sparsity(fn, i):
        p = fn(i)
        if not p:
            raise _lib.PinolocoError(_lib.lib().pl_last_error().decode() or "no sparsity")
        nrow, ncol = int(p[0]), int(p[1])
        colind = np.array([p[2 + k] for k in range(ncol + 1)], dtype=np.int64)
        nnz = int(colind[-1])
        row = np.array([p[3 + ncol + k] for k in range(nnz)], dtype=np.int64)
        return nrow, ncol, colind, row

    def __call__(self, *args):
        if len(args) != self.n_in:
            raise ValueError(f"{self.name} takes {self.n_in} inputs")
        ins = []
        for a, (nrow, ncol, colind, row) in zip(args, self.sp_in):
            v = np.ascontiguousarray(np.asarray(a, dtype=np.float64).reshape(-1, order="F"))
            if v.size != colind[-1]:
                raise ValueError(f"{self.name}: input of {v.size} values, sparsity has {colind[-1]}")
            ins.append(v)
        outs = [np.zeros(int(colind[-1])) for (_, _, colind, _) in self.sp_out]
        arg = (C.POINTER(C.c_double) * max(self.sz_arg, 1))(*[_lib.dptr(v) for v in ins])
        res = (C.POINTER(C.c_double) * max(self.sz_res, 1))(*[_lib.dptr(v) for v in outs])
        iw = (C.c_longlong * max(self.sz_iw, 1))()
        w = (C.c_double * max(self.sz_w, 1))()
        if self._f(arg, res, iw, w, 0) != 0:
            raise _lib.PinolocoError(f"{self.name} failed: {_lib.lib().pl_last_error().decode()}")
        result = []
        for v, (nrow, ncol, colind, row) in zip(outs, self.sp_out):
            if colind[-1] == nrow * ncol:  # dense (column-major)
                result.append(v.reshape((nrow, ncol), order="F"))
            else:
                result.append(sp.csc_matrix((v, row, colind), shape=(nrow, ncol)))
        return result
