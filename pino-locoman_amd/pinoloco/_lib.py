"""ctypes binding of libpinoloco.so (include/pinoloco.h).

Loads the in-tree HIP extension and fails loudly when it is missing: there is no
CPU fallback on the product path.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# PINOLOCO_LIB: load another build of the same sources (kernel A/B experiments)
LIB_PATH = os.environ.get("PINOLOCO_LIB") or os.path.join(HERE, "libpinoloco.so")

_dp = C.POINTER(C.c_double)
_ip = C.POINTER(C.c_int)


class ModelDesc(C.Structure):
    _fields_ = [("njoints", C.c_int), ("nq", C.c_int), ("nv", C.c_int),
                ("parent", _ip), ("jtype", _ip), ("axis", _dp), ("placement_R", _dp), ("placement_p", _dp),
                ("mass", _dp), ("lever", _dp), ("inertia", _dp), ("gravity", _dp),
                ("nframes", C.c_int), ("frame_parent", _ip), ("frame_R", _dp), ("frame_p", _dp)]


class OcpDesc(C.Structure):
    _fields_ = [("dynamics", C.c_int), ("nodes", C.c_int), ("tau_nodes", C.c_int), ("include_acc", C.c_int),
                ("include_base", C.c_int), ("n_feet", C.c_int), ("foot_frames", C.c_int * 4),
                ("ext_force_frame", C.c_int), ("arm_ee_frame", C.c_int), ("base_frame", C.c_int),
                ("mu", C.c_double), ("q0", _dp), ("joint_pos_min", _dp), ("joint_pos_max", _dp),
                ("joint_vel_max", _dp), ("joint_torque_max", _dp),
                ("rho", C.c_double), ("sigma", C.c_double), ("alpha", C.c_double), ("eps_abs", C.c_double),
                ("eps_rel", C.c_double), ("eps_prim_inf", C.c_double), ("eps_dual_inf", C.c_double),
                ("max_iter", C.c_int), ("scaling", C.c_int), ("check_termination", C.c_int),
                ("warm_start", C.c_int), ("gait_type", C.c_int), ("gait_period", C.c_double),
                ("debug_paths", C.c_uint)]


# pl_ocp_desc.debug_paths bits (include/pinoloco.h PL_PATH_*): the earlier builds' paths the
# regression tests compare with, and the phase-timing instrumentation; 0 in production
PATHS = {"jac_dual_all": 1, "jac_const_every": 2, "hess_full_tree": 4, "hess_dual_all": 8, "fchain_list": 16,
         "ruiz_per_pass": 32, "no_mpc_graph": 64, "admm_timing": 128, "ip_refine_gather": 256,
         "hess_pairs": 512, "rc_one_group": 1024}


class Stats(C.Structure):
    _fields_ = [("status", C.c_int), ("admm_iters", C.c_int), ("ls_accepted", C.c_int), ("ls_branch", C.c_int),
                ("ls_trials", C.c_int), ("pad", C.c_int), ("ls_alpha", C.c_double), ("viol_max", C.c_double),
                ("pri_res", C.c_double), ("dua_res", C.c_double), ("f", C.c_double)]


class IpSettings(C.Structure):
    _fields_ = [("tol", C.c_double), ("mu_init", C.c_double), ("bound_push", C.c_double), ("bound_frac", C.c_double),
                ("delta_w", C.c_double), ("delta_c", C.c_double), ("max_iter", C.c_int), ("ls_max", C.c_int),
                ("n_refine", C.c_int), ("hessian", C.c_int)]


class IpStats(C.Structure):
    _fields_ = [("status", C.c_int), ("iter", C.c_int), ("ls_trials", C.c_int), ("nfilter", C.c_int),
                ("err", C.c_double), ("mu", C.c_double), ("alpha", C.c_double), ("alpha_z", C.c_double),
                ("f", C.c_double), ("viol_max", C.c_double), ("alphas", C.c_double * 32),
                ("ref_solves", C.c_int), ("pad", C.c_int)]


EXPORTS = {
    "pl_last_error": (C.c_char_p, []),
    "pl_version": (C.c_int, []),
    "pl_build_info": (C.c_char_p, []),
    "pl_model_create": (C.c_int, [C.POINTER(ModelDesc), C.POINTER(C.c_void_p)]),
    "pl_model_destroy": (None, [C.c_void_p]),
    "pl_ocp_create": (C.c_int, [C.c_void_p, C.POINTER(OcpDesc), C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    "pl_ocp_destroy": (None, [C.c_void_p]),
    "pl_ocp_dims": (C.c_int, [C.c_void_p, _ip, _ip, _ip, _ip]),
    "pl_ocp_pattern": (C.c_int, [C.c_void_p, _ip, _ip]),
    "pl_ocp_set_params": (C.c_int, [C.c_void_p, _dp]),
    "pl_ocp_get_params": (C.c_int, [C.c_void_p, _dp]),
    "pl_ocp_set_x": (C.c_int, [C.c_void_p, _dp]),
    "pl_ocp_get_x": (C.c_int, [C.c_void_p, _dp]),
    "pl_ocp_init_solver": (C.c_int, [C.c_void_p]),
    "pl_ocp_solve": (C.c_int, [C.c_void_p, C.POINTER(Stats), _dp]),
    "pl_ocp_set_sqp_iters": (C.c_int, [C.c_void_p, C.c_int]),
    "pl_ocp_set_solver": (C.c_int, [C.c_void_p, C.c_int]),
    "pl_ocp_set_admm_kernel": (C.c_int, [C.c_void_p, C.c_int]),
    "pl_ocp_get_admm_kernel": (C.c_int, [C.c_void_p]),
    "pl_ocp_get_admm_groups": (C.c_int, [C.c_void_p]),
    "pl_ocp_set_ip_settings": (C.c_int, [C.c_void_p, C.POINTER(IpSettings)]),
    "pl_ocp_ip_stats": (C.c_int, [C.c_void_p, C.POINTER(IpStats)]),
    "pl_ocp_get_lam": (C.c_int, [C.c_void_p, _dp]),
    "pl_ocp_set_lam": (C.c_int, [C.c_void_p, C.c_void_p]),
    "pl_debug_ip_direction": (C.c_int, [C.c_void_p, _dp, _dp, _dp, _dp, _dp]),
    "pl_casadi_bind": (C.c_int, [C.c_void_p, C.c_int]),
    "pl_casadi_unbind": (None, []),
    "pl_casadi_bind_compiled": (C.c_int, [C.c_void_p, C.c_int, C.c_void_p]),
    "pl_eval_sqp_data": (C.c_int, [C.c_void_p, _dp, _dp, _dp, _dp, _dp]),
    "pl_eval_f": (C.c_int, [C.c_void_p, _dp]),
    "pl_ocp_get_step": (C.c_int, [C.c_void_p, _dp]),
    "pl_mpc_setup": (C.c_int, [C.c_void_p, _dp, _dp]),
    "pl_mpc_step": (C.c_int, [C.c_void_p, C.c_int]),
    "pl_mpc_get_state": (C.c_int, [C.c_void_p, _dp]),
    "pl_mpc_get_stats": (C.c_int, [C.c_void_p, C.POINTER(Stats)]),
    "pl_mpc_export": (C.c_int, [C.c_void_p, C.c_void_p]),
    "pl_mpc_download": (C.c_int, [C.c_void_p, _dp]),
    "pl_ocp_profile_read_hess": (C.c_int, [C.c_void_p, _dp]),
    "pl_mpc_graph_info": (C.c_int, [C.c_void_p, C.POINTER(C.c_longlong)]),
    "pl_mpc_set_ip_lam": (C.c_int, [C.c_void_p, C.c_int]),
    "pl_ocp_sync": (C.c_int, [C.c_void_p]),
    "pl_state_integrate": (C.c_int, [C.c_void_p, _dp, _dp, _dp]),
    "pl_state_difference": (C.c_int, [C.c_void_p, _dp, _dp, _dp]),
    "pl_ocp_profile": (C.c_int, [C.c_void_p, C.c_int]),
    "pl_ocp_profile_read": (C.c_int, [C.c_void_p, _dp]),
    "pl_ocp_sizes": (C.c_int, [C.c_void_p, C.POINTER(C.c_longlong)]),
    "pl_debug_consts": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, _ip]),
    "pl_debug_get": (C.c_int, [C.c_void_p, C.c_char_p, _dp, C.c_longlong]),
    "pl_debug_set": (C.c_int, [C.c_void_p, C.c_char_p, _dp, C.c_longlong]),
    "pl_debug_nodes": (C.c_int, [C.c_void_p, _ip]),
    "pl_debug_admm": (C.c_int, [C.c_void_p, C.c_int, C.c_int]),
    "pl_dyn_create": (C.c_int, [C.c_void_p, _ip, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_void_p)]),
    "pl_dyn_destroy": (None, [C.c_void_p]),
    "pl_dyn_sizes": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _ip, _ip]),
    "pl_dyn_eval": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int, _dp, _dp, _dp, _dp, _dp]),
}

_lib = None


class PinolocoError(RuntimeError):
    pass


def lib():
    """Load libpinoloco.so (building it first if only the sources are present)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        from . import build as _build
        try:
            _build.build()
        except Exception as exc:  # noqa: BLE001
            raise PinolocoError(f"HIP extension {LIB_PATH} is missing and could not be built: {exc}") from exc
    L = C.CDLL(LIB_PATH)
    for name, (res, args) in EXPORTS.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def build_sha() -> str:
    """The sha256 of the sources the loaded library was built from (pl_build_info)."""
    info = lib().pl_build_info().decode()
    return info.split("pl_src_sha256=")[1].split()[0]


def check(rc):
    if rc != 0:
        raise PinolocoError(lib().pl_last_error().decode())
    return rc


def dptr(a: np.ndarray):
    assert a.dtype == np.float64 and a.flags.c_contiguous
    return a.ctypes.data_as(_dp)


def iptr(a: np.ndarray):
    assert a.dtype == np.int32 and a.flags.c_contiguous
    return a.ctypes.data_as(_ip)


class ModelHandle:
    """pl_model built from a pinoloco.model.Model."""

    def __init__(self, model):
        from .model import JT_FREEFLYER, JT_REVOLUTE
        nj = model.njoints
        self._keep = []

        def arr(x, dt=np.float64):
            a = np.ascontiguousarray(np.asarray(x, dtype=dt))
            self._keep.append(a)
            return a

        parent = arr([j.parent for j in model.joints], np.int32)
        jtype = arr([j.jtype for j in model.joints], np.int32)
        axis = arr(np.concatenate([j.axis for j in model.joints]))
        pR = arr(np.concatenate([j.placement.R.ravel() for j in model.joints]))
        pp = arr(np.concatenate([j.placement.p for j in model.joints]))
        mass = arr([Y.mass for Y in model.inertias])
        lever = arr(np.concatenate([Y.lever for Y in model.inertias]))
        inertia = arr(np.concatenate([Y.I.ravel() for Y in model.inertias]))
        grav = arr(model.gravity)
        fpar = arr([f.parent_joint for f in model.frames], np.int32)
        fR = arr(np.concatenate([f.placement.R.ravel() for f in model.frames]))
        fp = arr(np.concatenate([f.placement.p for f in model.frames]))
        assert JT_FREEFLYER == 1 and JT_REVOLUTE == 2
        d = ModelDesc(nj, model.nq, model.nv, iptr(parent), iptr(jtype), dptr(axis), dptr(pR), dptr(pp),
                      dptr(mass), dptr(lever), dptr(inertia), dptr(grav), len(model.frames), iptr(fpar),
                      dptr(fR), dptr(fp))
        h = C.c_void_p()
        check(lib().pl_model_create(C.byref(d), C.byref(h)))
        self.h = h
        self.nq, self.nv = model.nq, model.nv

    def integrate(self, x, dx):
        x = np.ascontiguousarray(np.asarray(x, dtype=np.float64).ravel())
        dx = np.ascontiguousarray(np.asarray(dx, dtype=np.float64).ravel())
        out = np.zeros(self.nq + self.nv)
        check(lib().pl_state_integrate(self.h, dptr(x), dptr(dx), dptr(out)))
        return out

    def difference(self, x0, x1):
        x0 = np.ascontiguousarray(np.asarray(x0, dtype=np.float64).ravel())
        x1 = np.ascontiguousarray(np.asarray(x1, dtype=np.float64).ravel())
        out = np.zeros(2 * self.nv)
        check(lib().pl_state_difference(self.h, dptr(x0), dptr(x1), dptr(out)))
        return out

    def __del__(self):
        try:
            if getattr(self, "h", None) and _lib is not None:
                _lib.pl_model_destroy(self.h)
        except Exception:  # noqa: BLE001
            pass
