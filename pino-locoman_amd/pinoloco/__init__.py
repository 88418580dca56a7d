"""pinoloco: MI355X-native batched MPC inner loop (OSQP-SQP path of pino-locoman).

Public surface mirrors the reference: ``make_ocp``/``OCP_ARGS``
(optimization/ocp_factory.py, ocp_args.py), robots (utils/robot.py) and gait
tables (utils/gait_sequence.py).  The compute path is libpinoloco.so (HIP, gfx950).
"""
from .gait import GaitSequence, get_spline_vel_z, horizon_dts  # noqa: F401
from .robots import B2, B2G, Go2, ROBOTS  # noqa: F401

__all__ = ["GaitSequence", "get_spline_vel_z", "horizon_dts", "Go2", "B2", "B2G", "ROBOTS",
           "make_ocp", "OCP_ARGS", "BatchedOCP"]


def __getattr__(name):
    if name in ("make_ocp", "OCP_ARGS", "BatchedOCP", "OCP"):
        from . import ocp
        return getattr(ocp, name)
    raise AttributeError(name)
