import os
import sys

import numpy as np
import pytest

ROOT = os.path.normpath(os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
for p in (ROOT, os.path.join(ROOT, "pino-locoman_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs the product path via the C-ABI")
    config.addinivalue_line("markers", "slow: CPU test that takes more than a few seconds")


def golden(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def make_robot(name, gait="trot", period=0.8):
    from pinoloco import robots
    R = robots.ROBOTS[name]()
    R.set_gait_sequence(gait, period)
    return R


@pytest.fixture(scope="session")
def hip_available():
    """True when a HIP device is visible; GPU tests fail (not skip) without one."""
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False
