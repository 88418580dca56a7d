"""Generate the shipped model tables (pinoloco/models/*.json) from the reference URDF/SRDF.

Run in the build container (the reference is mounted read-only at /root/reference):

    python tools/gen_models.py [/root/reference]

The URDF/SRDF files are read as data; only the derived tables are committed.
Mirrors ``utils/robot.py:45-118``: Go2 and B2 load as-is, B2G locks the gripper
(joint 20) and, for ``ignore_arm``, joints 14..20.
"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pino-locoman_amd"))

from pinoloco import model as mdl  # noqa: E402


def build(ref, robot, lock=None):
    urdf = os.path.join(ref, "robots", f"{robot}_description", "urdf", f"{robot}.urdf")
    srdf = os.path.join(ref, "robots", f"{robot}_description", "srdf", f"{robot}.srdf")
    m = mdl.build_model_from_urdf(urdf)
    if lock:
        m = mdl.build_reduced_model(m, lock)
    mdl.load_reference_configurations(m, srdf)
    return m


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    out = os.path.join(HERE, "..", "pino-locoman_amd", "pinoloco", "models")
    os.makedirs(out, exist_ok=True)
    specs = {
        "go2": ("go2", None),
        "b2": ("b2", None),
        "b2g": ("b2g", [20]),
        "b2g_noarm": ("b2g", list(range(14, 21))),
    }
    for name, (robot, lock) in specs.items():
        m = build(ref, robot, lock)
        m.save(os.path.join(out, f"{name}.json"))
        print(f"{name}: nq={m.nq} nv={m.nv} njoints={m.njoints} nframes={len(m.frames)} "
              f"mass={m.total_mass():.6f} poses={list(m.reference_configurations)}")


if __name__ == "__main__":
    main()
