"""Print pl_ocp_sizes for the bench workload (B2G whole_body_rnea N=50, B=1024)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "pino-locoman_amd"))
from pinoloco import robots  # noqa: E402
from pinoloco.ocp import BatchedOCP  # noqa: E402
from pinoloco.synthetic import build_batch  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
R = robots.ROBOTS["b2g"]()
R.set_gait_sequence("trot", 0.8)
lay, P, X, XS, T0 = build_batch(R, "whole_body_rnea", 50, B, 0)
bo = BatchedOCP(R, "whole_body_rnea", 50, batch=B, device=0)
bo.set_params(P)
bo.set_x(X)
bo.init_solver()
print(os.environ.get("PINOLOCO_LIB", "in-tree"), bo.sizes())
