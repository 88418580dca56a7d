"""bench.py contract pieces that run without a GPU: the rank launcher (--gpus N
spawns N ranks itself when no torchrun environment is present), the roofline byte
accounting and the revision check of the PMC traffic file."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT


@pytest.mark.slow
def test_gpus2_launches_two_ranks():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--dry-run", "--batch", "3",
                        "--robot", "go2", "--nodes", "6"], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["config"]["global_batch"] == 6 and out["gathered_rows"] == 6


def test_world_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "4", "--dry-run"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_admm_bytes_stored_triangle():
    import bench
    # node table columns: [nw, nu, x_off, row_off, nrow, ncol, ent_off, nent, ntile, nunit, s_off, ncpl]
    ntab = np.zeros((3, 12), dtype=np.int32)
    ntab[:, 0] = [10, 12, 4]
    ntab[:, 9] = [1, 2, 1]
    sz = {"nnz": 100, "n": 26, "m": 30}
    tri = np.array([55, 78, 10.0])
    want = 8 * (2 * tri.sum() - tri[0] - tri[-1] + 100 + 7 * 26 + 7 * 30)
    assert bench.admm_bytes_per_problem_iter(sz, ntab) == want
    blk = np.array([1, 2, 1]) * 64 * 16.0
    wantp = 8 * (2 * blk.sum() - blk[0] - blk[-1] + 100 + 7 * 26 + 7 * 30)
    assert bench.admm_bytes_per_problem_iter(sz, ntab, padded=True) == wantp


def test_traffic_file_is_revision_keyed(tmp_path, monkeypatch):
    import bench
    f = tmp_path / "t.json"
    rec = {"src_sha": bench.traffic_source_sha(), "batch": 8, "nodes": 5, "workload": "w",
           "bytes_per_problem_iter": 1.0}
    f.write_text(json.dumps(rec))
    monkeypatch.setattr(bench, "TRAFFIC_FILE", str(f))
    assert bench.measured_traffic(8, 5, "w")["bytes_per_problem_iter"] == 1.0
    assert bench.measured_traffic(16, 5, "w") is None
    rec["src_sha"] = "0" * 16
    f.write_text(json.dumps(rec))
    assert bench.measured_traffic(8, 5, "w") is None
