"""Per-launch HBM traffic of k_admm from rocprofv3 --pmc passes.

Usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR BENCH_LOG OUT.json

BENCH_LOG is the output of the bench.py command the passes profiled, run with
--warmup 0 so every k_admm launch lies inside its timed region: its JSON line gives
the problem-iterations those launches executed, and the result is stored per
problem-iteration (bench.py scales it to its own launches), keyed to the sha256 of
the k_admm sources (bench.traffic_source_sha) so a stale measurement is never used.

FETCH_DIR holds the counter_collection.csv of a `--pmc FETCH_SIZE` pass and
WRITE_DIR that of a `--pmc WRITE_SIZE` pass (separate passes: the two do not fit
one TCC pass on gfx950).  Per MI355X_MICROARCH.md ("HBM / rocprofv3"): FETCH_SIZE
and WRITE_SIZE are in KB; on gfx950 FETCH_SIZE reports half of the bytes of a wide
coalesced streaming read, so it is doubled; WRITE_SIZE is taken as is.
"""
import csv
import glob
import json
import os
import sys


def _rows(d):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    out = []
    for f in files:
        with open(f) as fh:
            out.extend(csv.DictReader(fh))
    return out


def per_launch(d, counter, kernel="k_admm<"):  # not k_admm_init
    vals = {}
    for r in _rows(d):
        if r.get("Counter_Name") != counter or kernel not in r.get("Kernel_Name", ""):
            continue
        key = r.get("Dispatch_Id") or r.get("Correlation_Id")
        vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} in {d}")
    v = sorted(vals.values())
    return sum(v) / len(v), len(v)


def bench_line(path):
    with open(path) as fh:
        for line in reversed(fh.read().splitlines()):
            if line.startswith("{"):
                return json.loads(line)
    raise SystemExit(f"no JSON line in {path}")


def main():
    fdir, wdir, blog, out = sys.argv[1:5]
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from bench import traffic_source_sha  # noqa: E402
    fetch_kb, nf = per_launch(fdir, "FETCH_SIZE")
    write_kb, nw = per_launch(wdir, "WRITE_SIZE")
    fetch_b = 2.0 * fetch_kb * 1024.0  # gfx950: FETCH_SIZE = half the streamed bytes
    write_b = write_kb * 1024.0
    bl = bench_line(blog)
    rf = bl["roofline"]
    if rf["launches"] != nf:
        raise SystemExit(f"bench timed {rf['launches']} k_admm launches, the PMC pass saw {nf}: run it with --warmup 0")
    iters = rf["problem_iters_per_launch"]
    res = {"kernel": "k_admm", "src_sha": traffic_source_sha(), "batch": bl["config"]["batch_per_gpu"],
           "nodes": bl["config"]["nodes"], "workload": bl["config"]["workload"],
           "fetch_size_kb_raw": fetch_kb, "write_size_kb_raw": write_kb,
           "fetch_bytes_corrected": fetch_b, "write_bytes": write_b,
           "bytes_per_launch": fetch_b + write_b, "launches_fetch": nf, "launches_write": nw,
           "problem_iters_per_launch": iters, "bytes_per_problem_iter": (fetch_b + write_b) / iters,
           "algorithmic_bytes_per_problem_iter": rf["bytes_per_problem_iter"],
           "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), KB->B x1024; WRITE_SIZE as is"}
    os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
