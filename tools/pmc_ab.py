"""Compare per-launch PMC counters of k_admm between two builds (tools/gpu_pmc_ab.sh output).

Usage: python tools/pmc_ab.py DIR   (DIR holds old_sq, old_tcp, new_sq, new_tcp)
"""
import csv
import glob
import os
import sys


def per_launch(d, kernel="k_admm<"):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if kernel not in r.get("Kernel_Name", ""):
                    continue
                key = (r["Counter_Name"], r.get("Dispatch_Id") or r.get("Correlation_Id"))
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    out = {}
    for (c, _), v in vals.items():
        out.setdefault(c, []).append(v)
    return {c: sum(v) / len(v) for c, v in out.items()}


def main():
    d = sys.argv[1]
    res = {}
    for v in ("old", "new"):
        res[v] = {}
        for p in ("sq", "tcp"):
            res[v].update(per_launch(os.path.join(d, f"{v}_{p}")))
    for c in sorted(set(res["old"]) | set(res["new"])):
        a, b = res["old"].get(c), res["new"].get(c)
        ratio = f"{b / a:.3f}" if a and b else "-"
        print(f"{c:36s} old {a:16.4g} new {b:16.4g} new/old {ratio}")


if __name__ == "__main__":
    main()
