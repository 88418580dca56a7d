"""F64 flops per Lagrangian-Hessian evaluation (every k_lag_hess_* kernel of one evaluation) from a rocprofv3 --pmc pass (tools/gpu_hess_pmc.sh pass 3:
SQ_INSTS_VALU_FMA_F64, SQ_INSTS_VALU_MUL_F64, SQ_INSTS_VALU_ADD_F64 are wave-level instruction
counts: flops = 64 lanes x (2 FMA + MUL + ADD)), keyed to the Hessian sources (bench.py
hess_source_sha) so bench.py never applies it to another kernel revision.

Usage: python tools/hess_flops.py <pmc dir> <out json> <batch> <nodes> <mapping>
"""
import csv
import collections
import glob
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))


def main():
    d, out, batch, nodes, mapping = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_lag_hess" not in r["Kernel_Name"]:
                continue
            per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        raise SystemExit("no k_lag_hess dispatches")
    # one Hessian evaluation = one dispatch of each of its kernels (k_lag_hess_tree / _vv / _lin /
    # _cone for the rnea family, k_lag_hess_pb otherwise): total flops over the evaluations
    names = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_lag_hess" in r["Kernel_Name"]:
                names[r["Dispatch_Id"]] = r["Kernel_Name"]
    n_eval = max(collections.Counter(names[k] for k in per).values())
    tot = sum(64.0 * (2 * c["SQ_INSTS_VALU_FMA_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_ADD_F64"])
              for c in per.values())
    fl = [tot / n_eval] * n_eval
    import bench
    rec = {"flops_per_launch": sum(fl) / len(fl), "dispatches": len(fl), "batch": batch, "nodes": nodes,
           "workload": f"b2g whole_body_rnea N={nodes} MPC step", "mapping": mapping, "src_sha": bench.hess_source_sha(),
           "counters": "SQ_INSTS_VALU_{FMA,MUL,ADD}_F64 x 64 lanes (FMA = 2 flops), executed instructions"}
    json.dump(rec, open(out, "w"), indent=1)
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
