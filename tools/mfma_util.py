"""Summarise the MFMA pass of tools/gpu_mfma.sh: per factor kernel, F64 MFMA flops
(SQ_INSTS_VALU_MFMA_MOPS_F64 x 512, rocprofv3's derived FLOPS_F64 expression), the
achieved TFLOP/s over the dispatch duration, the fraction of the gfx950 dense F64
matrix peak, and MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs).
Usage: python tools/mfma_util.py PMC_DIR OUT_JSON"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

PEAK_F64_MATRIX_TFLOPS = 78.6  # MI355X dense F64 matrix spec (no sparsity)
SIMDS = 1024
XCDS = 8


def main(d, out):
    pmc = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    kt = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not pmc:
        sys.exit(f"no counter_collection.csv under {d}")
    acc = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for path in pmc:
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"].split("(")[0]
                kk = "k_fnode" if "k_fnode" in k else ("k_fchain" if "k_fchain" in k else k)
                acc[kk][r["Counter_Name"]] += float(r["Counter_Value"])
                disp[kk].add(r["Dispatch_Id"])
    dur = defaultdict(float)
    for path in kt:
        with open(path) as f:
            for r in csv.DictReader(f):
                k = r["Kernel_Name"]
                kk = "k_fnode" if "k_fnode" in k else ("k_fchain" if "k_fchain" in k else None)
                if kk:
                    dur[kk] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
    res = {}
    for k, c in acc.items():
        flops = c["SQ_INSTS_VALU_MFMA_MOPS_F64"] * 512
        t = dur.get(k, 0.0)
        gui = c["GRBM_GUI_ACTIVE"] / XCDS  # summed over the 8 XCDs
        res[k] = dict(dispatches=len(disp[k]), seconds=t, mfma_f64_flops=flops,
                      mfma_f64_tflops=flops / t * 1e-12 if t else None,
                      frac_of_f64_matrix_peak=flops / t * 1e-12 / PEAK_F64_MATRIX_TFLOPS if t else None,
                      mfma_busy_frac=c["SQ_VALU_MFMA_BUSY_CYCLES"] / (gui * SIMDS) if gui else None,
                      valu_f64_fma=c["SQ_INSTS_VALU_FMA_F64"], valu_f64_add=c["SQ_INSTS_VALU_ADD_F64"],
                      valu_f64_mul=c["SQ_INSTS_VALU_MUL_F64"], mfma_f64_insts=c["SQ_INSTS_VALU_MFMA_F64"],
                      waves=c["SQ_WAVES"], counters=dict(c))
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    for k, r in res.items():
        print(k, {x: r[x] for x in ("dispatches", "seconds", "mfma_f64_tflops", "frac_of_f64_matrix_peak",
                                    "mfma_busy_frac")})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
