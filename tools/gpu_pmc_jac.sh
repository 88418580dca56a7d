#!/bin/bash
# SQ instruction-mix / stall counters of k_eval_jac at the headline config (separate --pmc passes)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VMEM"
P3="SQ_WAIT_INST_LDS SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM SQ_WAVES SQ_INSTS_BRANCH"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $P --kernel-include-regex k_eval_jac --output-format csv -d gpurun_out/jq$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --batch 256 > gpurun_out/jq$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/jq$i.log; }
done
python - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float)
for f in sorted(glob.glob("gpurun_out/jq*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(tot.items()):
    print(f"{k:28s} {v:16.0f}")
PY
