#!/bin/bash
# SQ instruction-mix / stall counters of k_lag_hess (interior-point Hessian) at B2G rnea N=50,
# B = 1024 (or the third argument), one IP MPC step (separate --pmc passes), plus its rocprof kernel stats and the F64
# flops per evaluation (tools/hess_flops.py).  Usage: bash tools/gpu_hess_pmc.sh <tag> [batch]
set -o pipefail
export TMPDIR=/tmp
T=${1:-r04_hess}
O=gpurun_out/$T
mkdir -p $O
MAP=sweep
BATCH=${2:-1024}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --solver fatrop --steps 1 --warmup 0 --no-cpu-baseline --batch $BATCH --host-io-steps 0 > $O/prof.log 2>&1 || { echo "prof failed"; tail -5 $O/prof.log; exit 1; }
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
P2="SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VMEM"
P3="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INST_CYCLES_VMEM SQ_WAVES SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_SMEM"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-include-regex k_lag_hess --output-format csv -d $O/q$i -o run -- python3 bench.py --solver fatrop --steps 1 --warmup 0 --no-cpu-baseline --batch $BATCH --host-io-steps 0 > $O/q$i.log 2>&1 || { echo "pass $i failed"; tail -3 $O/q$i.log; }
done
python - "$O" <<'PY'
import csv, glob, collections, sys, json
O = sys.argv[1]
tot = collections.defaultdict(float)
for f in sorted(glob.glob(f"{O}/q*/**/*counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        tot[r["Counter_Name"]] += float(r["Counter_Value"])
for k, v in sorted(tot.items()):
    print(f"{k:28s} {v:16.0f}")
json.dump(tot, open(f"{O}/summary.json", "w"), indent=1)
PY
python tools/hess_flops.py $O/q3 $O/hess_flops.json $BATCH 50 $MAP
