#!/bin/bash
# k_admm latency counters: average SMEM / LDS / instruction-fetch latency
# (SQ_INST_LEVEL_x / SQ_INSTS_x) and the LDS wait share, one --pmc pass each.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
P1="SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_IFETCH SQ_IFETCH_LEVEL"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex 'k_admm<' --output-format csv -d gpurun_out/lat$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/lat$i.log 2>&1 || exit 1
done
