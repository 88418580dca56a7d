#!/bin/bash
# MFMA utilisation of the block factor (k_fnode / k_fchain): one --pmc pass with the
# kernel trace (8 SQ + 1 GRBM counters), summarised by tools/mfma_util.py.
# Usage (on the box): bash tools/gpu_mfma.sh
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
P="SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex 'k_fnode|k_fchain' --output-format csv -d "$R/gpurun_out/pmc_mfma" -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_mfma.log 2>&1 || exit 1
python tools/mfma_util.py gpurun_out/pmc_mfma gpurun_out/mfma_util.json
