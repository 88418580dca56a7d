#!/bin/bash
# MFMA counters of the factor chain on configs 1 and 3 (the E_{i+1} = Wc S Wc^T MFMA path)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04u}
O=gpurun_out/$T
cd "$R" && mkdir -p "$O"
export TMPDIR=/tmp
P="SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex 'k_fnode|k_fchain' --output-format csv -d "$R/$O/pmc_cfg3" -o run -- python3 bench.py --robot b2 --dynamics whole_body_aba --nodes 40 --batch 256 --steps 2 --warmup 0 --no-cpu-baseline --host-io-steps 0 > $O/pmc_cfg3.log 2>&1 || { echo "cfg3 pass failed"; tail -3 $O/pmc_cfg3.log; exit 1; }
python tools/mfma_util.py $O/pmc_cfg3 $O/mfma_util_cfg3.json && head -12 $O/mfma_util_cfg3.json
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex 'k_fnode|k_fchain' --output-format csv -d "$R/$O/pmc_cfg1" -o run -- python3 bench.py --robot go2 --dynamics centroidal_vel --nodes 20 --batch 1024 --steps 2 --warmup 0 --no-cpu-baseline --host-io-steps 0 > $O/pmc_cfg1.log 2>&1 || { echo "cfg1 pass failed"; tail -3 $O/pmc_cfg1.log; exit 1; }
python tools/mfma_util.py $O/pmc_cfg1 $O/mfma_util_cfg1.json && head -12 $O/mfma_util_cfg1.json
