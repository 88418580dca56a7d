#!/bin/bash
# One bench line per BASELINE config, each run once under rocprofv3 --kernel-trace --stats (the
# JSON line and the per-kernel CSV come from the same command, so every line's roofline
# avg_launch_ms reproduces from its CSV), and the MFMA counter pass on the block factor.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04c}
O=gpurun_out/$T
cd "$R" && mkdir -p "$O"
export TMPDIR=/tmp
: > $O/configs.jsonl
run() {
  local tag=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/$tag" -o run -- python3 bench.py "$@" > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  grep '^{' $O/$tag.log | tail -1 >> $O/configs.jsonl
  grep '^{' $O/$tag.log | tail -1 | cut -c1-220
}
run cfg1_go2_cv_n20_b1024 --robot go2 --dynamics centroidal_vel --nodes 20 --batch 1024 --steps 40 --warmup 2
run cfg2_go2_rnea_n20_b1 --robot go2 --dynamics whole_body_rnea --nodes 20 --batch 1 --steps 40 --warmup 2
run cfg3_b2_aba_n40_b256 --robot b2 --dynamics whole_body_aba --nodes 40 --batch 256 --steps 40 --warmup 2
run cfg4_b2g_acc_n50_b1024 --robot b2g --dynamics whole_body_acc --nodes 50 --batch 1024 --steps 20 --warmup 2
P="SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex 'k_fnode|k_fchain' --output-format csv -d "$R/$O/pmc_mfma" -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --host-io-steps 0 > $O/pmc_mfma.log 2>&1 || { echo "mfma pass failed"; tail -3 $O/pmc_mfma.log; exit 1; }
python tools/mfma_util.py $O/pmc_mfma $O/mfma_util.json && cat $O/mfma_util.json | head -30
