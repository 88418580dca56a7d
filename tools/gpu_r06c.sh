#!/bin/bash
# r06: ADMM mapping per config (sweep / sweep2 / chain forced at the config's batch), the
# factor's MFMA utilisation on the current sources, and the k_admm HBM traffic passes.
set -o pipefail
mkdir -p gpurun_out/r06c
export TMPDIR=/tmp
O=gpurun_out/r06c
: > $O/kernels.jsonl
for cfg in "--robot go2 --dynamics centroidal_vel --nodes 20 --batch 1024" \
           "--robot b2 --dynamics whole_body_aba --nodes 40 --batch 256" \
           "--robot b2g --dynamics whole_body_acc --nodes 50 --batch 1024" \
           "--robot b2g --dynamics whole_body_rnea --nodes 50 --batch 1024"; do
  for k in sweep sweep2 chain; do
    timeout -k 10 300 python bench.py $cfg --admm-kernel $k --steps 10 --warmup 2 --no-cpu-baseline --host-io-steps 0 > $O/k.log 2>&1
    rc=$?
    if [ $rc -eq 0 ]; then tail -1 $O/k.log >> $O/kernels.jsonl; else echo "{\"cfg\": \"$cfg\", \"kernel\": \"$k\", \"rc\": $rc, \"err\": \"$(tail -1 $O/k.log | tr -d '\"')\"}" >> $O/kernels.jsonl; fi
    case "$rc" in 0|1) ;; *) exit 1;; esac
  done
done
P="SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc $P --kernel-include-regex 'k_fnode|k_fchain' --output-format csv -d "$PWD/$O/pmc_mfma" -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --host-io-steps 0 > $O/pmc_mfma.log 2>&1 || exit 1
python tools/mfma_util.py $O/pmc_mfma $O/mfma_util.json > $O/mfma_util.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_admm<' --output-format csv -d "$PWD/$O/pmc_fetch" -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --host-io-steps 0 > $O/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_admm<' --output-format csv -d "$PWD/$O/pmc_write" -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --host-io-steps 0 > $O/pmc_write.log 2>&1 || exit 1
python tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/pmc_fetch.log $O/admm_traffic.json > $O/pmc_traffic.log 2>&1
echo done
