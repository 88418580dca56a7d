#!/bin/bash
# Same-box PMC A/B of two library builds (ab/lib_old.so, ab/lib_new.so) on the headline bench:
# one SQ + TA pass and one TCP pass per build (separate runs, within the per-block limits),
# no trace domains.  python tools/pmc_ab.py gpurun_out/r06q then compares k_admm per launch.
set -o pipefail
export TMPDIR=/tmp
O=$PWD/gpurun_out/r06q
mkdir -p $O
B="bench.py --steps 2 --warmup 0 --no-cpu-baseline --host-io-steps 0"
for v in old new; do
  export PINOLOCO_LIB=$PWD/ab/lib_$v.so
  timeout -s KILL 150 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum --output-format csv -d $O/${v}_sq -o run -- python3 $B > $O/${v}_sq.log 2>&1 || { tail -5 $O/${v}_sq.log; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum --output-format csv -d $O/${v}_tcp -o run -- python3 $B > $O/${v}_tcp.log 2>&1 || { tail -5 $O/${v}_tcp.log; exit 1; }
done
echo done
