#!/bin/bash
# Chain-confined Hessian passes (tree_pass only_ch in k_lag_hess_pb / k_lag_hess_lin): IP parity
# tests, the IP bench line under rocprofv3 with PL_HESS_CHAIN=1 and 0, the Hessian's F64 flops.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04h}
O=gpurun_out/$T
cd "$R" && mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ip.py -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_ip.log 2>&1 || { tail -30 $O/pytest_ip.log; exit 1; }
tail -2 $O/pytest_ip.log
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -k "eval_sqp_data or sqp_step" > $O/pytest_jac.log 2>&1 || { tail -30 $O/pytest_jac.log; exit 1; }
tail -2 $O/pytest_jac.log
for v in 1 0; do
  PL_HESS_CHAIN=$v timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_ip$v" -o run -- python3 bench.py --solver fatrop --steps 2 --warmup 1 --host-io-steps 0 --no-cpu-baseline > $O/prof_ip$v.log 2>&1 || { tail -20 $O/prof_ip$v.log; exit 1; }
  grep '^{' $O/prof_ip$v.log | tail -1 | cut -c1-300
  head -5 $O/prof_ip$v/run_kernel_stats.csv | cut -c1-140
done
bash tools/gpu_hess_pmc.sh $T/hess pb 1024 > $O/hess_pmc.log 2>&1; tail -2 $O/hess_pmc.log
