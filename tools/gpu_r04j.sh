#!/bin/bash
# k_eval_jac_lin (rnea a / f columns from a primal pass): Jacobian and step parity, then the
# per-kernel A/B against PL_JAC_LIN=0 under rocprofv3 at the headline, and the IP parity tests.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04j}
O=gpurun_out/$T
cd "$R" && mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu.py -k "eval_sqp_data or sqp_step or mpc_loop or full_size or casadi" > $O/pytest_jac.log 2>&1 || { tail -30 $O/pytest_jac.log; exit 1; }
tail -2 $O/pytest_jac.log
for v in 1 0; do
  PL_JAC_LIN=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_lin$v" -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-io-steps 0 > $O/bench_lin$v.log 2>&1 || { tail -20 $O/bench_lin$v.log; exit 1; }
  grep '^{' $O/bench_lin$v.log | tail -1 | cut -c1-200
  grep -E "k_eval_jac" $O/prof_lin$v/run_kernel_stats.csv | cut -d, -f1-4
done
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ip.py > $O/pytest_ip.log 2>&1 || { tail -30 $O/pytest_ip.log; exit 1; }
tail -2 $O/pytest_ip.log
