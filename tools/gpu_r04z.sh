#!/bin/bash
# Base-position columns as constants (rows.h seed_pos): parity (Jacobian, steps, loops, IP, CasADi),
# the headline Jacobian times, the IP line with its CPU baseline under rocprofv3, Hessian flops.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04z}
O=gpurun_out/$T
cd "$R" && mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu.py tests/test_ip.py tests/test_casadi_ext.py tests/test_graph_gpu.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/head" -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-io-steps 0 > $O/head.log 2>&1 || { tail -5 $O/head.log; exit 1; }
grep '^{' $O/head.log | tail -1 | cut -c1-200; grep -E "eval_jac" $O/head/run_kernel_stats.csv | cut -d, -f1-4
bash tools/gpu_hess_pmc.sh $T/hess pb 1024 > $O/hess_pmc.log 2>&1; tail -1 $O/hess_pmc.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_ip" -o run -- python3 bench.py --solver fatrop --steps 3 --warmup 1 --host-io-steps 0 > $O/prof_ip.log 2>&1 || { tail -20 $O/prof_ip.log; exit 1; }
grep '^{' $O/prof_ip.log | tail -1 | cut -c1-1500
head -8 $O/prof_ip/run_kernel_stats.csv | cut -c1-140
