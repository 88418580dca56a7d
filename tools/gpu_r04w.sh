#!/bin/bash
# k_admm_rc with its chains on one wave (PL_RC_ONEWAVE, r04): chain-kernel parity, phase timing,
# configs 2 and 3 A/B against the workgroup-wide chains.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04w}
O=gpurun_out/$T
cd "$R" && mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu.py tests/test_admm_kernels.py tests/test_graph_gpu.py -k "chain or loop or graph or admm" > $O/pytest_chain.log 2>&1 || { tail -30 $O/pytest_chain.log; exit 1; }
tail -2 $O/pytest_chain.log
for v in 1 0; do
  PL_RC_ONEWAVE=$v timeout -k 10 120 python tools/gpu_rc_timing.py go2 whole_body_rnea 20 1 > $O/rc_timing_go2_$v.txt 2>&1 || { tail -5 $O/rc_timing_go2_$v.txt; exit 1; }
  cat $O/rc_timing_go2_$v.txt
done
for rep in 1 2; do
for v in 1 0; do
  PL_RC_ONEWAVE=$v timeout -k 10 200 python bench.py --robot go2 --dynamics whole_body_rnea --nodes 20 --batch 1 --steps 40 --warmup 2 --no-cpu-baseline --host-io-steps 0 > $O/cfg2_ow$v.log 2>&1 || { tail -5 $O/cfg2_ow$v.log; exit 1; }
  echo "cfg2 onewave=$v $(grep '^{' $O/cfg2_ow$v.log | tail -1 | grep -o '"ms_per_step": [0-9.]*')"
  PL_RC_ONEWAVE=$v timeout -k 10 200 python bench.py --robot b2 --dynamics whole_body_aba --nodes 40 --batch 256 --steps 20 --warmup 2 --no-cpu-baseline --host-io-steps 0 > $O/cfg3_ow$v.log 2>&1 || { tail -5 $O/cfg3_ow$v.log; exit 1; }
  echo "cfg3 onewave=$v $(grep '^{' $O/cfg3_ow$v.log | tail -1 | grep -o '"ms_per_step": [0-9.]*')"
done
done
# k_ip_refine with the per-node coalesced H_i dx (r04)
timeout -k 10 400 python -u -m pytest tests/test_ip.py -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_ip.log 2>&1 || { tail -30 $O/pytest_ip.log; exit 1; }
tail -2 $O/pytest_ip.log
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_ip" -o run -- python3 bench.py --solver fatrop --steps 2 --warmup 1 --host-io-steps 0 --no-cpu-baseline > $O/prof_ip.log 2>&1 || { tail -20 $O/prof_ip.log; exit 1; }
grep '^{' $O/prof_ip.log | tail -1 | cut -c1-300
head -8 $O/prof_ip/run_kernel_stats.csv | cut -c1-140
# the cheap Jacobian columns written once (default) vs every evaluation (PL_JAC_CHEAP=1)
timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -q --timeout 180 --timeout-method thread -p no:cacheprovider -k "eval_sqp_data or sqp_step or casadi or multi_iteration" > $O/pytest_jac.log 2>&1 || { tail -30 $O/pytest_jac.log; exit 1; }
tail -2 $O/pytest_jac.log
for v in 0 1; do
  PL_JAC_CHEAP=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_cheap$v" -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-io-steps 0 > $O/bench_cheap$v.log 2>&1 || { tail -20 $O/bench_cheap$v.log; exit 1; }
  grep '^{' $O/bench_cheap$v.log | tail -1 | cut -c1-200
  grep -E "k_eval_jac" $O/prof_cheap$v/run_kernel_stats.csv | cut -d, -f1-4
done
