#!/bin/bash
# r06: k_admm_rc over several workgroups per problem -- chain parity (bit-identical to the one-
# workgroup kernel), the chain loops, phase timing, and config 2 / config 3 bench lines (new and
# PL_PATH_RC_ONE_GROUP side by side).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_admm_kernels.py -m gpu > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log
[ "$rc" = 0 ] || exit 1
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu.py -m gpu -k "chain" > $O/pytest_chain.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_chain.log
case "$rc" in 0|1|5) ;; *) exit 1;; esac
timeout -k 10 120 python tools/gpu_rc_timing.py go2 whole_body_rnea 20 1 > $O/rc_timing_go2.txt 2>&1 || exit 1
timeout -k 10 120 python tools/gpu_rc_timing.py go2 whole_body_rnea 20 1 rc_one_group > $O/rc_timing_go2_one.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --robot go2 --dynamics whole_body_rnea --nodes 20 --batch 1 --steps 40 --warmup 2 > $O/cfg2.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --robot go2 --dynamics whole_body_rnea --nodes 20 --batch 1 --steps 40 --warmup 2 --debug-paths rc_one_group > $O/cfg2_one.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --robot b2 --dynamics whole_body_aba --nodes 40 --batch 256 --steps 40 --warmup 2 > $O/cfg3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof2" -o run -- python3 bench.py --robot go2 --dynamics whole_body_rnea --nodes 20 --batch 1 --steps 10 --warmup 2 --no-cpu-baseline --host-io-steps 0 > $O/prof2.log 2>&1 || exit 1
echo done
