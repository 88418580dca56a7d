#!/bin/bash
# A/B of the ADMM sweep kernels: parity suite on the default (two waves per problem),
# then bench lines for both kernels.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_w2.log 2>&1 || exit 1
PL_ADMM_WAVES=1 timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/bench_w1.log 2>&1 || exit 1
exit $rc
