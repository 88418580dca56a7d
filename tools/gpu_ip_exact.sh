#!/bin/bash
# exact-Hessian interior point: the IP GPU tests on the given -k expression
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_ip.py -m gpu -v --timeout 300 --timeout-method thread -k "$1" > gpurun_out/ip_exact.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/ip_exact.log
grep -E "passed|failed" gpurun_out/ip_exact.log | tail -1
