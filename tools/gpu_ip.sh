#!/bin/bash
# Interior-point parity tests on the GPU (tests/test_ip.py -m gpu).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ip.py -m gpu -v --timeout 300 --timeout-method thread ${IP_K:+-k "$IP_K"} > gpurun_out/pytest_ip.log 2>&1
rc=$?
echo "pytest exit $rc" >> gpurun_out/pytest_ip.log
tail -30 gpurun_out/pytest_ip.log
exit $rc
