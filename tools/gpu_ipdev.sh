#!/bin/bash
# interior-point development loop: the IP GPU tests, then the Fatrop-branch bench line with kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ip.py -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_ip.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_ip.log
grep -E "passed|failed" gpurun_out/pytest_ip.log | tail -2
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit 1;; esac
bash tools/gpu_ipprof.sh
