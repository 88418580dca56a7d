#!/bin/bash
# Full GPU test suite + smoke + parity report (development loop)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 300 python tools/parity_report.py > gpurun_out/parity_report.log 2>&1 || exit 1
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3
