#!/bin/bash
# fused equilibration: parity vs the per-pass kernels, per-fixture step errors, headline kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_qp_kernels.py -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/qp_tests.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/qp_tests.log
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit 1;; esac
grep -E "passed|failed" gpurun_out/qp_tests.log | tail -1
timeout -k 10 500 python -u tools/parity_report.py > gpurun_out/parity_report.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_qp" -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_qp.log 2>&1 || exit 1
tail -1 gpurun_out/prof_qp.log | cut -c1-300
