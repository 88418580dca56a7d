#!/bin/bash
# factor LDS change: GPU tests (no IP) + headline kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread --ignore=tests/test_ip.py > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit 1;; esac
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_fac" -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_fac.log 2>&1 || exit 1
tail -1 gpurun_out/prof_fac.log | cut -c1-200
