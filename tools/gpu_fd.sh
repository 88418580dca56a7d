#!/bin/bash
# whole_body_rnea include_acc=False on the GPU (general coupling factor), then the full GPU suite
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -k "fd or include_acc or general_coupling" > gpurun_out/pytest_fd.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_fd.log
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit 1;; esac
grep -E "passed|failed" gpurun_out/pytest_fd.log | tail -2
[ "$rc" = 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2
