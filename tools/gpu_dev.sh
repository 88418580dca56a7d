#!/bin/bash
# development loop: GPU tests, then bench + rocprofv3 kernel stats of the headline config
# (and, with AB=1, the legacy Schur chain in the same call for an A/B)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit 1;; esac
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit 1
tail -1 gpurun_out/bench.log | cut -c1-200
if [ "${AB:-0}" = 1 ]; then
  PL_FCHAIN_LEGACY=1 timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_legacy.log 2>&1 || exit 1
  tail -1 gpurun_out/bench_legacy.log | cut -c1-200
fi
