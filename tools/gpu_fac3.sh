#!/bin/bash
# factor change: full GPU suite, factor phase timing, bench + kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -2
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit 1;; esac
timeout -k 10 300 python tools/gpu_admm_timing.py 1024 > gpurun_out/timing.log 2>&1 || exit 1
tail -9 gpurun_out/timing.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit 1
grep -E "k_admm<|k_fchain|k_fnode" gpurun_out/prof/run_kernel_stats.csv | cut -d, -f1-4
tail -1 gpurun_out/prof.log | cut -c1-160
