#!/bin/bash
# GPU round check: parity tests, smoke, bench line, rocprofv3 kernel stats.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests -m gpu -q --timeout 400 > gpurun_out/pytest_gpu.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_gpu.log
rc=$(tail -1 gpurun_out/pytest_gpu.log | awk '{print $3}')
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 &&
export TMPDIR=/tmp &&
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/prof.log 2>&1
