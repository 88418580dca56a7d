#!/bin/bash
# kernel stats of the interior-point (Fatrop branch) bench line at the headline config
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/ipprof" -o run -- python3 bench.py --solver fatrop --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/ipprof.log 2>&1 || exit 1
head -12 gpurun_out/ipprof/run_kernel_stats.csv | cut -d, -f1-4
