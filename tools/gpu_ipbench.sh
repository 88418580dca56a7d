#!/bin/bash
# Interior-point bench line + kernel stats (headline config, solver=fatrop)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --solver fatrop --steps 5 --warmup 1 > gpurun_out/bench_ip.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_ip" -o run -- python3 bench.py --solver fatrop --steps 3 --warmup 1 > gpurun_out/prof_ip.log 2>&1 || exit 1
tail -2 gpurun_out/bench_ip.log
