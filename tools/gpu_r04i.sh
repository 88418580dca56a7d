#!/bin/bash
# Interior-point line at the headline config with its CPU baseline, under rocprofv3 (final build)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04i}
O=gpurun_out/$T
cd "$R" && mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_ip" -o run -- python3 bench.py --solver fatrop --steps 3 --warmup 1 --host-io-steps 0 > $O/prof_ip.log 2>&1 || { tail -20 $O/prof_ip.log; exit 1; }
grep '^{' $O/prof_ip.log | tail -1 | cut -c1-1500
head -12 $O/prof_ip/run_kernel_stats.csv | cut -c1-140
