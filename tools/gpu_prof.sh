#!/bin/bash
# rocprofv3 kernel-trace summary of a short bench run
set -o pipefail
mkdir -p gpurun_out/prof
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --batch ${PL_BATCH:-1024} --no-cpu-baseline > gpurun_out/prof/bench.log 2>&1
echo "exit=$?" >> gpurun_out/prof/bench.log
find gpurun_out/prof -name "*stats*" | head
