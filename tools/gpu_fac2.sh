#!/bin/bash
# factor kernels: parity subset + headline kernel stats
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_admm_kernels.py -m gpu -x -q --timeout 300 --timeout-method thread -k "sqp_step or loop or kernels_agree or bit_identical" > gpurun_out/pytest_fac.log 2>&1 || exit 1
tail -1 gpurun_out/pytest_fac.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_fac" -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_fac.log 2>&1 || exit 1
tail -1 gpurun_out/prof_fac.log | cut -c1-200
