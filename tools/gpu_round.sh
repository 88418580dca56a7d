#!/bin/bash
# GPU round check: parity tests, smoke, bench line, rocprofv3 kernel stats and the
# two PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs) for k_admm traffic.
# Usage (on the box): bash tools/gpu_round.sh [tag]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-run}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log
  case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit 1;; esac
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
  timeout -k 10 300 python tools/parity_report.py > gpurun_out/parity_report.log 2>&1 || exit 1
fi
timeout -k 10 600 python bench.py > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_admm<' --output-format csv -d "$R/gpurun_out/pmc_fetch" -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --host-io-steps 0 > gpurun_out/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_admm<' --output-format csv -d "$R/gpurun_out/pmc_write" -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --host-io-steps 0 > gpurun_out/pmc_write.log 2>&1 || exit 1
python tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/pmc_fetch.log gpurun_out/admm_traffic.json
