#!/bin/bash
# Round-4 evidence loop: GPU tests + smoke + bench + rocprof stats (+ optional PMC traffic).
# Usage (on the box): bash tools/gpu_r04.sh <tag> [traffic]
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04}
O=gpurun_out/$T
cd "$R" && mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_gpu.log
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit 1;; esac
grep -E "passed|failed" $O/pytest_gpu.log | tail -3
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
if [ "$2" = "traffic" ]; then
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_admm<' --output-format csv -d "$R/$O/pmc_fetch" -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --host-io-steps 0 > $O/pmc_fetch.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_admm<' --output-format csv -d "$R/$O/pmc_write" -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --host-io-steps 0 > $O/pmc_write.log 2>&1 || exit 1
  python tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/pmc_fetch.log $O/admm_traffic.json
fi
tail -1 $O/bench.log | cut -c1-400
