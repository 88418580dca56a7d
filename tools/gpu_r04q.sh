#!/bin/bash
# Interior point with the linear-column Hessian blocks: IP parity tests, the IP bench line at
# the headline config (with its CPU baseline) under rocprofv3, the Hessian's F64 flops, and the
# k_admm PMC traffic of the current sources.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04q}
O=gpurun_out/$T
cd "$R" && mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_ip.py tests/test_admm_kernels.py -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_ip.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_ip.log
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; tail -5 $O/pytest_ip.log; exit 1;; esac
grep -E "passed|failed" $O/pytest_ip.log | tail -2; grep FAILED $O/pytest_ip.log | head
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_ip" -o run -- python3 bench.py --solver fatrop --steps 2 --warmup 1 --host-io-steps 0 > $O/prof_ip.log 2>&1 || exit 1
grep '^{' $O/prof_ip.log | tail -1 | cut -c1-600
head -6 $O/prof_ip/run_kernel_stats.csv | cut -c1-140
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_admm<' --output-format csv -d "$R/$O/pmc_fetch" -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --host-io-steps 0 > $O/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_admm<' --output-format csv -d "$R/$O/pmc_write" -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --host-io-steps 0 > $O/pmc_write.log 2>&1 || exit 1
python tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/pmc_fetch.log $O/admm_traffic.json
bash tools/gpu_hess_pmc.sh $T/hess pb 1024 > $O/hess_pmc.log 2>&1; tail -2 $O/hess_pmc.log
