#!/bin/bash
# IP kernels with chunked CSC gathers (k_ip.hip gc_dot): IP parity and the IP line kernel times
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04r}
O=gpurun_out/$T
cd "$R" && mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_ip.py > $O/pytest_ip.log 2>&1 || { tail -30 $O/pytest_ip.log; exit 1; }
tail -2 $O/pytest_ip.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_ip" -o run -- python3 bench.py --solver fatrop --steps 3 --warmup 1 --host-io-steps 0 > $O/prof_ip.log 2>&1 || { tail -20 $O/prof_ip.log; exit 1; }
grep '^{' $O/prof_ip.log | tail -1 | cut -c1-300
grep -E "k_ip_refine|k_ip_kkt|k_ip_step|k_admm_init" $O/prof_ip/run_kernel_stats.csv | cut -d, -f1-4
