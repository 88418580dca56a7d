#!/bin/bash
# r06: the forward-over-reverse Hessian columns -- parity (against the r05 pair kernel and the r04
# hyper-dual node rows), the IP test file, the IP line and its kernel stats.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_r04_paths.py tests/test_ip.py -m gpu > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log
case "$rc" in 0|1) ;; *) exit 1;; esac
timeout -k 10 400 python bench.py --solver fatrop --steps 10 --warmup 1 > $O/bench_ip.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof" -o run -- python3 bench.py --solver fatrop --steps 1 --warmup 1 --no-cpu-baseline --host-io-steps 0 > $O/prof.log 2>&1 || exit 1
echo done
