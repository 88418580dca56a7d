set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_ip.py tests/test_r04_paths.py tests/test_dynamics.py -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ipadv.log 2>&1; echo "pytest rc $?" >> gpurun_out/pytest_ipadv.log
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/iptrace" -o run -- python3 bench.py --solver fatrop --steps 1 --warmup 1 --no-cpu-baseline --host-io-steps 0 > gpurun_out/iptrace.log 2>&1 || exit 1
echo done
