# Full GPU parity suite, smoke, bench + rocprofv3 kernel stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log
case "$rc" in 0|1) ;; *) exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" -o run -- python3 bench.py --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit 1
echo done
