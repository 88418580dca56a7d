#!/bin/bash
# r06: new parity tests first (25-step loops in the benchmark batch, refinement counts and the
# gather path), then the whole GPU suite, smoke and the driver's bench command.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s \
  tests/test_gpu.py::test_device_mpc_loop_over_bench_steps_inside_batch \
  tests/test_ip.py::test_ip_gpu_refinement_counts_and_gather_path > gpurun_out/pytest_new.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_new.log
case "$rc" in 0|1) ;; *) exit 1;; esac
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log
case "$rc" in 0|1) ;; *) exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit 1
echo done
