#!/bin/bash
# r06: the new parity tests (25-step loops, the IP default-driver loops, refinement counts,
# compiled_solver through the CasADi ABI), the whole GPU suite, smoke, the driver's bench
# command and the interior-point line.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -s \
  tests/test_gpu.py::test_device_mpc_loop_over_bench_steps_inside_batch \
  tests/test_ip.py::test_ip_gpu_default_driver_loop_inside_batch \
  tests/test_ip.py::test_ip_gpu_refinement_counts_and_gather_path \
  tests/test_ip.py::test_run_mpc_load_compiled_solver_external \
  tests/test_ip.py::test_ip_gpu_gauss_newton_option > gpurun_out/pytest_new.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_new.log
case "$rc" in 0|1) ;; *) exit 1;; esac
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log
case "$rc" in 0|1) ;; *) exit 1;; esac
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --solver fatrop --steps 10 --warmup 1 > gpurun_out/bench_ip.log 2>&1 || exit 1
echo done
