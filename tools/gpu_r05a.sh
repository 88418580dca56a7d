set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/gpu_factor_stages.py go2_rnea_n20_stand go2 whole_body_rnea 20 2 > gpurun_out/fstages2.log 2>&1 || exit 1
for f in go2_rnea_n20_stand go2_rnea_n20_walk go2_rnea_fd_n20; do timeout -k 10 200 python tools/gpu_reduced_diag.py $f go2 whole_body_rnea 20 sweep > gpurun_out/rdiag2_$f.log 2>&1 || exit 1; done
timeout -k 10 600 python -u -m pytest tests/test_gpu.py -x -q --timeout 300 --timeout-method thread -k "sqp_step or loop" > gpurun_out/pytest_step.log 2>&1; echo "pytest rc $?" >> gpurun_out/pytest_step.log
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_ldl.log 2>&1 || exit 1
echo done
