set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/native/mfma_f64_check > gpurun_out/mfma_check.log 2>&1 || { cat gpurun_out/mfma_check.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
timeout -k 10 200 python tools/gpu_admm_timing.py 1024 > gpurun_out/timing.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/prof.log 2>&1 || exit 1
