set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ip.py -v --timeout 300 --timeout-method thread -m gpu -k "matches_oracle and b2g" > gpurun_out/pytest_ipb2g.log 2>&1; echo "pytest rc $?" >> gpurun_out/pytest_ipb2g.log
bash tools/gpu_r05a.sh
