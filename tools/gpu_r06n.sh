#!/bin/bash
# r06: the factor chain's panel sweep -- parity (goldens, loops, IP, kernels), then rocprofv3 of the
# headline bench with the panel sweep and with the r05 4-pivot sweep (PL_PATH_FCHAIN_SWEEP4).
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py tests/test_admm_kernels.py tests/test_ip.py tests/test_r04_paths.py -m gpu > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log
[ "$rc" = 0 ] || exit 1
for v in panel sweep4; do
  P=""; [ $v = sweep4 ] && P="--debug-paths fchain_sweep4"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/$v" -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --host-io-steps 0 $P > $O/$v.log 2>&1 || exit 1
done
timeout -k 10 120 python tools/gpu_fchain_timing.py b2g whole_body_rnea 50 1024 > $O/fct.txt 2>&1 || exit 1
echo done
