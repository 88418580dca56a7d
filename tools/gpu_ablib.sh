#!/bin/bash
# A/B of two builds of the library: parity suite on the in-tree build, then phase timing
# and short bench lines for the in-tree build and $1 (another build, via PINOLOCO_LIB).
# Usage (on the box): bash tools/gpu_ablib.sh pino-locoman_amd/pinoloco/_ab/lib_x.so [tests]
set -o pipefail
mkdir -p gpurun_out
ALT=$(realpath "$1")
TESTS=${2:-tests/test_gpu.py}
timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_ab.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/gpu_admm_timing.py > gpurun_out/timing_new.log 2>&1 || exit 1
PINOLOCO_LIB=$ALT timeout -k 10 300 python tools/gpu_admm_timing.py > gpurun_out/timing_old.log 2>&1 || exit 1
for k in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_new_$k.log 2>&1 || exit 1
  PINOLOCO_LIB=$ALT timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_old_$k.log 2>&1 || exit 1
done
