#!/bin/bash
# A/B of the two-wave ADMM kernel (k_admm2, B < 512): GPU parity suite on the in-tree
# build, then config 3 (B2 aba N=40, B=256) bench lines for the in-tree build and $1.
set -o pipefail
mkdir -p gpurun_out
ALT=$(realpath "$1")
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_ab.log
[ $rc -eq 0 ] || exit $rc
C3="--robot b2 --dynamics whole_body_aba --nodes 40 --batch 256 --steps 20 --warmup 2 --no-cpu-baseline"
for k in 1 2; do
  timeout -k 10 300 python bench.py $C3 > gpurun_out/c3_new_$k.log 2>&1 || exit 1
  PINOLOCO_LIB=$ALT timeout -k 10 300 python bench.py $C3 > gpurun_out/c3_old_$k.log 2>&1 || exit 1
done
