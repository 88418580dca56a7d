#!/bin/bash
# Short headline bench lines for the in-tree build and every library under
# pino-locoman_amd/pinoloco/_ab/ (compiler-option A/B of the same sources).
set -o pipefail
mkdir -p gpurun_out
for k in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/libs_intree_$k.log 2>&1 || exit 1
  for L in pino-locoman_amd/pinoloco/_ab/*.so; do
    n=$(basename $L .so)
    PINOLOCO_LIB=$(realpath $L) timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/libs_${n}_$k.log 2>&1 || exit 1
  done
done
