#!/bin/bash
# k_admm (one wave per problem) vs k_admm2 (two waves) at the headline config, B = 1024
# and B = 512: short bench lines (PL_ADMM_WAVES overrides the default choice).
set -o pipefail
mkdir -p gpurun_out
for B in 1024 512; do
  for W in 1 2; do
    PL_ADMM_WAVES=$W timeout -k 10 300 python bench.py --batch $B --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/waves_${B}_${W}.log 2>&1 || exit 1
  done
done
