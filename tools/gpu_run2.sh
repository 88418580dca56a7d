#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --batch 256 --no-cpu-baseline > gpurun_out/bench_b256.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 5 --warmup 1 --batch 1024 --no-cpu-baseline > gpurun_out/bench_b1024.log 2>&1
echo "exit=$?" >> gpurun_out/bench_b1024.log
