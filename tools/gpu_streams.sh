#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gpu_streams.py 1 2 4 > gpurun_out/streams.log 2>&1 || exit 1
PL_ADMM_KERNEL=sweep timeout -k 10 300 python -u tools/gpu_streams.py 2 4 >> gpurun_out/streams.log 2>&1
