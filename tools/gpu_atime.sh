#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/gpu_admm_timing.py 1024 > gpurun_out/admm_timing.log 2>&1
