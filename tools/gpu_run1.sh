#!/bin/bash
# first GPU bring-up: small parity run under a timeout
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/gpu_check.py go2 whole_body_rnea 20 2 > gpurun_out/check_go2.log 2>&1
echo "exit=$?" >> gpurun_out/check_go2.log
