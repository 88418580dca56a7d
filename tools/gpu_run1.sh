#!/bin/bash
# small parity runs under timeouts (go2 N=20, b2g N=50)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/gpu_check.py go2 whole_body_rnea 20 2 > gpurun_out/check_go2.log 2>&1 &&
timeout -k 10 400 python tools/gpu_check.py b2g whole_body_rnea 50 2 > gpurun_out/check_b2g.log 2>&1
