#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python tools/gpu_factor_err.py go2_rnea_n20_stand go2 whole_body_rnea 20 > gpurun_out/ferr.log 2>&1 && timeout -k 10 300 python tools/gpu_factor_err.py go2_rnea_n20_walk go2 whole_body_rnea 20 >> gpurun_out/ferr.log 2>&1 && timeout -k 10 300 python tools/gpu_factor_err.py go2_rnea_n20 go2 whole_body_rnea 20 >> gpurun_out/ferr.log 2>&1
