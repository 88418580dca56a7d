set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/gpu_rc_timing.py go2 whole_body_rnea 20 1 > gpurun_out/rc_timing.log 2>&1 && timeout -k 10 200 python tools/gpu_rc_timing.py b2 whole_body_aba 40 256 >> gpurun_out/rc_timing.log 2>&1 && timeout -k 10 200 python tools/gpu_rc_timing.py b2g whole_body_rnea 50 1024 >> gpurun_out/rc_timing.log 2>&1
