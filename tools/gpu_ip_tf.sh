#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
NREF=${3:-2} timeout -k 10 900 python -u tools/gpu_ip_tf.py "$1" "$2" > gpurun_out/ip_tf.log 2>&1
