set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python tools/gpu_sizes.py > gpurun_out/sizes.log 2>&1 && PINOLOCO_LIB=$PWD/pino-locoman_amd/pinoloco/_ab/lib_base.so timeout -k 10 200 python tools/gpu_sizes.py >> gpurun_out/sizes.log 2>&1 && timeout -k 10 300 python tools/gpu_admm_timing.py > gpurun_out/timing_new.log 2>&1 && PINOLOCO_LIB=$PWD/pino-locoman_amd/pinoloco/_ab/lib_base.so timeout -k 10 300 python tools/gpu_admm_timing.py > gpurun_out/timing_old.log 2>&1
