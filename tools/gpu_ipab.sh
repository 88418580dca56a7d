set -o pipefail
mkdir -p gpurun_out
T="tests/test_ip.py::test_ip_gpu_matches_oracle"
timeout -k 10 200 python -m pytest "$T" -x -q --timeout 120 > gpurun_out/ip_new1.log 2>&1; echo "new1 $?" >> gpurun_out/ip_ab.txt
timeout -k 10 200 python -m pytest "$T" -x -q --timeout 120 > gpurun_out/ip_new2.log 2>&1; echo "new2 $?" >> gpurun_out/ip_ab.txt
PINOLOCO_LIB=$PWD/pino-locoman_amd/pinoloco/_ab/lib_head.so timeout -k 10 200 python -m pytest "$T" -x -q --timeout 120 > gpurun_out/ip_head.log 2>&1; echo "head $?" >> gpurun_out/ip_ab.txt
PINOLOCO_LIB=$PWD/pino-locoman_amd/pinoloco/_ab/lib_seg.so timeout -k 10 200 python -m pytest "$T" -x -q --timeout 120 > gpurun_out/ip_seg.log 2>&1; echo "seg $?" >> gpurun_out/ip_ab.txt
true
