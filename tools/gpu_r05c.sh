# Sweep variants of the block factor (PL_SWEEP_T 0 / 1 / 2): step errors of every SQP fixture
# against the golden KKT oracle (k_admm), and the factor's stage accuracy on the stand problem.
set -o pipefail
mkdir -p gpurun_out
for v in 0 1 2; do
  PINOLOCO_LIB=$PWD/pino-locoman_amd/pinoloco/_ab/lib_sweep$v.so PARITY_KERNELS=sweep PARITY_TAG=sweep$v \
    timeout -k 10 300 python tools/parity_report.py > gpurun_out/parity_sweep$v.log 2>&1 || exit 1
done
echo done
