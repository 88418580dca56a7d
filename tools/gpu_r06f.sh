#!/bin/bash
# r06: the split column kernels (no spills) -- Hessian parity, IP tests, the IP line, and the F64
# instruction counts of the Hessian kernels for the IP roofline.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_r04_paths.py tests/test_ip.py -m gpu > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log
case "$rc" in 0|1) ;; *) exit 1;; esac
P3="SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INST_CYCLES_VMEM SQ_WAVES SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_INSTS_SMEM"
timeout -s KILL 300 rocprofv3 --pmc $P3 --kernel-include-regex k_lag_hess --output-format csv -d "$PWD/$O/q3" -o run -- python3 bench.py --solver fatrop --steps 1 --warmup 0 --no-cpu-baseline --batch 1024 --host-io-steps 0 > $O/q3.log 2>&1 || exit 1
python tools/hess_flops.py $O/q3 $O/hess_flops.json 1024 50 sweep > $O/hess_flops.log 2>&1
cp $O/hess_flops.json profiles/traffic/hess_flops.json
timeout -k 10 400 python bench.py --solver fatrop --steps 10 --warmup 1 > $O/bench_ip.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof" -o run -- python3 bench.py --solver fatrop --steps 1 --warmup 1 --no-cpu-baseline --host-io-steps 0 > $O/prof.log 2>&1 || exit 1
echo done
