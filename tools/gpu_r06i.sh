#!/bin/bash
# r06: k_admm without the forward steps' one-line HBM reads -- sweep parity, headline bench,
# k_admm PMC traffic passes.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu.py tests/test_admm_kernels.py -m gpu -k "sweep or kernels_agree or bit_identical" > $O/pytest.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest.log
[ "$rc" = 0 ] || exit 1
timeout -k 10 400 python bench.py --steps 10 --warmup 2 --host-io-steps 0 --no-cpu-baseline > $O/bench.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex 'k_admm<' --output-format csv -d "$PWD/$O/pmc_fetch" -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --host-io-steps 0 > $O/pmc_fetch.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex 'k_admm<' --output-format csv -d "$PWD/$O/pmc_write" -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline --host-io-steps 0 > $O/pmc_write.log 2>&1 || exit 1
python tools/pmc_traffic.py $O/pmc_fetch $O/pmc_write $O/pmc_fetch.log $O/admm_traffic.json > $O/pmc_traffic.log 2>&1
echo done
