#!/bin/bash
# k_fnode's assembly stream prefetched (r04): parity (the factor feeds every path), factor phase
# timing, the headline and configs 1 / 3 under rocprofv3.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04a}
O=gpurun_out/$T
cd "$R" && mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu.py tests/test_qp_kernels.py tests/test_ip.py -k "sqp_step or qp or loop or ip" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for a in "b2g whole_body_rnea 50 1024" "b2 whole_body_aba 40 256"; do
  n=$(echo $a | tr ' ' '_')
  timeout -k 10 200 python tools/gpu_fchain_timing.py $a > $O/fac_$n.txt 2>&1 || { tail -5 $O/fac_$n.txt; exit 1; }
  tail -8 $O/fac_$n.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/head" -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-io-steps 0 > $O/head.log 2>&1 || { tail -5 $O/head.log; exit 1; }
grep '^{' $O/head.log | tail -1 | cut -c1-200; grep -E "fnode|fchain|k_admm<" $O/head/run_kernel_stats.csv | cut -d, -f1-4
