#!/bin/bash
# k_fchain's E_{i+1}: staged short lists (rnea / acc) and the MFMA Wc S Wc^T (aba / centroidal):
# the GPU parity suite, the chain phase timing, configs 1 / 3 / headline with PL_FCHAIN_MF=1 and 0.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04e}
O=gpurun_out/$T
cd "$R" && mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu.py tests/test_admm_kernels.py tests/test_qp_kernels.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for a in "go2 centroidal_vel 20 1024" "b2 whole_body_aba 40 256" "b2g whole_body_rnea 50 1024"; do
  n=$(echo $a | tr ' ' '_')
  timeout -k 10 200 python tools/gpu_fchain_timing.py $a > $O/fchain_$n.txt 2>&1 || { tail -5 $O/fchain_$n.txt; exit 1; }
  cat $O/fchain_$n.txt
done
for v in 1 0; do
  PL_FCHAIN_MF=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/cfg1_mf$v" -o run -- python3 bench.py --robot go2 --dynamics centroidal_vel --nodes 20 --batch 1024 --steps 20 --warmup 2 --no-cpu-baseline --host-io-steps 0 > $O/cfg1_mf$v.log 2>&1 || { tail -5 $O/cfg1_mf$v.log; exit 1; }
  echo "cfg1 mf=$v $(grep '^{' $O/cfg1_mf$v.log | tail -1 | grep -o '"ms_per_step": [0-9.]*')"; grep fchain $O/cfg1_mf$v/run_kernel_stats.csv | cut -d, -f1-4
  PL_FCHAIN_MF=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/cfg3_mf$v" -o run -- python3 bench.py --robot b2 --dynamics whole_body_aba --nodes 40 --batch 256 --steps 20 --warmup 2 --no-cpu-baseline --host-io-steps 0 > $O/cfg3_mf$v.log 2>&1 || { tail -5 $O/cfg3_mf$v.log; exit 1; }
  echo "cfg3 mf=$v $(grep '^{' $O/cfg3_mf$v.log | tail -1 | grep -o '"ms_per_step": [0-9.]*')"; grep fchain $O/cfg3_mf$v/run_kernel_stats.csv | cut -d, -f1-4
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/head" -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline --host-io-steps 0 > $O/head.log 2>&1 || { tail -5 $O/head.log; exit 1; }
grep '^{' $O/head.log | tail -1 | cut -c1-200; grep -E "fchain|eval_jac" $O/head/run_kernel_stats.csv | cut -d, -f1-4
