#!/bin/bash
# Reduced-chain ADMM kernel: parity tests, then per-config A/B against the sweep kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_admm_kernels.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_rc.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_rc.log
[ $rc -eq 0 ] || exit $rc
: > gpurun_out/rc_ab.jsonl
run() {
  k=$1; shift
  PL_ADMM_KERNEL=$k timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/cfg.log 2>&1 || { tail -20 gpurun_out/cfg.log; exit 1; }
  echo "{\"kernel\": \"$k\", \"args\": \"$*\", \"line\": $(tail -1 gpurun_out/cfg.log)}" >> gpurun_out/rc_ab.jsonl
}
for k in sweep2 chain; do
  run $k --robot b2 --dynamics whole_body_aba --nodes 40 --batch 256 --steps 10 --warmup 2
  run $k --robot go2 --dynamics whole_body_rnea --nodes 20 --batch 1 --steps 20 --warmup 2
done
for k in sweep chain; do
  run $k --steps 5 --warmup 1
done
PL_ADMM_KERNEL=chain timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_rc3" -o run -- python3 bench.py --no-cpu-baseline --robot b2 --dynamics whole_body_aba --nodes 40 --batch 256 --steps 10 --warmup 2 > gpurun_out/prof_rc3.log 2>&1 || exit 1
PL_ADMM_KERNEL=chain timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_rc2" -o run -- python3 bench.py --no-cpu-baseline --robot go2 --dynamics whole_body_rnea --nodes 20 --batch 1 --steps 20 --warmup 2 > gpurun_out/prof_rc2.log 2>&1 || exit 1
python3 -c "
import json
for l in open('gpurun_out/rc_ab.jsonl'):
    d=json.loads(l); x=d['line']; print(d['kernel'], d['args'][:60], round(x['value'],1), round(x['ms_per_step'],2), x.get('roofline',{}).get('avg_launch_ms'))
"
