#!/bin/bash
# Reduced-chain ADMM kernel: parity tests, phase timing, then per-config A/B against the sweeps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_admm_kernels.py -x -v --timeout 200 --timeout-method thread > gpurun_out/pytest_rc.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_rc.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/gpu_rc_timing.py go2 whole_body_rnea 20 1 > gpurun_out/rc_timing.log 2>&1 || exit 1
timeout -k 10 200 python tools/gpu_rc_timing.py b2 whole_body_aba 40 256 >> gpurun_out/rc_timing.log 2>&1 || exit 1
timeout -k 10 200 python tools/gpu_rc_timing.py b2g whole_body_rnea 50 1024 >> gpurun_out/rc_timing.log 2>&1 || exit 1
: > gpurun_out/rc_ab.jsonl
run() {
  k=$1; shift
  PL_ADMM_KERNEL=$k timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/cfg.log 2>&1 || { tail -20 gpurun_out/cfg.log; exit 1; }
  echo "{\"kernel\": \"$k\", \"args\": \"$*\", \"line\": $(tail -1 gpurun_out/cfg.log)}" >> gpurun_out/rc_ab.jsonl
}
run chain --robot b2 --dynamics whole_body_aba --nodes 40 --batch 256 --steps 10 --warmup 2
run chain --robot go2 --dynamics whole_body_rnea --nodes 20 --batch 1 --steps 20 --warmup 2
run chain --robot go2 --dynamics centroidal_vel --nodes 20 --batch 1024 --steps 10 --warmup 2
run sweep --robot go2 --dynamics centroidal_vel --nodes 20 --batch 1024 --steps 10 --warmup 2
run chain --steps 5 --warmup 1
run chain --batch 512 --steps 5 --warmup 1
run sweep2 --batch 512 --steps 5 --warmup 1
python3 -c "
import json
for l in open('gpurun_out/rc_ab.jsonl'):
    d=json.loads(l); x=d['line']; print(d['kernel'], d['args'][:60], round(x['value'],1), round(x['ms_per_step'],2), x.get('roofline',{}).get('avg_launch_ms'))
"
