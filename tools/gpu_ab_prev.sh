#!/bin/bash
# Same-box A/B: ab/libpinoloco_prev.so (previous commit) against the in-tree library,
# headline bench, alternating, k_admm avg launch from the line's roofline
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
: > gpurun_out/ab_prev.txt
for v in prev cur prev cur; do
  if [ $v = prev ]; then export PINOLOCO_LIB=$R/ab/libpinoloco_prev.so; else unset PINOLOCO_LIB; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab.log 2>&1 || { tail -5 gpurun_out/ab.log; exit 1; }
  python -c "
import json,sys
d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$v', round(d['value'],1), round(d['ms_per_step'],2), 'k_admm %.3f ms' % r['avg_launch_ms'], 'iters/launch', r['problem_iters_per_launch'])
" | tee -a gpurun_out/ab_prev.txt
done
