#!/bin/bash
# MPC-step graph replay: GPU closed-loop tests, then config 2 (one Go2 problem) with and
# without the graph, and config 3 (B2 aba N=40, B=256)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_admm_kernels.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_graph.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_graph.log; tail -2 gpurun_out/pytest_graph.log
[ "$rc" = 0 ] || exit 1
: > gpurun_out/graph_ab.jsonl
for g in 0 1 0 1; do
  PL_MPC_GRAPH=$g timeout -k 10 300 python bench.py --robot go2 --dynamics whole_body_rnea --nodes 20 --batch 1 --steps 60 --warmup 3 --no-cpu-baseline > gpurun_out/cfg.log 2>&1 || { tail -20 gpurun_out/cfg.log; exit 1; }
  echo "{\"graph\": $g, \"line\": $(tail -1 gpurun_out/cfg.log)}" >> gpurun_out/graph_ab.jsonl
done
python -c "
import json
for l in open('gpurun_out/graph_ab.jsonl'):
    d=json.loads(l); print('graph', d['graph'], 'ms/step %.3f' % d['line']['ms_per_step'], 'admm avg %.3f ms' % d['line']['roofline']['avg_launch_ms'])
"
