#!/bin/bash
# One bench line per BASELINE config and the interior-point
# line at the headline config; JSON lines into gpurun_out/configs.jsonl.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
: > gpurun_out/configs.jsonl
run() {
  timeout -k 10 400 python bench.py "$@" > gpurun_out/cfg.log 2>&1 || { tail -20 gpurun_out/cfg.log; exit 1; }
  tail -1 gpurun_out/cfg.log >> gpurun_out/configs.jsonl
}
run --robot go2 --dynamics centroidal_vel --nodes 20 --batch 1024 --steps 40 --warmup 2          # config 1
run --robot go2 --dynamics whole_body_rnea --nodes 20 --batch 1 --steps 40 --warmup 2            # config 2 (one problem)
run --robot b2 --dynamics whole_body_aba --nodes 40 --batch 256 --steps 40 --warmup 2            # config 3
run --robot b2g --dynamics whole_body_acc --nodes 50 --batch 1024 --steps 40 --warmup 2          # config 4
run --solver fatrop --steps 10 --warmup 1 --host-io-steps 0                                     # headline, Fatrop branch (ip_stats: the 11th MPC step)
cat gpurun_out/configs.jsonl | cut -c1-200
