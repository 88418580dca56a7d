#!/bin/bash
# A/B of library builds on the interior-point line (bench.py --solver fatrop, headline workload):
# the Hessian's per-launch time and solves/s, alternating the in-tree build with each alternative.
# Usage (on the box): bash tools/gpu_abip.sh alt1.so [alt2.so ...]
set -o pipefail
mkdir -p gpurun_out
libs=("" "$@")
for k in 1 2; do
  for i in "${!libs[@]}"; do
    L=${libs[$i]}
    PINOLOCO_LIB=${L:+$(realpath "$L")} timeout -k 10 300 python bench.py --solver fatrop --steps 1 --warmup 1 --no-cpu-baseline --host-io-steps 0 > gpurun_out/benchip_${i}_$k.log 2>&1 || exit 1
  done
done
for i in "${!libs[@]}"; do
  echo "lib $i ${libs[$i]:-in-tree}:"
  for k in 1 2; do tail -1 gpurun_out/benchip_${i}_$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', round(d['value'], 1), 'solves/s, hessian', round(d['roofline']['avg_launch_ms'], 2), 'ms/launch')"; done
done
