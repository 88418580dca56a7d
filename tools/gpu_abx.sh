#!/bin/bash
# A/B of library builds without the parity suite: ADMM phase timing and two short bench lines
# each, alternating the in-tree build with every alternative given (PINOLOCO_LIB).
# Usage (on the box): bash tools/gpu_abx.sh alt1.so [alt2.so ...]
set -o pipefail
mkdir -p gpurun_out
libs=("" "$@")
for k in 1 2; do
  for i in "${!libs[@]}"; do
    L=${libs[$i]}
    if [ $k -eq 1 ]; then
      PINOLOCO_LIB=${L:+$(realpath "$L")} timeout -k 10 300 python tools/gpu_admm_timing.py > gpurun_out/timing_$i.log 2>&1 || exit 1
    fi
    PINOLOCO_LIB=${L:+$(realpath "$L")} timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_${i}_$k.log 2>&1 || exit 1
  done
done
for i in "${!libs[@]}"; do
  echo "lib $i ${libs[$i]:-in-tree}: $(grep total gpurun_out/timing_$i.log)"
  for k in 1 2; do tail -1 gpurun_out/bench_${i}_$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('   ', round(d['value']), 'solves/s', round(d['roofline']['avg_launch_ms'], 3), 'ms/launch')"; done
done
