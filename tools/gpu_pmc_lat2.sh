#!/bin/bash
# k_admm average latencies (derived counters, one --pmc pass each)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for P in LdsLatency SmemLatency InstrFetchLatency VmemLatency; do
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-include-regex 'k_admm<' --output-format csv -d gpurun_out/lat_$P -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/lat_$P.log 2>&1 || exit 1
done
