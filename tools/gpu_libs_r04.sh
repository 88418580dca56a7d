#!/bin/bash
# Scheduler A/B of k_admm.hip (libraries under pino-locoman_amd/pinoloco/_ab/, same sources,
# other -mllvm --amdgpu-sched-strategy) against the in-tree build, twice each; phase timing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04l}
O=gpurun_out/$T
cd "$R" && mkdir -p "$O"
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "solves/s %.1f" % d["value"], "ms/step %.2f" % d["ms_per_step"], r["kernel"], "avg ms %.3f" % r["avg_launch_ms"])
PY
}
for k in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --host-io-steps 0 > $O/intree_$k.log 2>&1 || exit 1
  summ $O/intree_$k.log "intree(iterative-ilp)"
  for L in pino-locoman_amd/pinoloco/_ab/*.so; do
    n=$(basename $L .so)
    PINOLOCO_LIB=$(realpath $L) timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --host-io-steps 0 > $O/${n}_$k.log 2>&1 || exit 1
    summ $O/${n}_$k.log "$n"
  done
done
timeout -k 10 200 python tools/gpu_admm_timing.py 1024 > $O/phase_timing.txt 2>&1 || exit 1
head -13 $O/phase_timing.txt
