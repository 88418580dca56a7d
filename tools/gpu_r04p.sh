#!/bin/bash
# Full evidence at the current defaults (tests, smoke, bench, rocprof, PMC traffic), then the
# rows-scatter A/B on top of the deferred stores.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04p}
O=gpurun_out/$T
cd "$R" && mkdir -p "$O"
bash tools/gpu_r04.sh $T traffic || exit 1
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "solves/s %.1f" % d["value"], "ms/step %.2f" % d["ms_per_step"], r["kernel"], "avg ms %.3f" % r["avg_launch_ms"],
      "frac", r["frac"] if r["frac"] is None else "%.4f" % r["frac"])
PY
}
for rep in 1 2; do
  for v in 0 1; do
    PL_ADMM_SCATTER=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --host-io-steps 0 > $O/bench_sc${v}_$rep.log 2>&1 || exit 1
    summ $O/bench_sc${v}_$rep.log "defer+scatter=$v"
  done
done
