#!/bin/bash
# k_admm A/B at the headline config on one box: default, deferred stores (PL_ADMM_DEFER=1),
# rows scatter (PL_ADMM_SCATTER=1); a parity subset on the deferred variant; phase timing.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04o}
O=gpurun_out/$T
cd "$R" && mkdir -p "$O"
export TMPDIR=/tmp
PL_ADMM_DEFER=1 timeout -k 10 400 python -u -m pytest tests/test_gpu.py -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider -k "sweep and (b2g or eps2 or infeas)" > $O/pytest_defer.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_defer.log; tail -2 $O/pytest_defer.log
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit 1;; esac
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
  for cfg in "base" "PL_ADMM_DEFER=1" "PL_ADMM_SCATTER=1"; do
    env $([ "$cfg" = base ] || echo "$cfg") timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --host-io-steps 0 > $O/bench_${cfg//=/_}_$rep.log 2>&1 || exit 1
    summ $O/bench_${cfg//=/_}_$rep.log "$cfg"
  done
done
timeout -k 10 200 python tools/gpu_admm_timing.py 1024 > $O/phase_timing.txt 2>&1 || exit 1
head -14 $O/phase_timing.txt
