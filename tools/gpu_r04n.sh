#!/bin/bash
# Interior-point parity under the one-problem-per-lane Hessian, k_admm rows-scatter A/B, the IP
# step's kernel breakdown at B = 1024 and the Hessian's F64 flop count.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04n}
O=gpurun_out/$T
cd "$R" && mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_ip.py tests/test_gpu.py -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider -k "test_ip or eps5" > $O/pytest_ip.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_ip.log
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; tail -5 $O/pytest_ip.log; exit 1;; esac
grep -E "passed|failed" $O/pytest_ip.log | tail -2; grep FAILED $O/pytest_ip.log | head
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "solves/s %.1f" % d["value"], "ms/step %.2f" % d["ms_per_step"], r["kernel"], "avg ms %.3f" % r["avg_launch_ms"],
      "frac", r["frac"] if r["frac"] is None else "%.4f" % r["frac"])
PY
}
for v in 1 0 1 0; do
  PL_ADMM_SCATTER=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --host-io-steps 0 > $O/bench_sc$v.log 2>&1 || exit 1
  summ $O/bench_sc$v.log "scatter=$v"
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_ip" -o run -- python3 bench.py --solver fatrop --steps 1 --warmup 1 --no-cpu-baseline --host-io-steps 0 > $O/prof_ip.log 2>&1 || exit 1
summ $O/prof_ip.log "ip-b1024-under-rocprof"
head -8 $O/prof_ip/run_kernel_stats.csv | cut -c1-140
bash tools/gpu_hess_pmc.sh $T/hess > $O/hess_pmc.log 2>&1; tail -4 $O/hess_pmc.log
