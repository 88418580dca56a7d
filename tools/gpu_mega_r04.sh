#!/bin/bash
# One box, several answers (the pool is congested): GPU tests, k_admm scatter vs chunked A/B,
# interior-point Hessian mapping A/B, rocprof stats of the headline bench.
# Usage (on the box): bash tools/gpu_mega_r04.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04m}
O=gpurun_out/$T
cd "$R" && mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 660 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_gpu.log
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; tail -5 $O/pytest_gpu.log; exit 1;; esac
grep -E "passed|failed" $O/pytest_gpu.log | tail -3
grep -E "FAILED" $O/pytest_gpu.log | head -20
summ() {
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(sys.argv[2], "solves/s %.1f" % d["value"], "ms/step %.2f" % d["ms_per_step"], r["kernel"], "avg ms %.3f" % r["avg_launch_ms"],
      "frac", r["frac"] if r["frac"] is None else "%.4f" % r["frac"])
PY
}
for v in 0 1; do
  PL_ADMM_CHUNKED=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --host-io-steps 0 > $O/bench_chunked$v.log 2>&1 || exit 1
  summ $O/bench_chunked$v.log "chunked=$v"
done
for v in 0 1; do
  PL_HESS_PB=$v timeout -k 10 200 python bench.py --solver fatrop --steps 1 --warmup 1 --no-cpu-baseline --batch 256 --host-io-steps 0 > $O/ip_pb$v.log 2>&1 || exit 1
  summ $O/ip_pb$v.log "hess_pb=$v"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || exit 1
summ $O/prof.log "under-rocprof"
head -6 $O/prof/run_kernel_stats.csv | cut -c1-160
