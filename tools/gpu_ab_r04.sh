#!/bin/bash
# Round-4 A/B: k_admm entry-order scatters vs chunked gathers (PL_ADMM_CHUNKED=1) at the
# headline config, and the interior-point Hessian mappings (PL_HESS_PB=1) at B = 256;
# parity subset of the GPU tests first.  Usage (on the box): bash tools/gpu_ab_r04.sh <tag>
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04ab}
O=gpurun_out/$T
cd "$R" && mkdir -p "$O"
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu.py tests/test_admm_kernels.py -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider -k "sweep or kernels_agree or bit_identical or batch_invariance" > $O/pytest_sweep.log 2>&1
rc=$?; echo "pytest exit $rc" >> $O/pytest_sweep.log; tail -3 $O/pytest_sweep.log
case "$rc" in 0|1) ;; *) echo "stopping after pytest rc=$rc"; exit 1;; esac
for v in 0 1 0 1; do
  PL_ADMM_CHUNKED=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --host-io-steps 0 > $O/bench_chunked$v.log 2>&1 || exit 1
  python - $O/bench_chunked$v.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("chunked", sys.argv[2], "solves/s %.1f" % d["value"], "ms/step %.2f" % d["ms_per_step"], "k_admm ms %.3f" % d["roofline"]["avg_launch_ms"], "frac %.4f" % d["roofline"]["frac"])
PY
done
for v in 0 1; do
  PL_HESS_PB=$v timeout -k 10 300 python bench.py --solver fatrop --steps 1 --warmup 1 --no-cpu-baseline --batch 256 --host-io-steps 0 > $O/ip_pb$v.log 2>&1 || exit 1
  python - $O/ip_pb$v.log $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("hess_pb", sys.argv[2], "IP solves/s %.1f" % d["value"], "ms/step %.1f" % d["ms_per_step"], d.get("ip_stats"))
PY
done
PL_HESS_PB=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/prof_ip_pb1" -o run -- python3 bench.py --solver fatrop --steps 1 --warmup 0 --no-cpu-baseline --batch 256 --host-io-steps 0 > $O/prof_ip_pb1.log 2>&1 || exit 1
head -4 $O/prof_ip_pb1/run_kernel_stats.csv
