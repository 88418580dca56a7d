#!/bin/bash
# GPU tests + one profiled headline bench (driver's command: --steps 20 --warmup 5)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_SEL:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest exit $rc" >> gpurun_out/pytest_gpu.log
tail -3 gpurun_out/pytest_gpu.log
case "$rc" in 0) ;; *) echo "stopping after pytest rc=$rc"; exit 1;; esac
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/prof.log 2>&1 || exit 1
grep '^{' gpurun_out/prof.log | tail -1 | cut -c1-250
python - <<'PY'
import csv, glob
f = sorted(glob.glob("gpurun_out/prof/**/*kernel_stats.csv", recursive=True))[-1]
for r in list(csv.DictReader(open(f)))[:12]:
    print(f"{r['Name'][:44]:44s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:10.1f} us  {float(r['TotalDurationNs'])/25e6:8.3f} ms/step")
PY
