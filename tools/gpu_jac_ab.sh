#!/bin/bash
# A/B of k_eval_jac build variants: rebuild in the box's copy with PL_HIPCC_DEFS, then
# rocprofv3 kernel stats of a 2-step bench.  Usage: bash tools/gpu_jac_ab.sh "-DA=1" "-DA=2" ...
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for defs in "$@"; do
  i=$((i+1))
  PL_HIPCC_DEFS="$defs" timeout -k 10 300 python -c "import sys; sys.path.insert(0,'pino-locoman_amd'); from pinoloco import build; build.build(force=True)" > gpurun_out/jab_build$i.log 2>&1 || exit 1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/jab$i" -o run -- python3 bench.py --steps 2 --warmup 0 --no-cpu-baseline > gpurun_out/jab$i.log 2>&1 || exit 1
  echo "== $defs"; grep -E "k_eval_jac|k_admm<|k_fchain" gpurun_out/jab$i/run_kernel_stats.csv | cut -d, -f1-5
done
