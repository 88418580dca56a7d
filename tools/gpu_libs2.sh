#!/bin/bash
# Per-kernel timing A/B of the in-tree build against every library under
# pino-locoman_amd/pinoloco/_ab/: rocprofv3 kernel stats of a short headline run and of
# config 3 (B2 aba N=40, B=256) for each build.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
run() {  # name, lib
  local n=$1 L=$2
  PINOLOCO_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/pl_$n" -o h -- python3 bench.py --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/pl_${n}_h.log 2>&1 || exit 1
  PINOLOCO_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/pl_$n" -o c3 -- python3 bench.py --robot b2 --dynamics whole_body_aba --nodes 40 --batch 256 --steps 6 --warmup 1 --no-cpu-baseline > gpurun_out/pl_${n}_c3.log 2>&1 || exit 1
}
run intree "$R/pino-locoman_amd/pinoloco/libpinoloco.so"
for L in pino-locoman_amd/pinoloco/_ab/*.so; do run $(basename $L .so) "$(realpath $L)"; done
