#!/bin/bash
# Same-box A/B of two library builds by rocprofv3 kernel stats (ab/lib_old.so, ab/lib_new.so):
# python tools/ab_stats.py then compares the per-kernel averages.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/abp
mkdir -p $O
for r in 1 2; do
  for v in old new; do
    PINOLOCO_LIB=$PWD/ab/lib_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/${v}_$r" -o run -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline --host-io-steps 0 "$@" > $O/${v}_$r.log 2>&1 || { tail -5 $O/${v}_$r.log; exit 1; }
  done
done
echo done
