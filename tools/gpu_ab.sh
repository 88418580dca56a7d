#!/bin/bash
# A/B of two builds of the library on ONE box (box-to-box k_admm differs by up to ~10 %):
# alternating headline bench runs with ab/lib_old.so and ab/lib_new.so.
set -o pipefail
O=gpurun_out/ab
mkdir -p $O
: > $O/ab.jsonl
for r in 1 2; do
  for v in old new; do
    PINOLOCO_LIB=$PWD/ab/lib_$v.so timeout -k 10 300 python bench.py --steps 10 --warmup 2 --host-io-steps 0 --no-cpu-baseline "$@" > $O/b.log 2>&1 || { tail -5 $O/b.log; exit 1; }
    python -c "import json,sys; d=json.loads(open('$O/b.log').read().strip().splitlines()[-1]); print(json.dumps({'lib': '$v', 'value': d['value'], 'ms': d['ms_per_step'], 'admm_ms': d['roofline']['avg_launch_ms'], 'frac': d['roofline']['frac']}))" >> $O/ab.jsonl
  done
done
cat $O/ab.jsonl
