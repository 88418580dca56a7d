#!/bin/bash
# k_fchain phase timing on configs 1, 3 and the headline (s_memtime, cycles per node)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
T=${1:-r04f}
O=gpurun_out/$T
cd "$R" && mkdir -p "$O"
for a in "go2 centroidal_vel 20 1024" "b2 whole_body_aba 40 256" "b2g whole_body_rnea 50 1024" "go2 whole_body_rnea 20 1"; do
  n=$(echo $a | tr ' ' '_')
  timeout -k 10 200 python tools/gpu_fchain_timing.py $a > $O/fchain_$n.txt 2>&1 || { tail -5 $O/fchain_$n.txt; exit 1; }
  cat $O/fchain_$n.txt
done
