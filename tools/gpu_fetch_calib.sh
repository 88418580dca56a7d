#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration of the load widths k_admm uses (tools/native/fetch_calib.hip)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" && mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/native/fetch_calib > gpurun_out/fetch_calib.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/pmc_calib" -o run -- ./tools/native/fetch_calib > gpurun_out/pmc_calib.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d "$R/gpurun_out/pmc_calib2" -o run -- ./tools/native/fetch_calib > gpurun_out/pmc_calib2.log 2>&1 || exit 1
cat gpurun_out/fetch_calib.log
