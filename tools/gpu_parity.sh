#!/bin/bash
# per-fixture, per-ADMM-kernel step errors against the goldens (tools/parity_report.py)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u tools/parity_report.py > gpurun_out/parity_report.log 2>&1
