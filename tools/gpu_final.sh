#!/bin/bash
# Round evidence under the final sources: the round check (tests, smoke, parity report,
# bench, rocprofv3 kernel stats, PMC traffic), then one bench line per BASELINE config.
set -o pipefail
bash tools/gpu_round.sh "${1:-final}" || exit 1
bash tools/gpu_configs.sh || exit 1
