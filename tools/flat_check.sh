#!/bin/bash
# Flat-bucket parity (1B bucket vs the oracle, bucket tests), then the flat-1B timeline
set -o pipefail
mkdir -p "${1:-gpurun_out/fc}"
timeout -k 10 900 python -u -m pytest -q -x --timeout 600 --timeout-method thread -m gpu tests \
    -k "fullsize or bucket or compress" > "${1:-gpurun_out/fc}/tests.log" 2>&1 \
    || { tail -30 "${1:-gpurun_out/fc}/tests.log"; exit 1; }
tail -n 1 "${1:-gpurun_out/fc}/tests.log"
bash tools/timeline.sh "${1:-gpurun_out/fc}" flat-1B
