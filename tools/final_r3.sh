#!/bin/bash
# Round-3 closing evidence: the parity subset that the last library changes touch,
# then tools/gpu_check.sh (bench line, kernel trace + stats, FETCH / WRITE PMC) per workload.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests \
    -k "kth or resample or select_matches or batch or steady or half or model or dropin" > gpurun_out/final_tests.log 2>&1 \
    || { tail -20 gpurun_out/final_tests.log; exit 1; }
tail -1 gpurun_out/final_tests.log
bash tools/round_profiles.sh "$@"
