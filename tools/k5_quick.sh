#!/bin/bash
# K5 parity tests (both global-phase forms) + the K5 phase timers by size
set -o pipefail
mkdir -p gpurun_out/k5
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests \
    -k "replays_torch_topk or partial_sort or k5 or steady" > gpurun_out/k5/tests_quick.log 2>&1 \
    || { tail -30 gpurun_out/k5/tests_quick.log; exit 1; }
tail -n 1 gpurun_out/k5/tests_quick.log
timeout -k 10 300 python tools/k5_prof.py > gpurun_out/k5/k5prof.txt 2>&1 || exit $?
