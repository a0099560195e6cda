#!/bin/bash
# K5 / selection parity tests, then the model sets' kernel timelines
set -o pipefail
mkdir -p gpurun_out/k5
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread -m gpu tests \
    -k "replays_torch_topk or partial_sort or k5 or steady or batch_matches or select_matches" > gpurun_out/k5/tests_tl.log 2>&1 \
    || { tail -30 gpurun_out/k5/tests_tl.log; exit 1; }
tail -n 1 gpurun_out/k5/tests_tl.log
bash tools/timeline.sh "${1:-gpurun_out/tl6}" resnet50 vgg16_bn
