#!/bin/bash
# K5 phase timers: by size (tools/k5_prof.py) and per tensor of the model sets
set -o pipefail
mkdir -p gpurun_out/k5
timeout -k 10 300 python tools/k5_prof.py > gpurun_out/k5/k5prof.txt 2>&1 || exit $?
for wl in resnet50 vgg16_bn; do
  timeout -k 10 300 python tools/k5_models_prof.py $wl 10 > gpurun_out/k5/k5mp_$wl.txt 2>&1 || exit $?
done
tail -n 2 gpurun_out/k5/k5mp_*.txt
