#!/bin/bash
# Same-box A/B of K5 timings (tools/k5_bench.py select_ms, min of 3) and the model-set
# bench steps: this tree's library vs adam-compression_amd/lib/ab_old (a previous
# revision: make -C <old csrc> OUT_DIR=<repo>/adam-compression_amd/lib/ab_old).
set -o pipefail
mkdir -p gpurun_out/k5ab
export TMPDIR=/tmp
for r in 1 2; do
  for lib in adam-compression_amd/lib/libdgc_hip.so adam-compression_amd/lib/ab_old/libdgc_hip.so; do
    DGC_HIP_LIB=$PWD/$lib DGC_LIB_PARTIAL=1 K5_MODELS=0 timeout -k 10 200 python tools/k5_bench.py > gpurun_out/k5ab/k5_${r}_$(basename $(dirname $lib)).txt 2>&1 || exit 1
  done
done
for wl in ${K5AB_WL:-resnet50 vgg16_bn}; do
  timeout -k 10 600 python tools/ab_bench.py $wl adam-compression_amd/lib/libdgc_hip.so adam-compression_amd/lib/ab_old/libdgc_hip.so 2 > gpurun_out/k5ab/ab_$wl.txt 2>&1 || exit 1
done
