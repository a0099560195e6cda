#!/bin/bash
# rsbench (warm and flushed) and the K5 phase profile (profiling build)
set -o pipefail
mkdir -p gpurun_out/p4
export TMPDIR=/tmp
timeout -k 10 120 ./tools/rsbench > gpurun_out/p4/rsbench_warm.txt 2>&1 || exit 1
RS_FLUSH=1 timeout -k 10 120 ./tools/rsbench > gpurun_out/p4/rsbench_flush.txt 2>&1 || exit 1
timeout -k 10 200 python tools/k5_prof.py > gpurun_out/p4/k5_prof.txt 2>&1 || exit 1
