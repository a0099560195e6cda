#!/bin/bash
# K5 checks: the resample parity tests (both global-phase forms), the model-set
# steady-state tests, the bench lines of the model sets, and K5 timings by size.
set -o pipefail
mkdir -p gpurun_out/k5
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q -x --timeout 600 --timeout-method thread -m gpu tests \
    -k "replays_torch_topk or partial_sort or batch_matches or steady or k5 or decompress" > gpurun_out/k5/tests.log 2>&1 \
    || { tail -30 gpurun_out/k5/tests.log; exit 1; }
tail -2 gpurun_out/k5/tests.log
for wl in resnet50 vgg16_bn; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --workload $wl --no-cpu > gpurun_out/k5/bench_$wl.json 2>/dev/null || exit $?
done
python tools/bench_table.py gpurun_out/k5/bench_*.json
for mode in wg default multi; do
  if [ $mode = default ]; then unset DGC_K5_GLOBAL; else export DGC_K5_GLOBAL=$mode; fi
  K5_MODELS=0 timeout -k 10 300 python tools/k5_bench.py > gpurun_out/k5/k5bench_$mode.txt 2>&1 || exit $?
done
unset DGC_K5_GLOBAL
tail -n 12 gpurun_out/k5/k5bench_*.txt
