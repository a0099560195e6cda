#!/bin/bash
# K5 select timings (tools/k5_bench.py) with the default global phase vs one workgroup
set -o pipefail
for m in multi wg; do
  if [ $m = wg ]; then export DGC_K5_GLOBAL=wg; else unset DGC_K5_GLOBAL; fi
  timeout -k 10 120 python tools/k5_bench.py > gpurun_out/k5q_${m}.log 2>&1 || exit $?
  echo "== $m"; grep select_ms gpurun_out/k5q_${m}.log
done
