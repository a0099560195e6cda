#!/bin/bash
# K5 A/B: tools/k5_bench-style select timings with the multi-workgroup global phase vs one workgroup
set -o pipefail
for r in 1 2; do for m in multi wg; do
  if [ $m = wg ]; then export DGC_K5_GLOBAL=wg; else unset DGC_K5_GLOBAL; fi
  timeout -k 10 120 python tools/k5_bench.py > gpurun_out/k5_${m}_$r.log 2>&1 || exit $?
  echo "== $m $r"; grep -v amdgpu.ids gpurun_out/k5_${m}_$r.log
done; done
for r in 1 2; do for wl in resnet50 vgg16_bn; do for m in multi wg; do
  if [ $m = wg ]; then export DGC_K5_GLOBAL=wg; else unset DGC_K5_GLOBAL; fi
  timeout -k 10 200 python bench.py --workload $wl --no-cpu --steps 20 --warmup 5 > gpurun_out/k5ab_${wl}_${m}_$r.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/k5ab_${wl}_${m}_$r.json'));print('$wl','$m',round(d['ms_per_step'],4))"
done; done; done
for m in multi wg; do
  if [ $m = wg ]; then export DGC_K5_GLOBAL=wg; else unset DGC_K5_GLOBAL; fi
  timeout -k 10 200 python bench.py --workload flat-1B --no-cpu --steps 20 --warmup 5 > gpurun_out/k5ab_flat_${m}.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/k5ab_flat_${m}.json'));print('flat-1B','$m',round(d['ms_per_step'],4))"
done
