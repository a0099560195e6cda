#!/bin/bash
set -o pipefail
for r in 1 2; do for wl in resnet50 vgg16_bn; do for f in inline auto; do
  timeout -k 10 200 python bench.py --workload $wl --no-cpu --steps 20 --warmup 5 --fill $f > gpurun_out/ab_${wl}_${f}_$r.json || exit $?
  python -c "import json,sys;d=json.load(open('gpurun_out/ab_${wl}_${f}_$r.json'));print('$wl','$f',round(d['ms_per_step'],4),d['phase_ms'])"
done; done; done
