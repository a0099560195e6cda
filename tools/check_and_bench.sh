#!/bin/bash
# Parity subset, then the four bench lines: tools/check_and_bench.sh OUTDIR [pytest -k expr]
set -o pipefail
OUT=${1:-gpurun_out/cb}
K=${2:-}
mkdir -p "$OUT"
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest -q -x --timeout 600 --timeout-method thread -m gpu tests -k "$K" \
      > "$OUT/tests.log" 2>&1 || { tail -30 "$OUT/tests.log"; exit 1; }
  tail -3 "$OUT/tests.log"
fi
for wl in resnet50 vgg16_bn flat-1B flat-7B-bf16; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --workload $wl --no-cpu > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" || exit $?
done
python tools/bench_table.py "$OUT"/bench_*.json
