#!/bin/bash
# Decompress cost by world size (one MI355X, synthetic W-rank payloads): the tool's own
# timings plus a rocprofv3 kernel breakdown per W. Outputs under gpurun_out/dec/.
set -o pipefail
mkdir -p gpurun_out/dec
export TMPDIR=/tmp
for W in 1 2 4 8; do
  timeout -k 10 200 python tools/dec_bench.py --W $W --reps 10 > gpurun_out/dec/dec_W$W.json 2>/dev/null || exit $?
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/dec/prof_W$W" -o run \
      --output-format csv -- python tools/dec_bench.py --W $W --reps 10 > /dev/null 2>&1 || exit $?
done
cat gpurun_out/dec/dec_W*.json
