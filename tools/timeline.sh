#!/bin/bash
# Kernel-trace timelines of bench workloads: tools/timeline.sh OUTDIR WL...
set -o pipefail
OUT=$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
for wl in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_$wl" -o run --output-format csv \
      -- python bench.py --steps 10 --warmup 3 --workload $wl --no-cpu > "$OUT/bench_$wl.json" 2> "$OUT/prof_$wl.err" || exit $?
  python tools/profile_summary.py $wl "$OUT/prof_$wl" none "$OUT/sum" "$OUT/bench_$wl.json" > /dev/null || exit $?
done
