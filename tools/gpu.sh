#!/bin/bash
# Every GPU-box procedure of this repo in one script (run it through gpurun):
#
#   tools/gpu.sh tests OUT [pytest args...]    the -m gpu suite (or the files / -k given), -v log in OUT/tests.log
#   tools/gpu.sh bench OUT WL...               bench.py lines (20 steps, 5 warmup, no CPU baseline) + a table
#   tools/gpu.sh profile OUT WL...             per workload: the bench line, a rocprofv3 --kernel-trace --stats
#                                              run of the same command, one --pmc pass each for FETCH_SIZE and
#                                              WRITE_SIZE (summarise with tools/profile_summary.py)
#   tools/gpu.sh timeline OUT WL...            kernel-trace step timelines (tools/profile_summary.py)
#   tools/gpu.sh ab OUT WL...                  same-box A/B: this tree's library against lib/ab_old (built from an
#                                              older revision: make -C <old csrc> OUT_DIR=<repo>/adam-compression_amd/
#                                              lib/ab_old <that path>/libdgc_hip.so); REPS=n alternations (3)
#   tools/gpu.sh k5 OUT [size...]              K5 phase times by candidate count (needs `make -C ... k5prof`) and the
#                                              model sets' per-tensor replay stamps (tools/k5_prof.py,
#                                              tools/k5_models_prof.py)
#   tools/gpu.sh infos OUT WL...               per-tensor selection records of the model sets (tools/model_infos.py)
#   tools/gpu.sh dropin OUT [model]            drop-in DistributedOptimizer vs DGCBatch host / device time
#   tools/gpu.sh decompress OUT                decompress cost by world size (tools/dec_bench.py + kernel traces)
#
# Several can be chained with &&. Every GPU step runs under its own timeout; the script
# stops at the first failure (no retries).
set -o pipefail
export TMPDIR=/tmp
cmd=$1
OUT=${2:?usage: tools/gpu.sh CMD OUT ...}
shift 2
mkdir -p "$OUT"
case $cmd in
tests)
  timeout -k 10 1500 python -u -m pytest -v --timeout 1200 --timeout-method thread -m gpu "${@:-tests}" \
      > "$OUT/tests.log" 2>&1
  rc=$?
  tail -5 "$OUT/tests.log"
  exit $rc ;;
bench)
  for wl in "${@:-flat-1B}"; do
    timeout -k 10 600 python bench.py --steps 20 --warmup 5 --workload "$wl" --no-cpu ${BENCH_ARGS:-} \
        > "$OUT/bench_$wl.json" 2> "$OUT/bench_$wl.err" || { tail -20 "$OUT/bench_$wl.err"; exit 1; }
  done
  python tools/bench_table.py "$OUT"/bench_*.json ;;
profile)
  # SUFFIX names a variant's files (e.g. _alternating with BENCH_ARGS="--inputs alternating")
  for wl in "$@"; do
    CMD="bench.py --gpus 1 --steps 20 --warmup 5 --workload $wl --no-extras ${BENCH_ARGS:-}"
    W="$wl${SUFFIX:-}"
    timeout -k 10 600 python $CMD > "$OUT/bench_$W.json" 2> "$OUT/bench_$W.err" || exit 1
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_$W" -o run \
        --output-format csv -- python $CMD --no-cpu > "$OUT/bench_prof_$W.json" 2> "$OUT/prof_$W.err" || exit 1
    timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$GRAFT_REPO_ROOT/$OUT/pmc_$W" -o fetch \
        --output-format csv -- python $CMD --no-cpu > /dev/null 2> "$OUT/pmc_fetch_$W.err" || exit 1
    timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$GRAFT_REPO_ROOT/$OUT/pmc_$W" -o write \
        --output-format csv -- python $CMD --no-cpu > /dev/null 2> "$OUT/pmc_write_$W.err" || exit 1
    echo "profiled $W"
  done ;;
timeline)
  for wl in "$@"; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_$wl" -o run --output-format csv \
        -- python bench.py --steps 10 --warmup 3 --workload "$wl" --no-cpu --no-extras > "$OUT/bench_$wl.json" \
        2> "$OUT/prof_$wl.err" || exit 1
    python tools/profile_summary.py "$wl" "$OUT/prof_$wl" none "$OUT/sum" "$OUT/bench_$wl.json" > /dev/null || exit 1
    cat "$OUT/sum/step_timeline_$wl.txt"
  done ;;
ab)
  for wl in "$@"; do
    timeout -k 10 900 python tools/ab_bench.py "$wl" adam-compression_amd/lib/libdgc_hip.so \
        adam-compression_amd/lib/ab_old/libdgc_hip.so "${REPS:-3}" > "$OUT/ab_$wl.txt" 2>&1 \
        || { cat "$OUT/ab_$wl.txt"; exit 1; }
    cat "$OUT/ab_$wl.txt"
  done ;;
k5)
  timeout -k 10 300 python tools/k5_prof.py "$@" > "$OUT/k5_phases.jsonl" 2> "$OUT/k5_phases.err" || exit 1
  for wl in resnet50 vgg16_bn; do
    timeout -k 10 200 python tools/k5_models_prof.py "$wl" 12 > "$OUT/k5_$wl.jsonl" 2> "$OUT/k5_$wl.err" || exit 1
  done
  cat "$OUT/k5_phases.jsonl" ;;
infos)
  for wl in "${@:-resnet50}"; do
    timeout -k 10 200 python tools/model_infos.py "$wl" 14 all > "$OUT/infos_$wl.txt" 2>&1 || exit 1
  done ;;
dropin)
  timeout -k 10 300 python tools/dropin_prof.py "${1:-resnet50}" 20 > "$OUT/dropin.txt" 2>&1 || { cat "$OUT/dropin.txt"; exit 1; }
  cat "$OUT/dropin.txt" ;;
decompress)
  for W in 1 2 4 8; do
    timeout -k 10 200 python tools/dec_bench.py --W $W --reps 10 > "$OUT/dec_W$W.json" 2>/dev/null || exit 1
    timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$OUT/prof_W$W" -o run \
        --output-format csv -- python tools/dec_bench.py --W $W --reps 10 > /dev/null 2>&1 || exit 1
  done
  cat "$OUT"/dec_W*.json ;;
*)
  echo "unknown command $cmd" >&2
  exit 2 ;;
esac
