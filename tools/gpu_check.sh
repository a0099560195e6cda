#!/bin/bash
# Profile exactly one bench command on the GPU box: the bench itself, a rocprofv3
# kernel-trace + --stats run of the same command, and one --pmc pass per counter.
#   tools/gpu_check.sh WORKLOAD STEPS WARMUP [extra bench args...]
# Outputs under gpurun_out/: bench_WL.json, prof_WL/, pmc_WL/ (then tools/profile_summary.py).
set -o pipefail
WL=${1:-flat-1B}
STEPS=${2:-20}
WARM=${3:-5}
shift 3
mkdir -p gpurun_out
rm -rf "gpurun_out/prof_$WL" "gpurun_out/pmc_$WL"
export TMPDIR=/tmp
CMD="bench.py --gpus 1 --steps $STEPS --warmup $WARM --workload $WL $*"
timeout -k 10 400 python $CMD > "gpurun_out/bench_$WL.json" 2> "gpurun_out/bench_$WL.err" || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$WL" -o run \
    --output-format csv -- python $CMD --no-cpu > "gpurun_out/bench_prof_$WL.json" 2> "gpurun_out/prof_$WL.err" || exit $?
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$WL" -o fetch \
    --output-format csv -- python $CMD --no-cpu > /dev/null 2> "gpurun_out/pmc_fetch_$WL.err" || exit $?
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$WL" -o write \
    --output-format csv -- python $CMD --no-cpu > /dev/null 2> "gpurun_out/pmc_write_$WL.err" || exit $?
echo "done $WL"
