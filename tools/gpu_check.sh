#!/bin/bash
# One GPU session: parity tests, ablations, a rocprofv3 kernel-trace of the bench, the bench.
#   tools/gpu_check.sh TAG [bench args...]
# Outputs under gpurun_out/: pytest_gpu.log, ablate.json, prof_TAG/, bench.json
TAG=${1:-x}
shift
mkdir -p gpurun_out
rm -rf gpurun_out/prof_$TAG gpurun_out/bench.json gpurun_out/ablate.json
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python tools/ablate.py > gpurun_out/ablate.json 2> gpurun_out/ablate.err || exit $?
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$TAG" -o run \
    --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu "$@" \
    > gpurun_out/bench_prof.json 2> gpurun_out/bench_prof.err || exit $?
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu "$@" > gpurun_out/bench.json 2> gpurun_out/bench.err || exit $?
# HBM traffic counters, one counter per pass (FETCH_SIZE and WRITE_SIZE do not fit one pass on gfx950)
if [ "${DGC_PMC:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG" -o fetch --output-format csv \
      -- python bench.py --steps 3 --warmup 1 --no-cpu "$@" > /dev/null 2> gpurun_out/pmc_fetch.err || exit $?
  timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_$TAG" -o write --output-format csv \
      -- python bench.py --steps 3 --warmup 1 --no-cpu "$@" > /dev/null 2> gpurun_out/pmc_write.err || exit $?
fi
