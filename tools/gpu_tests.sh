#!/bin/bash
# The -m gpu suite on the box, new/targeted tests first: tools/gpu_tests.sh [pytest args...]
# Log: gpurun_out/gpu_tests.log (one line per test, -v), summary at the end.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest -v --timeout 1200 --timeout-method thread -m gpu "$@" \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?
tail -40 gpurun_out/gpu_tests.log
exit $rc
