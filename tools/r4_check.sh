# targeted GPU tests, then the default bench (with extras): tools/r4_check.sh OUT [pytest -k expr]
set -o pipefail
OUT=${1:-gpurun_out/r4c}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread -m gpu tests/test_gpu_guards.py tests/test_gpu_dropin.py tests/test_gpu_multirank.py tests/test_gpu_batch.py ${2:+-k "$2"} > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
timeout -k 10 600 python bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
tail -c 1500 $OUT/bench.json
