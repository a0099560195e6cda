set -o pipefail
mkdir -p gpurun_out/p3
export TMPDIR=/tmp
timeout -k 10 120 ./tools/rsbench > gpurun_out/p3/rsbench.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "resample or kth_largest or select_matches" > gpurun_out/p3/tests.log 2>&1 || { tail -30 gpurun_out/p3/tests.log; exit 1; }
tail -2 gpurun_out/p3/tests.log
timeout -k 10 200 python tools/k5_prof.py > gpurun_out/p3/k5_prof.txt 2>&1 || exit 1
timeout -k 10 200 python tools/k5_models_prof.py resnet50 10 > gpurun_out/p3/k5m_resnet50.txt 2>&1 || exit 1
