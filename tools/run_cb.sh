set -o pipefail
bash tools/check_and_bench.sh gpurun_out/cb4 "parity or batch or steady or fullsize or multirank" || exit $?
timeout -k 10 300 python tools/k5_prof.py > gpurun_out/cb4/k5prof.txt 2>&1 || exit $?
bash tools/timeline.sh gpurun_out/tl4 resnet50 vgg16_bn
