set -o pipefail
mkdir -p gpurun_out/p1
timeout -k 10 300 python tools/k5_prof.py > gpurun_out/p1/k5_prof.txt 2>&1 || exit $?
timeout -k 10 300 python tools/model_infos.py resnet50 8 all > gpurun_out/p1/infos_resnet50.txt 2>&1 || exit $?
timeout -k 10 300 python tools/model_infos.py vgg16_bn 8 all > gpurun_out/p1/infos_vgg16_bn.txt 2>&1 || exit $?
cat gpurun_out/p1/k5_prof.txt
