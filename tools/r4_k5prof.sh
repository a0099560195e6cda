set -o pipefail
mkdir -p gpurun_out/r4k5
timeout -k 10 200 python tools/k5_models_prof.py resnet50 12 > gpurun_out/r4k5/resnet50.jsonl 2> gpurun_out/r4k5/resnet50.err || exit $?
timeout -k 10 200 python tools/k5_models_prof.py vgg16_bn 12 > gpurun_out/r4k5/vgg16_bn.jsonl 2> gpurun_out/r4k5/vgg16_bn.err || exit $?
timeout -k 10 200 python tools/model_infos.py resnet50 12 all > gpurun_out/r4k5/infos_resnet50.txt 2>&1 || exit $?
