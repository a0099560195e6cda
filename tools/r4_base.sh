set -o pipefail
mkdir -p gpurun_out/r4base
for wl in resnet50 vgg16_bn flat-1B; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --workload $wl --no-cpu > gpurun_out/r4base/bench_$wl.json 2> gpurun_out/r4base/bench_$wl.err || exit $?
  tail -c 300 gpurun_out/r4base/bench_$wl.json
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --workload flat-1B --no-cpu --fill inline > gpurun_out/r4base/bench_flat-1B_inline.json 2> gpurun_out/r4base/inline.err || exit $?
bash tools/timeline.sh gpurun_out/r4base/tl resnet50 vgg16_bn
