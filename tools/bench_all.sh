set -o pipefail
mkdir -p gpurun_out/r3a
for wl in flat-1B resnet50 vgg16_bn flat-7B-bf16; do
  echo "== $wl"; date
  timeout -k 10 400 python bench.py --steps 20 --warmup 5 --workload $wl > gpurun_out/r3a/bench_$wl.json 2> gpurun_out/r3a/bench_$wl.err || exit $?
  tail -c 600 gpurun_out/r3a/bench_$wl.json
done
