set -o pipefail
mkdir -p gpurun_out/r4k5
timeout -k 10 300 python tools/k5_prof.py 2000 8200 18700 30000 72000 > gpurun_out/r4k5/phases.jsonl 2> gpurun_out/r4k5/phases.err || exit $?
cat gpurun_out/r4k5/phases.jsonl
