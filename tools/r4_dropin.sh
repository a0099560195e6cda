set -o pipefail
OUT=gpurun_out/r4d
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/dropin_prof.py resnet50 20 > $OUT/host.txt 2>&1 || { cat $OUT/host.txt; exit 1; }
cat $OUT/host.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $GRAFT_REPO_ROOT/$OUT/prof -o run -- python tools/dropin_prof.py resnet50 10 > $OUT/prof.txt 2>&1 || exit 1
