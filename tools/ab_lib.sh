#!/bin/bash
# Same-box A/B of this tree's library against adam-compression_amd/lib/ab_old (built
# from the previous revision: make -C adam-compression_amd/csrc OUT_DIR=../lib/ab_old)
#   tools/ab_lib.sh WORKLOAD [reps]
set -o pipefail
timeout -k 10 600 python tools/ab_bench.py "$1" adam-compression_amd/lib/libdgc_hip.so adam-compression_amd/lib/ab_old/libdgc_hip.so "${2:-2}"
