#!/bin/bash
# kernel resource usage (VGPRs, scratch) of one .hip file: tools/kres.sh file.hip
cd "$(dirname "$0")/../adam-compression_amd/csrc" || exit 1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -I../../include \
  -munsafe-fp-atomics -c "$1" -o /tmp/kres_$$.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk '/Function Name:/{n=$5} /VGPRs:/{v=$4} /ScratchSize/{print n, "vgpr=" v, "scratch=" $5}' | sort
rm -f /tmp/kres_$$.o
