#!/bin/bash
# tools/gpu_check.sh for several workloads in one call (bench line, kernel trace +
# --stats, FETCH_SIZE and WRITE_SIZE passes each); summarise afterwards with
# tools/profile_summary.py into profiles/<round>/.
set -o pipefail
for wl in "$@"; do
  echo "== $wl $(date +%T)"
  bash tools/gpu_check.sh "$wl" 20 5 || exit $?
done
