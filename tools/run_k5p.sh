#!/bin/bash
# run_k5.sh (K5 parity, model benches, K5 timings by mode), then the K5 phase timers
set -o pipefail
bash tools/run_k5.sh || exit $?
bash tools/run_k5mp.sh || exit $?
