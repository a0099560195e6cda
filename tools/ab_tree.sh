#!/bin/bash
# Same-box A/B of this tree against the whole tree in .ab_head (git worktree add .ab_head HEAD,
# plus its built library), for changes above the library.  tools/ab_tree.sh WORKLOAD [reps]
set -o pipefail
timeout -k 10 600 python tools/ab_bench.py "$1" . .ab_head "${2:-2}"
