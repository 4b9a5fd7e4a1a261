#!/bin/bash
# rows per wave of the persistent 96-row kernels (configs[1]: 8 shots, nt 1000, T = 4), interleaved
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2; do
  for rw in "$@"; do
    timeout -k 10 120 python tools/sweep_tb.py --only 4 --reps 20 --rw $rw 2>/dev/null | tail -1 || exit $?
  done
done
