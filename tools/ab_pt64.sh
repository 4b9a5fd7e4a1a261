#!/bin/bash
# Persistent region classes by shot count (configs[1] geometry, nt 1000, T 4), interleaved, two rounds:
# 12 = 64 x 96 regions (the plan's rows per wave), 8 = 64 x 64 of 8 waves x 8 rows, 16 = 64 x 64 of
# 16 waves x 4 rows (tools/sweep_tb.py --mode).  profiles/r3/pt64_ab.txt was taken with an earlier
# build that selected 16 through an environment switch ("mode=8 pt64_rw=4" there = mode 16 here).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2; do
  for ns in 5 3 8; do
    for mode in 12 8 16; do
      echo -n "ns=$ns mode=$mode round $round: "
      timeout -k 10 120 python tools/sweep_tb.py --only 4 --reps 20 --ns $ns --mode $mode 2>/dev/null | tail -1 || exit $?
    done
  done
done
