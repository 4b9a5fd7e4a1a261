#!/bin/bash
# A/B of library builds on the persistent FWI kernels (configs[1]: 8 shots, nt 1000, T = 4):
#   bash tools/ab_libs.sh lib/a.so lib/b.so ...   (paths relative to red-diffeq_amd/)
# each build timed twice, interleaved (tools/sweep_tb.py; RDQ_HIP_LIB selects the build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for round in 1 2; do
  for lib in "$@"; do
    echo -n "$lib round $round: "
    RDQ_HIP_LIB=$PWD/red-diffeq_amd/$lib timeout -k 10 120 python tools/sweep_tb.py --only 4 --reps 20 2>/dev/null | tail -1 || exit $?
  done
done
