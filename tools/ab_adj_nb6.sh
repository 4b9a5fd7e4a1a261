#!/bin/bash
# Adjoint: 12 waves x 8 rows with a workgroup barrier per step (default build) vs the barrier-free
# exchange (RDQ_PT_NB_ADJ=1 build) at 8 and 6 rows per wave; configs[1], interleaved, three rounds
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
L=$PWD/red-diffeq_amd/lib
for round in 1 2 3; do
  for cfg in "head 6,8" "head 6,6" "nbadj 6,8" "nbadj 6,6"; do
    set -- $cfg
    echo -n "$1 rw $2 round $round: "
    RDQ_HIP_LIB=$L/libred_diffeq_hip_$1.so timeout -k 10 120 python tools/sweep_tb.py --only 4 --reps 20 --rw $2 2>/dev/null | tail -1 || exit $?
  done
done
