#!/bin/bash
# Round 6: the two-shots-per-workgroup persistent forward (k_fwd_p2): its bitwise test first, then
# multi-launch surveys with and without shot pairs, interleaved (configs[3]'s 32 shots, 16 shots),
# then the configs[1] reorder A/B builds.  Usage: tools/gpu_r6_pairs.sh OUTDIR
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r6/pairs}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread \
    "tests/test_gpu_plan_contract.py::test_forward_two_shots_per_workgroup_bitexact" > $O/pair_test.log 2>&1 \
    || { echo "pair test rc=$?"; tail -30 $O/pair_test.log; exit 1; }
tail -1 $O/pair_test.log
# (ns, region mode): configs[3]'s 32 shots and 16 shots in the default class; configs[1]'s 8 shots in the
# 64 x 64 class (two launches one shot per workgroup, one launch with pairs) and the default
for rep in 1 2; do
  for cfg in 32:1 16:1 8:16 8:1; do
    ns=${cfg%%:*}; md=${cfg##*:}
    for np in "" "--no-pairs"; do
      n=ns$ns.m$md$np
      timeout -k 10 120 python -u tools/sweep_tb.py --only 4 --reps 6 --ns $ns --mode $md $np > $O/$n.$rep.json 2> $O/$n.$rep.err \
          || { echo "$n rc=$?"; tail -5 $O/$n.$rep.err; exit 1; }
      echo "$n $rep $(tail -c 190 $O/$n.$rep.json)"
    done
  done
done
