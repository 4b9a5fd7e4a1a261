#!/bin/bash
# Round 6: tuning probes of the barrier-free adjoint, interleaved x3 at configs[1] (tools/sweep_tb.py):
# base; agrad0 = the step's gradient at priority 0 (lib_exp build); adjoint pre-sweep delay 0 / 50 / 100 ticks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r6/adjtune}
mkdir -p $O
for rep in 1 2 3; do
  for v in base agrad0 d0 d50 d100; do
    L=""; D=""
    case $v in
      agrad0) L="red-diffeq_amd/lib_exp/lib$v.so";;
      d*) D="--delay 25,${v#d}";;
    esac
    RDQ_HIP_LIB=$L timeout -k 10 120 python -u tools/sweep_tb.py --only 4 --reps 8 $D > $O/$v.$rep.json 2> $O/$v.$rep.err \
        || { echo "$v rc=$?"; tail -5 $O/$v.$rep.err; exit 1; }
    echo "$v $rep $(tail -c 120 $O/$v.$rep.json)"
  done
done
