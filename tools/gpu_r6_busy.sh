#!/bin/bash
# Latency-hiding probe of the persistent forward (round 6): timing-only builds (tools/exp_build.py) that
# spin 0.5 / 1 / 2 us between an epoch's publish and its hand-off sweep.  If the forward's time stays
# flat, the hand-off wait is in-flight latency that other work could fill.  Interleaved A/B x2.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r6/busy}
mkdir -p $O
for rep in 1 2; do
  for v in base busy50 busy100 busy200; do
    if [ $v = base ]; then L=""; else L="red-diffeq_amd/lib_exp/lib$v.so"; fi
    RDQ_HIP_LIB=$L timeout -k 10 120 python -u tools/sweep_tb.py --only 4 --reps 6 > $O/$v.$rep.json 2> $O/$v.$rep.err \
        || { echo "$v rc=$?"; tail -5 $O/$v.$rep.err; exit 1; }
    echo "$v $rep $(tail -c 300 $O/$v.$rep.json)"
  done
done
