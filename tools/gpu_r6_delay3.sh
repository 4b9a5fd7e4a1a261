#!/bin/bash
# Round 6: pre-sweep delays re-checked on the final kernels (flag-word / mailbox exchange, adjoint trims),
# interleaved x3 at configs[1] (tools/sweep_tb.py --delay fwd,adj ticks of 10 ns; base = the defaults 15,0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r6/delay3}
mkdir -p $O
for rep in 1 2 3; do
  for v in base 0,0 8,0 25,0 15,8 15,15; do
    D=""; [ $v = base ] || D="--delay $v"
    timeout -k 10 120 python -u tools/sweep_tb.py --only 4 --reps 8 $D > $O/$v.$rep.json 2> $O/$v.$rep.err \
        || { echo "$v rc=$?"; tail -5 $O/$v.$rep.err; exit 1; }
    echo "$v $rep $(tail -c 100 $O/$v.$rep.json)"
  done
done
