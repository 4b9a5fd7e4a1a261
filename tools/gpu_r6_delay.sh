#!/bin/bash
# Pre-sweep delay sweep of the persistent kernels at configs[1] (rdq_fwi_set_sweep_delay; forward and adjoint
# delays in 10 ns ticks), interleaved, 3 repetitions.  Usage: tools/gpu_r6_delay.sh OUTDIR DELAYS...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r6/delay}
shift
mkdir -p $O
for rep in 1 2 3; do
  for d in "$@"; do
    timeout -k 10 120 python -u tools/sweep_tb.py --only 4 --reps 8 --delay $d > $O/$d.$rep.json 2> $O/$d.$rep.err \
        || { echo "$d rc=$?"; tail -5 $O/$d.$rep.err; exit 1; }
    echo "$d $rep $(tail -c 110 $O/$d.$rep.json)"
  done
done
