#!/bin/bash
# Pre-sweep spin probe of the persistent kernels (round 6): timing-only builds (tools/exp_build.py) that wait
# N x 10 ns between an epoch's publish (forward: f<N>; adjoint, after its deferred gradient: a<N>) and the
# first hand-off sweep pass.  Interleaved A/B, 3 repetitions.  Usage: tools/gpu_r6_spin.sh OUTDIR VARIANTS...
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=${1:-gpurun_out/r6/spin}
shift
mkdir -p $O
for rep in 1 2 3; do
  for v in base "$@"; do
    if [ $v = base ]; then L=""; else L="red-diffeq_amd/lib_exp/lib$v.so"; fi
    RDQ_HIP_LIB=$L timeout -k 10 120 python -u tools/sweep_tb.py --only 4 --reps 8 > $O/$v.$rep.json 2> $O/$v.$rep.err \
        || { echo "$v rc=$?"; tail -5 $O/$v.$rep.err; exit 1; }
    echo "$v $rep $(tail -c 120 $O/$v.$rep.json)"
  done
done
