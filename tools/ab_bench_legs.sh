#!/bin/bash
# Interleaved A/B of bench.py's loop legs (configs[1] step, configs[2] / notebook / B = 25 RED loops)
# between the in-tree library and another build of it (a tools/exp_build.py output), twice each.
# usage: tools/ab_bench_legs.sh <lib_exp/libX.so> <outdir>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
LIB=$1; O=${2:-gpurun_out/ab_legs}
mkdir -p $O
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-configs4 --no-cpu-baseline > $O/base_$i.json 2> $O/base_$i.err || exit $?
  RDQ_HIP_LIB=$LIB timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-configs4 --no-cpu-baseline > $O/exp_$i.json 2> $O/exp_$i.err || exit $?
done
