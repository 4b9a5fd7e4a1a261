#!/bin/bash
# Round-2 evidence on one MI355X: bench line, rocprofv3 kernel stats of the same command, phase
# profile of the persistent kernels, PMC passes (traffic + VALU / wait counters).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r2
timeout -k 10 400 python -u bench.py --steps 10 --warmup 3 > gpurun_out/r2/bench.json 2> gpurun_out/r2/bench.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2/prof -o bench -- \
    python3 bench.py --steps 10 --warmup 3 --no-loop --no-red --no-cpu-baseline > gpurun_out/r2/prof_bench.json 2> gpurun_out/r2/prof.err || exit $?
timeout -k 10 300 python -u tools/sweep_tb.py --only 4 --profile > gpurun_out/r2/phase_profile.json 2> /dev/null || exit $?
ONLY=4 timeout -k 10 900 bash tools/gpu_pmc.sh > gpurun_out/r2/pmc.log 2>&1 || exit $?
echo done
